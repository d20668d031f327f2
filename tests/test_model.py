"""Model-level behaviour: causality, masks, tokenizers, inference equivalence."""
import numpy as np
import pytest
import torch

import pytorch_rt1_for_distributed_training_amd as rt1
from pytorch_rt1_for_distributed_training_amd import spaces
from pytorch_rt1_for_distributed_training_amd.models import action_space, build_rt1
from pytorch_rt1_for_distributed_training_amd.models.action_tokenizer import RT1ActionTokenizer
from pytorch_rt1_for_distributed_training_amd.models.efficientnet import block_specs, feature_map_size
from pytorch_rt1_for_distributed_training_amd.models.transformer import rt1_attention_mask


def tiny(**kw):
    return build_rt1(rt1.preset("tiny").replace(**kw))


def test_param_count_full_model():
    m = build_rt1(rt1.RT1Config())
    assert sum(p.numel() for p in m.parameters()) == 35_324_320
    assert sum(p.numel() for p in m.parameters() if p.requires_grad) == 35_324_320 - 131_584
    assert len(m.state_dict()) == 806


def test_block_table_and_feature_sizes():
    specs = block_specs()
    assert len(specs) == 26
    assert [s.out_ch for s in specs][-1] == 384
    assert [s.index for s in specs if s.stride == 2] == [2, 5, 8, 18]
    assert feature_map_size(256, 456) == (8, 15)
    assert feature_map_size(300, 300) == (10, 10)
    assert abs(specs[25].drop_rate - 0.2 * 25 / 26) < 1e-12


def _reference_mask(T, K, A):
    """Direct transcription of the reference's double loop semantics."""
    L = K + A
    S = T * L

    def act_idx(k):
        return -1 if k % L < K else k // L
    m = np.tril(np.ones((S, S), dtype=np.int64))
    for i in range(S):
        for j in range(S):
            ai, aj = act_idx(i), act_idx(j)
            if ai != -1 and aj != -1 and (aj < ai or (aj == ai and j <= i)):
                m[i, j] -= 1
    return m


@pytest.mark.parametrize("T,K,A", [(6, 8, 3), (2, 8, 3), (15, 8, 3), (3, 4, 2)])
def test_attention_mask_matches_reference_construction(T, K, A):
    assert np.array_equal(rt1_attention_mask(T, K, A).numpy(), _reference_mask(T, K, A))


def test_causality_future_frames_do_not_change_past_predictions():
    """Reference transformer_network_test.py:99-157: zeroing future inputs keeps past outputs."""
    torch.manual_seed(0)
    m = tiny(seq_len=3).eval()
    x = torch.rand(1, 3, 3, 64, 64)
    emb = torch.randn(1, 3, 512)
    tokens = m.tokenize_images(x, emb, shift=(0, 0))
    full = m.transformer_hidden(m.assemble_tokens(tokens))
    cut = tokens.clone()
    cut[:, 2] = 0
    part = m.transformer_hidden(m.assemble_tokens(cut))
    L = m.tokens_per_step
    torch.testing.assert_close(full[:, :2 * L], part[:, :2 * L], rtol=0, atol=0)


def test_action_tokenizer_roundtrip_and_oov():
    sp = spaces.Dict({"terminate": spaces.Discrete(2), "world": spaces.Box(-1.0, 1.0, (3,), np.float32)})
    from collections import OrderedDict
    sp = spaces.Dict(OrderedDict([("terminate", spaces.Discrete(2)), ("world", spaces.Box(-1.0, 1.0, (3,), np.float32))]))
    tok = RT1ActionTokenizer(sp, vocab_size=1024)
    assert tok.tokens_per_action == 4
    for _ in range(10):
        a = {"terminate": torch.randint(0, 2, (2,)), "world": torch.rand(2, 3) * 2 - 1}
        t = tok.tokenize(a)
        d = tok.detokenize(t)
        assert torch.equal(d["terminate"], a["terminate"])
        assert torch.allclose(d["world"], a["world"], atol=2.0 / 1023 + 1e-6)
    # truncation, clamping
    t = tok.tokenize({"terminate": torch.tensor([1]), "world": torch.tensor([[2.0, -2.0, 0.0]])})
    assert t.tolist() == [[1, 1023, 0, 511]]
    # OOV discrete: the reference resets only tokens > n (token == n passes through)
    d = tok.detokenize(torch.tensor([[3, 0, 0, 0], [2, 0, 0, 0]]))
    assert d["terminate"].tolist() == [0, 2]


def test_rt1_action_space_tokens():
    tok = RT1ActionTokenizer(action_space(rt1.RT1Config()), 256)
    t = tok.tokenize({"terminate_episode": torch.tensor([[0, 1]]), "action": torch.tensor([[[0.1, -0.1], [0.0, 0.05]]])})
    assert t.tolist() == [[[0, 255, 0], [1, 127, 191]]]


def test_single_pass_inference_equals_three_pass_reference_loop():
    """The reference runs the transformer once per action token (transformer_network.py:246-268);
    since inserted action tokens are zeroed before the transformer, one pass is identical."""
    torch.manual_seed(0)
    m = tiny(seq_len=3).eval()
    state = m.initial_state(1)
    img = torch.rand(1, 3, 64, 64)
    emb = torch.randn(1, 512)
    for step in range(5):
        torch.manual_seed(100 + step)
        out, new_state = m({"image": img, "natural_language_embedding": emb}, dict(state))
        logits_single = m.get_aux_info()["action_predictions_logits"]
        # three-pass reference loop over the same state
        torch.manual_seed(100 + step)
        toks = m.tokenize_images(img[:, None], emb[:, None])
        seq = int(state["seq_idx"][0])
        T, L, K = 3, m.tokens_per_step, 8
        ts = min(seq, T - 1)
        st = torch.roll(state["context_image_tokens"], -1, 1) if seq == T else state["context_image_tokens"]
        st = torch.cat([st[:, :ts], toks, st[:, ts + 1:]], 1)
        logits3 = []
        for k in range(3):
            h = m.transformer_hidden(m.assemble_tokens(st))
            logits3.append(m._transformer._output_tokens(h[:, K - 1 + ts * L + k]))
        torch.testing.assert_close(logits_single[0], torch.stack(logits3, 1)[0], rtol=1e-5, atol=1e-5)
        assert int(new_state["seq_idx"][0]) == min(seq + 1, T)
        assert out["action"].shape == (1, 2)
        state = new_state


def test_film_zero_init_is_identity():
    from pytorch_rt1_for_distributed_training_amd.models.efficientnet import FiLMEfficientNet
    torch.manual_seed(0)
    with_film = FiLMEfficientNet(include_film=True).eval()
    no_film = FiLMEfficientNet(include_film=False).eval()
    sd = {k: v for k, v in with_film.state_dict().items() if not k.startswith("films.")}
    no_film.load_state_dict(sd)
    x = torch.rand(2, 3, 64, 64)
    torch.testing.assert_close(with_film(x, torch.randn(2, 512)), no_film(x), rtol=0, atol=0)


def test_train_forward_shapes_and_loss_scaling():
    torch.manual_seed(0)
    m = tiny()
    b, t = 2, 2
    acts = {"terminate_episode": torch.zeros(b, t, dtype=torch.long), "action": torch.zeros(b, t, 2)}
    loss, aux = m.train_forward(torch.rand(b, t, 3, 64, 64), torch.randn(b, t, 512), acts)
    assert loss.shape == (b, t)
    assert aux["action_predictions"].shape == (b, t, 3)
    # loss = mean CE / (b * t * 11)
    ce_mean = float(loss.mean()) * (b * t * 11)
    assert 1.0 < ce_mean < 20.0
