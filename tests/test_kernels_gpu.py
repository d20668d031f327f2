"""HIP kernel numerics vs plain PyTorch fp32 references (MI355X only)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ext():
    from pytorch_rt1_for_distributed_training_amd import ops
    return ops.load()


def test_flat_adam_matches_reference(ext):
    from pytorch_rt1_for_distributed_training_amd.ops.adam import flat_adam_step, reference_adam_step
    torch.manual_seed(0)
    n = 1_000_003 + 1  # not a multiple of 4 -> exercises the scalar tail
    p = torch.randn(n, device="cuda")
    g = torch.randn(n, device="cuda")
    m = torch.randn(n, device="cuda") * 0.1
    v = torch.rand(n, device="cuda") * 0.1
    ref = [t.clone() for t in (p, g, m, v)]
    for step in (1, 2, 7):
        kw = dict(lr=5e-4, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.01 if step == 7 else 0.0, step=step,
                  grad_scale=0.25)
        flat_adam_step(p, g, m, v, **kw)
        reference_adam_step(ref[0], ref[1], ref[2], ref[3], **kw)
    torch.testing.assert_close(p, ref[0], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(m, ref[2], rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(v, ref[3], rtol=1e-5, atol=1e-8)


def test_engine_step_hip_backend_small(ext):
    from pytorch_rt1_for_distributed_training_amd.config import RT1Config
    from pytorch_rt1_for_distributed_training_amd.data.synthetic import make_batch
    from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine
    from pytorch_rt1_for_distributed_training_amd.models import build_rt1
    torch.manual_seed(0)
    cfg = RT1Config(height=96, width=96, seq_len=2, backend="hip")
    eng = TrainEngine(build_rt1(cfg), cfg, order_probe=False)
    assert eng.backend == "hip"
    batch = make_batch(2, 2, 96, 96, device="cuda")
    losses = [float(eng.train_step(batch)) for _ in range(3)]
    assert all(math.isfinite(x) for x in losses), losses


@pytest.mark.parametrize("T", [6, 2, 8, 15])
def test_rt1_attention_matches_eager(ext, T):
    from pytorch_rt1_for_distributed_training_amd.models.transformer import masked_attention, rt1_attention_mask
    from pytorch_rt1_for_distributed_training_amd.ops.attention import RT1AttentionFn
    torch.manual_seed(0)
    B, H, D, L, K = 3, 8, 128, 11, 8
    S = T * L
    qkv = torch.randn(B, S, 3, H, D, device="cuda").to(torch.bfloat16).requires_grad_(True)
    out = RT1AttentionFn.apply(qkv, L, K, 0.0, 0)
    q, k, v = qkv.detach().float().permute(2, 0, 3, 1, 4).unbind(0)
    q, k, v = (t.clone().requires_grad_(True) for t in (q, k, v))
    mask = rt1_attention_mask(T, K, L - K).cuda()
    ref, _ = masked_attention(q, k, v, mask, 0.0, False)
    ref = ref.permute(0, 2, 1, 3)
    err = float((out.float() - ref).norm() / ref.norm())
    assert err < 1e-2, err
    g = torch.randn_like(ref)
    out.backward(g.to(torch.bfloat16))
    ref.backward(g)
    dref = torch.stack([q.grad, k.grad, v.grad], 0).permute(1, 3, 0, 2, 4)
    derr = float((qkv.grad.float() - dref).norm() / dref.norm())
    assert derr < 2e-2, derr


def test_rt1_attention_dropout_mask_consistent(ext):
    """Forward dropout (in-kernel hash) == explicit keep-mask applied to the eager softmax."""
    from pytorch_rt1_for_distributed_training_amd.models.transformer import rt1_attention_mask
    from pytorch_rt1_for_distributed_training_amd.ops.attention import RT1AttentionFn
    torch.manual_seed(1)
    B, H, D, L, K, T = 2, 8, 128, 11, 8, 6
    S = T * L
    qkv = torch.randn(B, S, 3, H, D, device="cuda").to(torch.bfloat16)
    out = RT1AttentionFn.apply(qkv, L, K, 0.1, 1234)
    q, k, v = qkv.float().permute(2, 0, 3, 1, 4).unbind(0)
    mask = rt1_attention_mask(T, K, L - K).cuda()
    s = (q @ k.transpose(-1, -2) / D ** 0.5).masked_fill(mask == 0, float("-inf"))
    from pytorch_rt1_for_distributed_training_amd.ops import rng
    keep = ext.attn_keepmask(B * H, S, 0.1, 1234, qkv, rng.counter(qkv.device)).view(B, H, S, S).float()
    assert 0.85 < float(keep.mean()) < 0.95
    ref = (torch.softmax(s, -1) * keep / 0.9) @ v
    err = float((out.float() - ref.permute(0, 2, 1, 3)).norm() / ref.norm())
    assert err < 1e-2, err


def test_rt1_attention_backward_kernel_with_dropout(ext):
    """HIP attention backward (dropout mask regenerated in-kernel) == the fp32 torch backward with the
    explicit keep-mask of the same hash."""
    from pytorch_rt1_for_distributed_training_amd.ops.attention import RT1AttentionFn
    torch.manual_seed(2)
    B, H, D, L, K, T = 3, 8, 128, 11, 8, 6
    S = T * L
    qkv = torch.randn(B, S, 3, H, D, device="cuda").to(torch.bfloat16)
    from pytorch_rt1_for_distributed_training_amd.ops import rng
    ctr = rng.counter(qkv.device)
    out, lse = ext.attn_fwd(qkv, L, K, D ** -0.5, 0.1, 77, ctr)
    dout = torch.randn(B, S, H, D, device="cuda").to(torch.bfloat16)
    dq = ext.attn_bwd(qkv, out, dout, lse, L, K, D ** -0.5, 0.1, 77, ctr)
    dref, *_ = RT1AttentionFn._backward_torch(qkv, out, lse, dout, L, K, 0.1, 77, D ** -0.5)
    err = float((dq.float() - dref.float()).norm() / dref.float().norm())
    assert err < 1e-2, err


def test_native_rccl_communicator_single_rank():
    """csrc/comm.cpp: RCCL communicator on its own stream (world = 1 on the one-GPU box)."""
    from pytorch_rt1_for_distributed_training_amd.parallel.native_comm import NativeComm
    c = NativeComm.single(0)
    t = torch.arange(1000, device="cuda", dtype=torch.float32)
    ref = t.clone()
    w = c.all_reduce_(t)
    w.wait()
    torch.cuda.synchronize()
    assert torch.equal(t, ref)
    b = torch.randn(77, device="cuda").to(torch.bfloat16)
    b0 = b.clone()
    c.broadcast_(b, 0)
    parts = [torch.ones(10, device="cuda"), torch.full((3,), 2.0, device="cuda")]
    c.all_reduce_coalesced_(parts).wait()
    torch.cuda.synchronize()
    assert torch.equal(b, b0) and float(parts[1][0]) == 2.0
    c.destroy()


def test_native_comm_watchdog_aborts_a_stuck_collective():
    """The watchdog of csrc/comm.cpp: a collective pending past the timeout aborts the communicator (here with the
    process exit disabled, and a never-completing debug entry instead of a real hang)."""
    import time
    from pytorch_rt1_for_distributed_training_amd.parallel.native_comm import NativeComm
    c = NativeComm.single(0, timeout_s=0.5)
    c._c.set_exit_on_timeout(False)
    t = torch.ones(4096, device="cuda")
    c.all_reduce_(t).wait()
    torch.cuda.synchronize()
    time.sleep(1.0)                              # completed collectives never trip it
    assert not c.timed_out
    c._c.debug_add_stuck_entry("test: stuck all_reduce")
    deadline = time.time() + 10
    while not c.timed_out and time.time() < deadline:
        time.sleep(0.05)
    assert c.timed_out
    with pytest.raises(RuntimeError, match="aborted"):
        c.all_reduce_(t)
    c.destroy()


def test_fused_transformer_layer_matches_eager(ext):
    """RT1LayerFn (LN / residual / dropout / attention HIP kernels + bf16 GEMMs) vs the fp32 eager layer."""
    from pytorch_rt1_for_distributed_training_amd.models.transformer import _TransformerLayer, rt1_attention_mask
    from pytorch_rt1_for_distributed_training_amd.ops.attention import fused_layer
    torch.manual_seed(0)
    layer = _TransformerLayer(128, 8, 512, 0.1).cuda().eval()
    with torch.no_grad():
        for m in (layer.norm_1, layer.norm_2):
            m.weight.uniform_(0.5, 1.5)
            m.bias.normal_(0, 0.1)
    B, T, L, K = 4, 6, 11, 8
    S = T * L
    x = torch.randn(B, S, 512, device="cuda")
    mask = rt1_attention_mask(T, K, L - K).cuda()
    xr = x.clone().requires_grad_(True)
    ref, _ = layer(xr, mask)
    xf = x.clone().requires_grad_(True)
    out, _ = fused_layer(layer, xf, L, K, False)
    assert float((out - ref).norm() / ref.norm()) < 1e-2
    g = torch.randn_like(ref)
    ref.backward(g)
    gref = {n: p.grad.clone() for n, p in layer.named_parameters()}
    layer.zero_grad()
    out.backward(g)
    assert float((xf.grad - xr.grad).norm() / xr.grad.norm()) < 2e-2
    for n, p in layer.named_parameters():
        if n == "attn.k_linear.bias":     # softmax is shift-invariant per row: the true gradient is 0
            assert float(p.grad.norm()) < 0.05 * float(gref["attn.q_linear.bias"].norm())
            continue
        e = float((p.grad - gref[n]).norm() / (gref[n].norm() + 1e-12))
        assert e < 3e-2, (n, e)


def test_fused_transformer_two_layers_chained_layernorm(ext):
    """Two fused layers where layer 0's FF epilogue forms layer 1's LayerNorm (tfrow.hip) == two eager layers, forward
    and backward (layer 1's LN1 gamma / beta gradients come from its own QKV data-gradient epilogue)."""
    from pytorch_rt1_for_distributed_training_amd.models.transformer import _TransformerLayer, rt1_attention_mask
    from pytorch_rt1_for_distributed_training_amd.ops.attention import fused_layer
    torch.manual_seed(1)
    layers = [_TransformerLayer(128, 8, 512, 0.1).cuda().eval() for _ in range(2)]
    with torch.no_grad():
        for ly in layers:
            for m in (ly.norm_1, ly.norm_2):
                m.weight.uniform_(0.5, 1.5)
                m.bias.normal_(0, 0.1)
    B, T, L, K = 4, 6, 11, 8
    x = torch.randn(B, T * L, 512, device="cuda")
    mask = rt1_attention_mask(T, K, L - K).cuda()
    xr = x.clone().requires_grad_(True)
    ref = xr
    for ly in layers:
        ref, _ = ly(ref, mask)
    xf = x.clone().requires_grad_(True)
    h, aux = fused_layer(layers[0], xf, L, K, False, None, layers[1].norm_1)
    assert aux is not None and aux[0].dtype == torch.bfloat16
    out, aux2 = fused_layer(layers[1], h, L, K, False, aux, None)
    assert aux2 is None
    assert float((out - ref).norm() / ref.norm()) < 1e-2
    g = torch.randn_like(ref)
    ref.backward(g)
    gref = [{n: p.grad.clone() for n, p in ly.named_parameters()} for ly in layers]
    for ly in layers:
        ly.zero_grad()
    out.backward(g)
    assert float((xf.grad - xr.grad).norm() / xr.grad.norm()) < 2e-2
    for ly, gr in zip(layers, gref):
        for n, p in ly.named_parameters():
            if n == "attn.k_linear.bias":
                continue
            e = float((p.grad - gr[n]).norm() / (gr[n].norm() + 1e-12))
            assert e < 3e-2, (n, e)


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_resid_with_next_layernorm_equals_separate_kernels(ext, p):
    """tf_resid with the LayerNorm of its output == tf_resid then tf_ln_fwd, bit for bit; tf_ln_bwd's bf16 copy of dx
    and its column sums == tf_drop_bwd(dx, p=0)."""
    torch.manual_seed(4)
    T = 1000
    x = torch.randn(T, 512, device="cuda")
    a = torch.randn(T, 512, device="cuda").to(torch.bfloat16)
    b = torch.randn(512, device="cuda") * 0.1
    lg, lb = torch.rand(512, device="cuda") + 0.5, torch.randn(512, device="cuda") * 0.1
    ctr = torch.tensor([9], dtype=torch.int32, device="cuda")
    out, xn, mu, rs = ext.tf_resid(x, a, b, p, 77, ctr, lg, lb, 1e-6)
    (ref,) = ext.tf_resid(x, a, b, p, 77, ctr)
    assert torch.equal(out, ref)
    rxn, rmu, rrs = ext.tf_ln_fwd(ref, lg, lb, 1e-6)
    assert torch.equal(xn, rxn) and torch.equal(mu, rmu) and torch.equal(rs, rrs)
    dy = torch.randn(T, 512, device="cuda").to(torch.bfloat16)
    dres = torch.randn(T, 512, device="cuda")
    dx, dg, db, dxb, dsum = ext.tf_ln_bwd(dy, out, mu, rs, lg, dres, True)
    dx0, dg0, db0 = ext.tf_ln_bwd(dy, out, mu, rs, lg, dres)
    assert torch.equal(dx, dx0) and torch.equal(dg, dg0) and torch.equal(db, db0)
    rdb, rsum = ext.tf_drop_bwd(dx, 0.0, 0)
    assert torch.equal(dxb, rdb)
    torch.testing.assert_close(dsum, rsum, rtol=1e-5, atol=1e-4)


def test_fused_transformer_layer_dropout_train(ext):
    """train mode: attention + FF dropout active, finite grads, dropout actually changes the output"""
    from pytorch_rt1_for_distributed_training_amd.models.transformer import _TransformerLayer
    from pytorch_rt1_for_distributed_training_amd.ops.attention import fused_layer
    torch.manual_seed(3)
    layer = _TransformerLayer(128, 8, 512, 0.1).cuda().train()
    x = torch.randn(2, 66, 512, device="cuda", requires_grad=True)
    y1, _ = fused_layer(layer, x, 11, 8, True)
    y0, _ = fused_layer(layer, x, 11, 8, False)
    assert float((y1 - y0).norm()) > 0
    y1.square().mean().backward()
    assert all(torch.isfinite(p.grad).all() for p in layer.parameters())


@pytest.mark.parametrize("T,drop", [(15, 0.1), (15, 0.0), (6, 0.1), (23, 0.0)])
def test_rt1_attention_backward_long_kernel(ext, T, drop):
    """Streamed dK/dV + dQ kernels (any S <= 256) == the fp32 torch backward with the same keep-mask; at S <= 96
    they also agree with the single-workgroup kernel."""
    from pytorch_rt1_for_distributed_training_amd.ops import rng
    from pytorch_rt1_for_distributed_training_amd.ops.attention import RT1AttentionFn
    torch.manual_seed(5)
    B, H, D, L, K = 2, 8, 128, 11, 8
    S = T * L
    qkv = torch.randn(B, S, 3, H, D, device="cuda").to(torch.bfloat16)
    ctr = rng.counter(qkv.device)
    out, lse = ext.attn_fwd(qkv, L, K, D ** -0.5, drop, 91, ctr)
    dout = torch.randn(B, S, H, D, device="cuda").to(torch.bfloat16)
    dq = ext.attn_bwd_long(qkv, out, dout, lse, L, K, D ** -0.5, drop, 91, ctr)
    dref, *_ = RT1AttentionFn._backward_torch(qkv, out, lse, dout, L, K, drop, 91, D ** -0.5)
    for i, name in enumerate("qkv"):
        a, r = dq[:, :, i].float(), dref[:, :, i].float()
        err = float((a - r).norm() / r.norm())
        assert err < 1e-2, (name, err)
    if S <= 96:
        short = ext.attn_bwd(qkv, out, dout, lse, L, K, D ** -0.5, drop, 91, ctr)
        assert float((short.float() - dq.float()).norm() / short.float().norm()) < 5e-3


def test_fused_head_matches_eager(ext):
    """head.hip (gather + MFMA logits + CE + argmax, softmax-onehot gradient) vs fp32 torch on bf16-rounded
    operands: per-row CE, argmax, and the gradients of hidden / W / bias."""
    from pytorch_rt1_for_distributed_training_amd.models.transformer import action_prediction_positions
    from pytorch_rt1_for_distributed_training_amd.ops.head import head_ce
    torch.manual_seed(7)
    B, T, L, K, A, V, E = 5, 6, 11, 8, 3, 256, 512
    S = T * L
    lin = torch.nn.Linear(E, V).cuda()
    hidden = torch.randn(B, S, E, device="cuda", requires_grad=True)
    pos = action_prediction_positions(T, K, A).cuda()
    targets = torch.randint(0, V, (B, T * A), device="cuda")
    ce, pred = head_ce(lin, hidden, pos, targets)
    hr = hidden.detach().to(torch.bfloat16).float().requires_grad_(True)
    Wr = lin.weight.detach().to(torch.bfloat16).float().requires_grad_(True)
    br = lin.bias.detach().clone().requires_grad_(True)
    logits = torch.nn.functional.linear(hr[:, pos], Wr, br)                       # (B, P, V)
    ref = torch.nn.functional.cross_entropy(logits.reshape(-1, V), targets.reshape(-1), reduction="none")
    torch.testing.assert_close(ce, ref, rtol=2e-3, atol=2e-3)
    top2 = logits.detach().reshape(-1, V).topk(2, dim=-1).values
    clear = (top2[:, 0] - top2[:, 1]) > 1e-3                                      # rows without a near tie
    assert torch.equal(pred.long()[clear], logits.detach().reshape(-1, V).argmax(-1)[clear])
    w = torch.rand_like(ce)
    (ce * w).sum().backward()
    (ref * w).sum().backward()
    for got, want, name in ((hidden.grad, hr.grad, "hidden"), (lin.weight.grad, Wr.grad, "W"),
                            (lin.bias.grad, br.grad, "bias")):
        err = float((got.float() - want).norm() / want.norm())
        assert err < 1e-2, (name, err)
    untouched = torch.ones(S, dtype=torch.bool, device="cuda")
    untouched[pos] = False
    assert float(hidden.grad[:, untouched].abs().max()) == 0.0


@pytest.mark.parametrize("B,S", [(4, 66), (3, 165), (2, 7)])
def test_token_embedding_kernel_matches_eager(ext, B, S):
    """pwtall.hip rt1_embed_fwd (K11): tokens @ W^T + b + pos[:S] in fp32, and the EmbedFn gradients, vs fp32
    torch on bf16-rounded operands."""
    from pytorch_rt1_for_distributed_training_amd.models.transformer import Transformer
    from pytorch_rt1_for_distributed_training_amd.ops import embed as emb
    torch.manual_seed(B * S)
    tf = Transformer(num_layers=1, layer_size=512, num_heads=8, feed_forward_size=512, dropout_rate=0.0,
                     vocab_size=256).cuda()
    with torch.no_grad():
        tf._position_emb.weight.normal_()
        tf._token_emb.bias.normal_()
    tok = torch.randn(B, S, 512, device="cuda").to(torch.bfloat16).requires_grad_(True)
    assert emb.supported(tf, tok)
    out = emb.embed(tf, tok)
    assert out.dtype == torch.float32 and out.shape == (B, S, 512)
    tr = tok.detach().float().requires_grad_(True)
    Wr = tf._token_emb.weight.detach().to(torch.bfloat16).float().requires_grad_(True)
    br = tf._token_emb.bias.detach().clone().requires_grad_(True)
    pr = tf._position_emb.weight.detach().clone().requires_grad_(True)
    ref = torch.nn.functional.linear(tr, Wr, br) + pr[:S]
    torch.testing.assert_close(out, ref, rtol=2e-3, atol=2e-3)
    g = torch.randn_like(out)
    (out * g).sum().backward()
    (ref * g).sum().backward()
    for got, want, name in ((tok.grad, tr.grad, "tokens"), (tf._token_emb.weight.grad, Wr.grad, "W"),
                            (tf._token_emb.bias.grad, br.grad, "bias"), (tf._position_emb.weight.grad, pr.grad, "pos")):
        err = float((got.float() - want).norm() / want.norm())
        assert err < 1e-2, (name, err)


@pytest.mark.parametrize("P", [100, 120, 225])
def test_token_learner_kernels_match_eager(ext, P):
    """tokenlearner.hip forward + backward vs the fp32 eager TokenLearnerModule (bf16-rounded input)."""
    from pytorch_rt1_for_distributed_training_amd.models.token_learner import TokenLearnerModule
    from pytorch_rt1_for_distributed_training_amd.ops.token_learner import token_learner
    torch.manual_seed(3)
    tl = TokenLearnerModule(512, 8).cuda()
    with torch.no_grad():
        tl.layerNorm.weight.uniform_(0.5, 1.5)
        tl.layerNorm.bias.normal_(0, 0.1)
    N = 6
    x = torch.randn(N, P, 512, device="cuda").to(torch.bfloat16)
    xk = x.clone().requires_grad_(True)
    out = token_learner(tl, xk)
    gk = {n: None for n, _ in tl.named_parameters()}
    xr = x.float().clone().requires_grad_(True)
    ref = tl.forward_nhwc(xr)
    assert float((out.float() - ref).norm() / ref.norm()) < 1e-2
    g = torch.randn_like(ref)
    out.backward(g.to(torch.bfloat16))
    gk = {n: p.grad.clone() for n, p in tl.named_parameters()}
    tl.zero_grad()
    ref.backward(g)
    assert float((xk.grad.float() - xr.grad).norm() / xr.grad.norm()) < 2e-2
    for n, p in tl.named_parameters():
        if n == "conv2.bias":       # softmax over positions is shift-invariant per token: the true gradient is 0
            assert float(gk[n].norm()) < 1e-3 * float(gk["conv2.weight"].norm()) + 1e-6
            continue
        e = float((gk[n] - p.grad).norm() / (p.grad.norm() + 1e-12))
        assert e < 3e-2, (n, e)


def test_multi_copy_gathers_into_flat_views(ext):
    """reduce.hip multi_copy_ (the flat-gradient gather): 70 fp32 tensors of odd sizes into views of one buffer,
    misaligned offsets included (scalar path), bitwise equal to the sources."""
    torch.manual_seed(0)
    sizes = [1, 3, 4, 5, 17, 64, 1000, 4097, 65537, 300_001] * 7
    srcs = [torch.randn(n, device="cuda") for n in sizes]
    flat = torch.zeros(sum(sizes) + len(sizes), device="cuda")
    dsts, off = [], 0
    for n in sizes:
        dsts.append(flat[off:off + n])
        off += n + 1                      # odd offsets: some views are not 16-B aligned
    ext.multi_copy_(dsts, srcs)
    for d, s in zip(dsts, srcs):
        assert torch.equal(d, s)
    assert flat[sizes[0]].item() == 0.0   # the gaps stay untouched
