"""Whole-model parity of the HIP backend against the fp32 eager PyTorch model (the reference's numerics).

Component tests compare each kernel with its fp32 op; these compare the WHOLE step: full-depth FiLM-EfficientNet-B3
+ TokenLearner + 8-layer transformer, hip backend (bf16 activations, fused kernels) vs torch backend (fp32) on
identical weights and batch, with dropout / drop-path / random shift off (reference test strategy:
``transformer_network_test.py:99-157`` checks the same model end to end).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _cfgs(**kw):
    from pytorch_rt1_for_distributed_training_amd.config import RT1Config
    base = dict(height=128, width=128, seq_len=2, num_layers=8, dropout_rate=0.0, drop_connect_rate=0.0,
                crop_ratio=0.0)
    base.update(kw)
    return RT1Config(backend="hip", dtype="bf16", **base), RT1Config(backend="torch", dtype="fp32", **base)


def _twins(**kw):
    from pytorch_rt1_for_distributed_training_amd.models import build_rt1
    ch, ct = _cfgs(**kw)
    torch.manual_seed(0)
    mh = build_rt1(ch)
    mt = build_rt1(ct)
    mt.load_state_dict(mh.state_dict())
    return ch, ct, mh, mt


def _engines(**kw):
    from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine
    ch, ct, mh, mt = _twins(**kw)
    eh = TrainEngine(mh, ch, order_probe=False, device=torch.device("cuda"))
    et = TrainEngine(mt, ct, order_probe=False, device=torch.device("cuda"))
    assert eh.backend == "hip" and et.backend == "torch"
    return eh, et


def _batch(cfg, b=4, seed=5):
    from pytorch_rt1_for_distributed_training_amd.data.synthetic import make_batch
    g = torch.Generator().manual_seed(seed)
    return make_batch(b, cfg.seq_len, cfg.height, cfg.width, device="cuda", generator=g)


def _grads(eng):
    eng.optimizer.zero_grad()
    loss, _ = eng.forward_loss(eng._batch)
    loss.backward()
    eng.flat.gather_grads()
    return float(loss), {n: p.grad.detach().float().clone() for n, p in eng.model.named_parameters()
                         if p.requires_grad}


SEEDS = (5, 7, 11)


# (height, width): 128x128 (fast), the benchmarked 300x300 and the reference CLI default 256x456.  The production
# kernels are shape-specialised (depthwise tile search keyed on the output map, grid caps keyed on map size / width,
# 5-output strips keyed on width divisibility), so the whole step is checked at the maps the bench and training run:
# 150/75/38/19/10 (300x300) and 128x228 .. 8x15 (256x456).
RESOLUTIONS = [(128, 128), (300, 300), (256, 456)]


@pytest.mark.parametrize("hw", RESOLUTIONS, ids=lambda hw: f"{hw[0]}x{hw[1]}")
def test_full_model_step_hip_bf16_vs_torch_fp32(hw):
    """Per-tensor gradient cosine vs fp32, averaged over three batches.  A single batch is not a stable measure for
    the most cancellation-prone tensors: the SE fc1 weight of block 0 scores hip 0.948 / 0.982 / 0.983 / 0.988 and
    torch-bf16 0.969 / 0.959 / 0.812 / 0.975 on batches 5 / 7 / 11 / 13, and re-ordering the fp32 SE sums alone
    moves it by 0.02 (profiles/r3_parity_seeds.log), so the per-tensor slack is checked on the batch mean."""
    from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine
    from pytorch_rt1_for_distributed_training_amd.models import build_rt1
    eh, et = _engines(height=hw[0], width=hw[1])
    # third model: the same weights under torch bf16 autocast -- the precision floor any bf16 implementation has
    cb = et.cfg.replace(dtype="bf16")
    mb = build_rt1(cb)
    mb.load_state_dict(et.model.state_dict())
    eb = TrainEngine(mb, cb, order_probe=False, device=torch.device("cuda"))
    for e in (eh, et, eb):
        e.model.train()
    cos_sum, cosb_sum, rms_t, rms_h = {}, {}, {}, {}
    for seed in SEEDS:
        batch = _batch(eh.cfg, seed=seed)
        eh._batch = et._batch = eb._batch = batch
        lh, gh = _grads(eh)
        lt, gt = _grads(et)
        _, gb = _grads(eb)
        assert abs(lh - lt) / abs(lt) < 2e-2, (seed, lh, lt)
        for n in gt:
            a, b = gh[n].flatten(), gt[n].flatten()
            nb = float(b.norm())
            if nb == 0.0:
                assert float(a.norm()) == 0.0, n
                continue
            cos_sum[n] = cos_sum.get(n, 0.0) + float(torch.dot(a, b) / (a.norm() * b.norm() + 1e-30))
            cosb_sum[n] = cosb_sum.get(n, 0.0) + float(torch.dot(gb[n].flatten(), b) /
                                                        (gb[n].norm() * b.norm() + 1e-30))
            rms_t[n] = max(rms_t.get(n, 0.0), nb / math.sqrt(gt[n].numel()))
            rms_h[n] = max(rms_h.get(n, 0.0), float(a.norm()) / math.sqrt(gt[n].numel()))
    cos = {n: v / len(SEEDS) for n, v in cos_sum.items()}
    # Gradients that are ZERO in exact arithmetic because of an invariance (attention keys' bias under the
    # softmax, TokenLearner's conv2 bias under its softmax over positions, BN3 beta / FiLM add-bias whose every
    # consumer is a BatchNorm'd conv) come out as rounding noise in both backends (fp32 rms ~1e-6..1e-8 of the
    # median tensor): cosine is meaningless there, so those are checked to stay negligible in the hip backend too.
    import re
    import statistics
    med = statistics.median(rms_t[n] for n in cos)
    # Structurally invariant tensors are recognised by name too: a per-channel constant added to a block output (the
    # project-BN beta, the FiLM add-projection's bias) only ever reaches BatchNorm'd convs, so its exact gradient is 0.
    # In fp32 their rounding noise grows with the map size: at 300x300 six of them sit above the 1e-4 rms threshold,
    # where hip and torch-bf16 alike score cosines of 0.1-0.4 against that noise (profiles/r6_parity_300_first.log).
    structural = re.compile(r"(blocks\.\d+\.block\.\d+\.1\.bias|films\.\d+\._projection_add\.bias)$")
    proj_bn = {f"_image_tokenizer._tokenizer.net.blocks.{i}.block.{len(b.block) - 1}.1.bias"
               for i, b in enumerate(eh.model._image_tokenizer._tokenizer.net.blocks)}
    invariant = {n for n in cos if rms_t[n] < 1e-4 * med or
                 (structural.search(n) and ("films" in n or n in proj_bn))}
    real = {n: c for n, c in cos.items() if n not in invariant}
    cos_b = {n: cosb_sum[n] / len(SEEDS) for n in real}
    worst = sorted(real.items(), key=lambda kv: kv[1])[:6]
    print(f"\n[{hw[0]}x{hw[1]}, b4 T2] loss hip {lh:.6f} torch-fp32 {lt:.6f}; {len(cos)} gradient tensors: {len(real)} compared by cosine "
          f"(mean over batches {SEEDS}; min {worst[0][1]:.5f}); {len(invariant)} zero-by-invariance, max hip rms "
          f"{max((rms_h[n] for n in invariant), default=0) / med:.2e} of the median")
    print(f"torch bf16-autocast vs fp32: min cosine {min(cos_b.values()):.5f}")
    for n, c in worst:
        print(f"  hip cos {c:.5f}   torch-bf16 cos {cos_b[n]:.5f}   {n}")
    import numpy as np
    ch = np.array([real[n] for n in real])
    cbv = np.array([cos_b[n] for n in real])
    q = lambda a: " / ".join(f"{v:.4f}" for v in np.percentile(a, [1, 5, 50]))
    worse = [n for n in real if real[n] < min(0.99, cos_b[n] - 0.02)]
    print(f"cosine percentiles 1/5/50 %: hip {q(ch)}   torch-bf16 {q(cbv)};  mean hip {ch.mean():.4f} "
          f"torch-bf16 {cbv.mean():.4f};  {len(worse)} tensors more than 0.02 below torch-bf16: {worse[:8]}")
    assert len(real) > 450
    # the hip backend is at least as faithful to fp32 as torch's own bf16 autocast, tensor by tensor and on average
    assert ch.mean() >= cbv.mean() - 0.005, (ch.mean(), cbv.mean())
    # the worst hip tensor is no worse than torch-bf16's worst (an absolute floor is not meaningful: the cancellation-
    # prone SE fc1 tensors sit at 0.95 in torch's own bf16 autocast too)
    assert ch.min() >= cbv.min(), (worst[:3], cbv.min())
    for n, c in real.items():
        assert c >= min(0.99, cos_b[n] - 0.02), (n, c, cos_b[n])


def test_loss_trajectory_20_steps_fixed_batch():
    """20 Adam steps on one batch.  lr 1e-4 keeps the fixed-batch loss from collapsing to ~1e-5 within a few
    steps (at the reference lr 5e-4 it memorises the batch by step 5, after which relative differences of
    near-zero losses say nothing); tolerance 5 % of the loss plus 0.2 % of the initial loss."""
    eh, et = _engines()
    for e in (eh, et):
        e.optimizer.param_groups[0]["lr"] = 1e-4
    batch = _batch(eh.cfg, seed=9)
    lh = [float(eh.train_step(batch)) for _ in range(20)]
    lt = [float(et.train_step(batch)) for _ in range(20)]
    print("\nhip  ", [round(x, 6) for x in lh], "\ntorch", [round(x, 6) for x in lt])
    for i, (a, b) in enumerate(zip(lh, lt)):
        assert abs(a - b) <= 0.05 * abs(b) + 2e-3 * abs(lt[0]), (i, a, b)
    assert lh[-1] < lh[0] and lt[-1] < lt[0]


def test_eval_mode_running_stats_forward():
    """Validation / test losses use the running-statistics BN path of the fused encoder (Trainer.validate)."""
    eh, et = _engines()
    for s in range(3):                                   # move the running stats away from their init
        eh.train_step(_batch(eh.cfg, seed=20 + s))
    torch.cuda.synchronize()
    et.model.load_state_dict(eh.model.state_dict())
    batch = _batch(eh.cfg, seed=30)
    lh = float(eh.eval_step(batch))
    lt = float(et.eval_step(batch))
    rm = eh.model._image_tokenizer._tokenizer.net.blocks[5].depthwise[1].running_mean
    assert float(rm.abs().sum()) > 0
    assert abs(lh - lt) / abs(lt) < 2e-2, (lh, lt)


def test_inference_graph_replay_vs_eager_vs_fp32_80_steps():
    from pytorch_rt1_for_distributed_training_amd.engine.infer import InferenceEngine
    from pytorch_rt1_for_distributed_training_amd.models import build_rt1
    ch, ct, mh, mt = _twins(seq_len=6)
    torch.manual_seed(0)
    mh2 = build_rt1(ch)
    mh2.load_state_dict(mh.state_dict())
    g_hip = InferenceEngine(mh, ch, device="cuda", backend="hip", graph=True)
    e_hip = InferenceEngine(mh2, ch, device="cuda", backend="hip", graph=False)
    e_t = InferenceEngine(mt, ct, device="cuda", backend="torch")
    gen = torch.Generator().manual_seed(3)
    agree = total = 0
    max_rel = 0.0
    for step in range(80):
        if step == 40:                                    # new episode half-way
            for e in (g_hip, e_hip, e_t):
                e.reset()
        img = torch.randint(0, 256, (1, 3, 128, 128), generator=gen, dtype=torch.uint8)
        ctx = torch.randn(1, 512, generator=gen)
        a = {k: v.clone() for k, v in g_hip.step(img, ctx).items()}
        b = e_hip.step(img, ctx)
        c = e_t.step(img, ctx)
        assert torch.equal(a["tokens"], b["tokens"]) and torch.equal(a["logits"], b["logits"]), step
        rel = float((a["logits"] - c["logits"]).abs().max() / (c["logits"].abs().max() + 1e-6))
        max_rel = max(max_rel, rel)
        agree += int((a["tokens"] == c["tokens"]).sum())
        total += a["tokens"].numel()
    print(f"\nhip graph == hip eager over 80 steps; vs torch fp32: max rel logit err {max_rel:.4f}, "
          f"token agreement {agree}/{total}")
    assert max_rel < 0.05
    assert agree / total >= 0.9
    # latency of one closed-loop policy step at the bench resolution
    from pytorch_rt1_for_distributed_training_amd.config import RT1Config
    cfg300 = RT1Config(height=300, width=300, seq_len=6, backend="hip")
    torch.manual_seed(0)
    eng300 = InferenceEngine(build_rt1(cfg300), cfg300, device="cuda", backend="hip", graph=True)
    ms = eng300.latency_ms(steps=40)
    eng_eager = InferenceEngine(build_rt1(cfg300), cfg300, device="cuda", backend="hip", graph=False)
    ms_eager = eng_eager.latency_ms(steps=20)
    print(f"policy step latency at 300x300, T=6, b=1: hipGraph {ms:.3f} ms, eager hip {ms_eager:.3f} ms")
    assert math.isfinite(ms) and ms < ms_eager
