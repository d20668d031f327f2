#!/usr/bin/env python3
"""Bitwise run-to-run comparison of the fused encoder's per-block outputs (forward only) and of the
per-block input gradients (backward), to localise a nondeterministic kernel."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests.test_graph_gpu import _batches, _cfg, _engine  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.ops import backbone  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.engine.step import split_batch  # noqa: E402

res = int(sys.argv[1]) if len(sys.argv) > 1 else 96
cfg = _cfg(dropout_rate=0.0, drop_connect_rate=0.0, crop_ratio=0.0, height=res, width=res)
(batch,) = _batches(cfg, 1)
eng = _engine(cfg, graph=False)
m = eng.model
m.train()
images, ctx, actions = split_batch(batch)

rec = []
gre = []
for cls in (backbone.StemFn, backbone.MBConvFn, backbone.TopFn):
    orig = cls.apply

    def wrapped(*a, _orig=orig, _name=cls.__name__):
        out = _orig(*a)
        rec.append((_name, out.detach().clone()))
        if out.requires_grad:
            idx = len(gre)
            gre.append(None)
            out.register_hook(lambda g, i=idx, n=_name: gre.__setitem__(i, (n, g.detach().clone())))
        return out
    cls.apply = staticmethod(wrapped)

runs = []
for r in range(4):
    rec.clear()
    gre.clear()
    eng.optimizer.zero_grad()
    tok = m.tokenize_images(images, ctx, None)
    tok.float().square().sum().backward()
    torch.cuda.synchronize()
    runs.append((list(rec), list(gre), tok.detach().clone()))

for r in range(1, 4):
    fr, gr, tk = runs[r]
    f0, g0, t0 = runs[0]
    print(f"run {r}: tokens max|d| {float((tk.float() - t0.float()).abs().max()):.3e}")
    for i, ((n, a), (_, b)) in enumerate(zip(f0, fr)):
        d = float((a.float() - b.float()).abs().max())
        if d > 0:
            print(f"   fwd {i:2d} {n}: max|d| {d:.3e} (|x| {float(a.float().abs().max()):.3e})")
            break
    for i, (x, y) in enumerate(zip(g0, gr)):
        if x is None or y is None:
            continue
        d = float((x[1].float() - y[1].float()).abs().max())
        if d > 0:
            print(f"   grad-of-output {i:2d} {x[0]}: max|d| {d:.3e} (|g| {float(x[1].float().abs().max()):.3e})")
