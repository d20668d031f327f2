#!/usr/bin/env python3
"""Run-to-run determinism of one forward+backward (same model, same batch, no optimizer step): lists the
parameters that contribute most to the gradient difference."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests.test_graph_gpu import _batches, _cfg, _engine  # noqa: E402

res = int(sys.argv[1]) if len(sys.argv) > 1 else 96
cfg = _cfg(dropout_rate=0.0, drop_connect_rate=0.0, crop_ratio=0.0, height=res, width=res)
(batch,) = _batches(cfg, 1)
eng = _engine(cfg, graph=False)
pn = {id(p): n for n, p in eng.model.named_parameters()}


def grads():
    eng.optimizer.zero_grad()
    loss, _ = eng.forward_loss(batch)
    loss.backward()
    eng.flat.gather_grads()
    return float(loss), eng.flat.grad.clone()


runs = [grads() for _ in range(3)]
for k in (1, 2):
    (la, ga), (lb, gb) = runs[0], runs[k]
    d = ga - gb
    print(f"run0 vs run{k}: loss {la:.7f} {lb:.7f} grad rel {float(d.norm() / ga.norm()):.3e}")
    contrib = []
    for p, o in zip(eng.flat.params, eng.flat.offsets):
        n = p.numel()
        contrib.append((float(d[o:o + n].norm()), float(ga[o:o + n].norm()), pn.get(id(p), "?")))
    contrib.sort(reverse=True)
    for c in contrib[:8]:
        print(f"   |dg| {c[0]:.3e}  |g| {c[1]:.3e}  {c[2]}")
