#!/usr/bin/env python3
"""Per-step loss / gradient differences: eager vs eager (determinism) and eager vs hipGraph replay."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests.test_graph_gpu import _batches, _cfg, _engine  # noqa: E402

cfg = _cfg(dropout_rate=0.0, drop_connect_rate=0.0, crop_ratio=0.0)
batches = _batches(cfg, 4)


def run(graph):
    eng = _engine(cfg, graph=graph)
    out = []
    for b in batches:
        loss = float(eng.train_step(b))
        out.append((loss, eng.flat.grad.clone(), eng.flat.data.clone()))
    return eng, out


_, a = run(False)
_, b = run(False)
eng, c = run(True)
names = []
for p, o in zip(eng.flat.params, eng.flat.offsets):
    names.append((o, p.numel()))
pn = {id(p): n for n, p in eng.model.named_parameters()}
for tag, other in (("eager-vs-eager", b), ("eager-vs-graph", c)):
    for i, ((la, ga, pa), (lb, gb, pb)) in enumerate(zip(a, other)):
        rel = float((ga - gb).norm() / ga.norm())
        prel = float((pa - pb).norm() / pa.norm())
        print(f"{tag} step {i}: loss {la:.6f} {lb:.6f} grad rel {rel:.3e} param rel {prel:.3e}")
        if rel > 1e-3:
            worst = []
            for p, (o, n) in zip(eng.flat.params, names):
                e = float((ga[o:o + n] - gb[o:o + n]).norm() / (ga[o:o + n].norm() + 1e-20))
                worst.append((e, pn.get(id(p), "?"), float(ga[o:o + n].norm())))
            worst.sort(reverse=True)
            print("   worst:", [(f"{e:.2e}", n, f"{g:.2e}") for e, n, g in worst[:6]])
