#!/usr/bin/env python3
"""Which parameters' gradients are not reproducible, eager vs eager and eager vs the captured graph (one GPU)?

From one state (parameters, Adam moments, BN statistics, RNG, dropout counter) the tool runs the same batch three
times -- eager step A, eager step B, one graph replay G -- restoring the state in between (TrainEngine._snapshot /
_restore), and prints the parameters whose gradients differ (max |diff| and the number of differing elements).
Switches bisect the kernel paths (e.g. RT1_AB=se_fused=0,proj_bwd=0; ops/switches.py).

  python tools/step_determinism.py [--batch 128] [--hw 300] [--repeats 2]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--hw", type=int, default=300)
    ap.add_argument("--seq", type=int, default=6)
    ap.add_argument("--repeats", type=int, default=2)
    ap.add_argument("--nodrop", action="store_true", help="dropout / drop-path / random shift off")
    a = ap.parse_args()
    from pytorch_rt1_for_distributed_training_amd.utils.tuned_gemms import enable_tuned_gemms
    enable_tuned_gemms()
    import torch
    from pytorch_rt1_for_distributed_training_amd.config import RT1Config
    from pytorch_rt1_for_distributed_training_amd.data.synthetic import make_batch
    from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine
    from pytorch_rt1_for_distributed_training_amd.models import build_rt1

    kw = dict(dropout_rate=0.0, drop_connect_rate=0.0, crop_ratio=0.0) if a.nodrop else {}
    cfg = RT1Config(height=a.hw, width=a.hw, seq_len=a.seq, backend="hip", **kw)
    torch.manual_seed(0)
    eng = TrainEngine(build_rt1(cfg), cfg, order_probe=False, graph=True)
    names = {id(p): n for n, p in eng.model.named_parameters()}
    g = torch.Generator().manual_seed(1)
    batches = [make_batch(a.batch, cfg.seq_len, cfg.height, cfg.width, device="cuda", generator=g, uint8=True)
               for _ in range(3)]
    eng.train_step(batches[0])          # eager + capture
    eng.train_step(batches[1])          # replay
    torch.cuda.synchronize()
    b = batches[2]

    def run(kind):
        snap = eng._snapshot()
        if kind == "graph":
            eng.train_step(b)
        else:
            eng._step_body(b)
        torch.cuda.synchronize()
        out = eng.flat.grad.clone()
        eng._restore(snap)
        torch.cuda.synchronize()
        return out

    def report(tag, x, y):
        if torch.equal(x, y):
            print(f"{tag}: bitwise equal", flush=True)
            return
        rows = []
        for p, (off, n) in zip(eng.flat.params, (eng.flat.segment(i) for i in range(len(eng.flat.params)))):
            d = (x[off:off + n] - y[off:off + n]).abs()
            m = float(d.max())
            if m > 0:
                rows.append((m, int((d > 0).sum()), n, names.get(id(p), "?")))
        rows.sort(reverse=True)
        print(f"{tag}: {len(rows)} parameters differ; largest:", flush=True)
        for m, cnt, n, nm in rows[:12]:
            print(f"   {nm}: max {m:.3e}, {cnt}/{n} elements", flush=True)

    ga = run("eager")
    for r in range(a.repeats):
        report(f"eager vs eager #{r + 1}", ga, run("eager"))
    report("eager vs graph", ga, run("graph"))


if __name__ == "__main__":
    main()
