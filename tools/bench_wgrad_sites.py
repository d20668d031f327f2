#!/usr/bin/env python3
"""Every csrc/kernels/wgrad.hip call of one eager hip-backend training step (shapes, prologue, call site captured by
wrapping the binding), re-timed in isolation with the configuration the step used and with every tile variant x
row-split count; prints the step's choice against the best few (median us, split partial sum included).  With
--bmm: the library split-K weight gradients (ops/backbone.py wgrad_bmm) instead, against other split counts and
against the MFMA kernel's variants x splits.

  python tools/bench_wgrad_sites.py [--batch 128] [--top 4] [--bmm]
"""
from __future__ import annotations

import argparse
import os
import sys
import traceback

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_dw_phases import timeit  # noqa: E402

PKG = "pytorch_rt1_for_distributed_training_amd"
SPLITS = (1, 2, 4, 8, 12, 16, 24, 32, 48, 64, 96, 128, 192, 256)


def _site() -> str:
    for fr in reversed(traceback.extract_stack()[:-2]):
        if PKG in fr.filename and "bench_wgrad_sites" not in fr.filename:
            return f"{fr.filename.split(PKG + '/')[-1]}:{fr.lineno}"
    return "?"


def Co_ci_bad(co: int, ci: int) -> bool:
    return co % 8 != 0 or ci % 8 != 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--top", type=int, default=4)
    ap.add_argument("--bmm", action="store_true")
    a = ap.parse_args()
    from pytorch_rt1_for_distributed_training_amd.config import RT1Config
    from pytorch_rt1_for_distributed_training_amd.data.synthetic import make_batch
    from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine, to_device
    from pytorch_rt1_for_distributed_training_amd.models import build_rt1
    from pytorch_rt1_for_distributed_training_amd.ops._ext import load

    ext = load()
    real = ext.wgrad
    calls = {}
    active = [False]

    def spy(dy, x, *args, **kw):
        if active[0]:
            key = (tuple(dy.shape), tuple(x.shape), len(args) > 0 and args[0] is not None, kw.get("variant", -1),
                   kw.get("splits", -1), _site())
            if key not in calls:
                calls[key] = (dy.clone(), x.clone(), args, dict(kw))
        return real(dy, x, *args, **kw)

    from pytorch_rt1_for_distributed_training_amd.ops import backbone
    real_bmm = backbone.wgrad_bmm
    real_splits = backbone._wgrad_splits

    def spy_bmm(dy, x):
        if active[0]:
            key = (tuple(dy.shape), tuple(x.shape), False, "bmm", real_splits(dy.shape[0], dy.shape[1] * x.shape[1]),
                   _site())
            if key not in calls:
                calls[key] = (dy.clone(), x.clone(), (), {})
        return real_bmm(dy, x)

    if a.bmm:
        backbone.wgrad_bmm = spy_bmm
    else:
        ext.wgrad = spy
    dev = torch.device("cuda", 0)
    cfg = RT1Config(height=300, width=300, seq_len=6, backend="hip")
    eng = TrainEngine(build_rt1(cfg), cfg, order_probe=False, device=dev)
    eng.graph = False
    batch = to_device(make_batch(a.batch, cfg.seq_len, cfg.height, cfg.width), dev)
    eng.train_step(batch)
    active[0] = True
    eng.train_step(batch)
    active[0] = False
    ext.wgrad = real
    backbone.wgrad_bmm = real_bmm
    del eng
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    print(f"{len(calls)} distinct wgrad calls")
    for (ds, xs, pro, v0, s0, site), (dy, x, args, kw) in sorted(calls.items(), key=lambda kv: -kv[0][0][0]):
        M = dy.shape[0]
        rows = []
        if v0 == "bmm":
            base = timeit(lambda: real_bmm(dy, x), a.iters)
            for s in SPLITS:
                if s * 256 > M:
                    continue
                backbone._wgrad_splits = lambda m, o, s=s: s
                rows.append((timeit(lambda: real_bmm(dy, x), a.iters), "bmm", s))
            backbone._wgrad_splits = real_splits
        else:
            base = timeit(lambda: real(dy, x, *args, **kw), a.iters)
        for v in range(6):
            for s in SPLITS:
                if s * 64 > M:
                    continue
                kw2 = dict(kw, variant=v, splits=s)
                if Co_ci_bad(ds[1], xs[1]):
                    continue
                try:
                    rows.append((timeit(lambda: real(dy, x, *args, **kw2), a.iters), v, s))
                except RuntimeError:
                    pass
        rows.sort(key=lambda r: r[0])
        best = " ".join(f"v{v}/s{s}:{t:.1f}" for t, v, s in rows[:a.top])
        print(f"M={M:8d} Co={ds[1]:5d} Ci={xs[1]:5d} pro={int(pro)} step(v{v0}/s{s0}) {base:7.1f} | best {best} | {site}",
              flush=True)
        del dy, x
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
