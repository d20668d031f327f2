#!/usr/bin/env python3
"""Production-faithful depthwise timing: record every depthwise kernel call (forward, x-mode forward, fused / x-mode
backward) that ONE eager training step of the bench configuration makes, with its exact arguments (tile / grid caps,
zout, residual epilogue, x-mode), then replay each recorded call alone and time it (HIP events, median).

``--ab <other .so>`` loads a second build of the extension into the same process (a ``build.py --variant`` build) and
replays every recorded call on BOTH builds, interleaved launch by launch on identical inputs: per call the two medians
and the relative difference of the outputs (forward: the output map; backward: dx / dz and dW).  The step itself is
recorded with the in-tree build (or RT1_HIP_SO).

  python tools/bench_dw_replay.py [--batch 128] [--res 300] [--iters 10] [--match bwd] [--ab build/base/<so>]
"""
from __future__ import annotations

import argparse
import importlib.util
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

NAMES = ("dw_fwd", "dw_fwd_x", "dw_bwd_fused", "dw_bwd_fused_x")


def _desc(name, args):
    shp = [tuple(a.shape) for a in args if isinstance(a, torch.Tensor) and a.dim() == 4]
    return f"{name} {shp[0] if shp else ''}"


def load_other(path):
    """A second build of _rt1_hip in this process (its pybind classes are module-local, so both can be loaded)."""
    spec = importlib.util.spec_from_file_location("_rt1_hip", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _time(fns, args, kw, iters):
    """Median us of each fn, launches interleaved (fn0, fn1, fn0, ...) so clock drift hits both alike."""
    for f in fns:
        for _ in range(2):
            f(*args, **kw)
    ts = [[] for _ in fns]
    for _ in range(iters):
        for k, f in enumerate(fns):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f(*args, **kw)
            e1.record()
            e1.synchronize()
            ts[k].append(e0.elapsed_time(e1) * 1e3)
    return [sorted(t)[len(t) // 2] for t in ts]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--res", type=int, default=300)
    ap.add_argument("--seq_len", type=int, default=6)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--match", default="")
    ap.add_argument("--ab", default="", help="second build of the extension (.so) to time against, same inputs")
    a = ap.parse_args()
    from pytorch_rt1_for_distributed_training_amd import ops
    from pytorch_rt1_for_distributed_training_amd.config import RT1Config
    from pytorch_rt1_for_distributed_training_amd.data.synthetic import make_batch
    from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine
    from pytorch_rt1_for_distributed_training_amd.models import build_rt1
    ext = ops.load()
    other = load_other(a.ab) if a.ab else None
    torch.manual_seed(0)
    cfg = RT1Config(height=a.res, width=a.res, seq_len=a.seq_len, backend="hip")
    eng = TrainEngine(build_rt1(cfg), cfg, order_probe=False, graph=False)
    g = torch.Generator().manual_seed(1)
    batch = make_batch(a.batch, cfg.seq_len, a.res, a.res, device="cuda", generator=g)
    eng.train_step(batch)                                    # warm-up (lazy state, tile caches)
    torch.cuda.synchronize()
    calls = []
    orig = {n: getattr(ext, n) for n in NAMES}

    def wrap(n):
        f = orig[n]

        def rec(*args, **kw):
            calls.append((n, args, kw))
            return f(*args, **kw)
        return rec
    for n in NAMES:
        setattr(ext, n, wrap(n))
    try:
        eng.train_step(make_batch(a.batch, cfg.seq_len, a.res, a.res, device="cuda", generator=g))
        torch.cuda.synchronize()
    finally:
        for n in NAMES:
            setattr(ext, n, orig[n])
    tot = {}
    print(f"[{os.environ.get('RT1_HIP_SO', 'in-tree build')}{' vs ' + a.ab if a.ab else ''}] "
          f"{len(calls)} depthwise calls in one step")
    for i, (n, args, kw) in enumerate(calls):
        d = _desc(n, args)
        if a.match and a.match not in d:
            continue
        fns = [orig[n]] + ([getattr(other, n)] if other is not None else [])
        us = _time(fns, args, kw, a.iters)
        kind = "fwd" if n.startswith("dw_fwd") else "bwd"
        for k, u in enumerate(us):
            tot[(kind, k)] = tot.get((kind, k), 0.0) + u
        extra = ""
        if other is not None:
            oa, ob = fns[0](*args, **kw), fns[1](*args, **kw)
            nout = 1 if kind == "fwd" else 2
            diffs = [float((oa[j].float() - ob[j].float()).norm() / (ob[j].float().norm() + 1e-12))
                     for j in range(nout)]
            extra = (f" | other {us[1]:9.1f} us  {100 * (us[0] - us[1]) / us[1]:+6.1f} %  out rel diff " +
                     " ".join(f"{x:.1e}" for x in diffs))
        print(f"{i:3d} {d:42s} {us[0]:9.1f} us{extra}", flush=True)
    for k in range(2 if other is not None else 1):
        name = "this build" if k == 0 else "other build"
        print(f"total ({name}): " + ", ".join(f"{kind} {v / 1e3:.3f} ms" for (kind, kk), v in sorted(tot.items())
                                              if kk == k) +
              f", all {sum(v for (kind, kk), v in tot.items() if kk == k) / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
