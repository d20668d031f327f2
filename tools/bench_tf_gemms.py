#!/usr/bin/env python3
"""The transformer's projection GEMMs at the bench shape (T = B x S = 8448 token rows at b128): hipBLASLt with the
recorded TunableOp solutions (what the step runs) against gemm.hip's tile configs, median of interleaved rounds.

  python tools/bench_tf_gemms.py [--rows 8448] [--iters 50] [--rounds 5]
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_rt1_for_distributed_training_amd.utils import tuned_gemms  # noqa: E402

tuned_gemms.enable_tuned_gemms()
from pytorch_rt1_for_distributed_training_amd import ops  # noqa: E402

BF = torch.bfloat16
# (name, N, K, nn, bias): forward C = X W^T (+ b), data gradient C = dY W
SHAPES = [("qkv fwd", 3072, 512, False, True), ("out fwd", 512, 1024, False, False), ("ff fwd", 512, 512, False, False),
          ("ff dgrad", 512, 512, True, False), ("out dgrad", 1024, 512, True, False), ("qkv dgrad", 512, 3072, True, False)]


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=8448)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    ext = ops.load()
    M = a.rows
    print(f"{'shape':10s} {'N':>5s} {'K':>5s} {'roof':>6s} {'lib':>7s} {'g0':>7s} {'g1':>7s} {'g2':>7s} {'g3':>7s} {'g4':>7s}", flush=True)
    for name, N, K, nn, has_b in SHAPES:
        x = torch.randn(M, K, device="cuda").to(BF)
        w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(BF)
        b = (torch.randn(N, device="cuda") * 0.1) if has_b else None
        wb = w.t().contiguous() if nn else w                      # NN: B is [K, N]
        bb = b.to(BF) if b is not None else None
        roof = max((M * K + N * K + M * N) * 2 / 5.0e12, 2 * M * N * K / 2.3e15) * 1e6
        ref = (x.float() @ (wb.float() if nn else w.float().t()) + (b if b is not None else 0)).to(BF)
        if nn:
            lib = lambda: torch.mm(x, wb)
        elif has_b:
            lib = lambda: torch.addmm(bb, x, w.t())
        else:
            lib = lambda: torch.mm(x, w.t())
        cands = {"lib": lib}
        for cfg in range(5):
            out = ext.gemm(x, wb, nn, b, cfg=cfg)[0]
            err = float((out.float() - ref.float()).norm() / ref.float().norm())
            assert err < 1e-2, (name, cfg, err)
            cands[f"g{cfg}"] = (lambda c=cfg: ext.gemm(x, wb, nn, b, cfg=c))
        times = {k: [] for k in cands}
        for _ in range(a.rounds):
            for k, fn in cands.items():
                times[k].append(timeit(fn, a.iters))
        med = {k: statistics.median(v) for k, v in times.items()}
        print(f"{name:10s} {N:5d} {K:5d} {roof:6.1f} " + " ".join(f"{med[k]:7.1f}" for k in cands), flush=True)


if __name__ == "__main__":
    main()
