#!/usr/bin/env python3
"""Time csrc/kernels/gemm256.hip against what the step runs today on the deep / wide 1x1-conv shapes: hipBLASLt (with
the recorded TunableOp solutions, as in the step), gemm.hip (best tile config) and pwgemm.hip's wide-N kernel where it
covers the shape.  Random operands (guide §5.4 rule 25), one process, interleaved rounds (rule 24); reports the median.

  python tools/bench_gemm256.py [--iters 30] [--rounds 3]
"""
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
# (name, M, N, K, nn): forward products (NT, C = A W^T) and data gradients (NN, C = dY W) at b128 / 300x300
SHAPES = [
    ("top fwd", 76800, 1536, 384, False), ("exp25 fwd", 76800, 2304, 384, False),
    ("exp19 fwd", 76800, 1392, 232, False), ("exp13 fwd", 277248, 816, 136, False),
    ("exp9 fwd", 277248, 576, 96, False), ("conv1x1 fwd", 76800, 512, 1536, False),
    ("proj25 fwd", 76800, 384, 2304, False), ("proj24 fwd", 76800, 384, 1392, False),
    ("proj19 fwd", 76800, 232, 1392, False),
    ("proj25 dgrad", 76800, 2304, 384, True), ("proj19 dgrad", 76800, 1392, 232, True),
    ("conv1x1 dgrad", 76800, 1536, 512, True), ("top dgrad", 76800, 384, 1536, True),
    ("exp25 dgrad", 76800, 384, 2304, True), ("exp19 dgrad", 76800, 232, 1392, True),
    ("qkv fwd", 8448, 3072, 512, False), ("qkv dgrad", 8448, 512, 3072, True),
]


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
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    ext = ops.load()
    print(f"{'shape':14s} {'M':>6s} {'N':>5s} {'K':>5s} {'roof':>6s} {'lib':>7s} {'gemm':>7s} {'pw':>7s} "
          f"{'g256':>7s} {'g128':>7s}  best-ours vs best-today", flush=True)
    for name, M, N, K, nn in SHAPES:
        x = torch.randn(M, K, device="cuda").to(BF)
        w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(BF)
        b = w.t().contiguous() if nn else w
        roof = max((M * K + N * K + M * N) * 2 / 5.3e12, 2 * M * N * K / 2.3e15) * 1e6
        cands = {"lib": (lambda: torch.mm(x, b)) if nn else (lambda: torch.mm(x, w.t())),
                 "gemm": None, "pw": None,
                 "g256": lambda: ext.gemm256(x, b, nn, bn=256), "g128": lambda: ext.gemm256(x, b, nn, bn=128)}
        if not nn and ext.pw_gemm_supported(K, N):
            cands["pw"] = lambda: ext.pw_gemm(x, w, 2048)
        res = {k: [] for k in cands}
        for _ in range(a.rounds):
            for k, fn in cands.items():
                if k == "gemm":
                    res[k].append(min(timeit(lambda c=c: ext.gemm(x, b, nn, cfg=c), a.iters) for c in range(3)))
                elif fn is not None:
                    res[k].append(timeit(fn, a.iters))
        med = {k: (statistics.median(v) if v else float("nan")) for k, v in res.items()}
        today = min(med[k] for k in ("lib", "gemm", "pw") if res[k])
        ours = min(med["g256"], med["g128"])
        print(f"{name:14s} {M:6d} {N:5d} {K:5d} {roof:6.1f} " +
              " ".join(f"{med[k]:7.1f}" for k in ("lib", "gemm", "pw", "g256", "g128")) +
              f"  {today / ours:.2f}x", flush=True)
    fused_project(ext, a.iters, a.rounds)


def fused_project(ext, iters, rounds):
    """Project conv of blocks 19-25: bn_apply + GEMM + bn_stats (library), gemm.hip with the prologue + statistics,
    and gemm256 with the same fusions."""
    for name, M, N, K in [("proj19", 76800, 232, 1392), ("proj24", 76800, 384, 1392), ("proj25", 76800, 384, 2304)]:
        hw = 100
        y = torch.randn(M, K, device="cuda").to(BF)
        sc, sh = torch.rand(K, device="cuda") + 0.5, torch.randn(K, device="cuda") * 0.3
        gate = torch.rand(M // hw, K, device="cuda")
        w = (torch.randn(N, K, device="cuda") * 0.05).to(BF)

        def lib():
            a = ext.bn_apply(y, sc, sh, 1, gate, hw)
            c = torch.mm(a, w.t())
            ext.bn_stats(c, 512)
        cands = {"lib": lib,
                 "gemm": lambda: ext.gemm(y, w, False, None, sc, sh, gate, hw, stats=True, cfg=1, store_a=True),
                 "g256": lambda: ext.gemm256(y, w, False, None, sc, sh, gate, hw, stats=True, store_a=True, bn=256),
                 "g128": lambda: ext.gemm256(y, w, False, None, sc, sh, gate, hw, stats=True, store_a=True, bn=128)}
        res = {k: [] for k in cands}
        for _ in range(rounds):
            for k, fn in cands.items():
                res[k].append(timeit(fn, iters))
        med = {k: statistics.median(v) for k, v in res.items()}
        print(f"{name} prologue+stats+store_a: " + " ".join(f"{k} {v:.1f}" for k, v in med.items()) +
              f"  -> {min(med['lib'], med['gemm']) / min(med['g256'], med['g128']):.2f}x", flush=True)


if __name__ == "__main__":
    main()
