#!/usr/bin/env python3
"""Time csrc/kernels/gemm.hip against torch.mm (hipBLASLt) on the step's library-GEMM shapes (same box, same inputs).

  python tools/bench_gemm_mfma.py [--iters 50]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_rt1_for_distributed_training_amd import ops  # noqa: E402

BF = torch.bfloat16
# (name, M, N, K, nn): forward products (NT, C = A W^T) and data gradients (NN, C = dY W)
SHAPES = [
    ("qkv fwd", 8448, 3072, 512, False), ("out fwd", 8448, 512, 1024, False), ("ff fwd", 8448, 512, 512, False),
    ("qkv dgrad", 8448, 512, 3072, True), ("out dgrad", 8448, 1024, 512, True), ("ff dgrad", 8448, 512, 512, True),
    ("proj19 fwd", 76800, 232, 1392, False), ("proj25 fwd", 76800, 384, 2304, False),
    ("proj18 fwd", 76800, 232, 816, False), ("conv1x1 fwd", 76800, 512, 1536, False),
    ("top fwd", 76800, 1536, 384, False), ("proj19 dgrad", 76800, 1392, 232, True),
    ("proj25 dgrad", 76800, 2304, 384, True), ("conv1x1 dgrad", 76800, 1536, 512, True),
    ("top dgrad", 76800, 384, 1536, True),
    ("exp19 dgrad", 76800, 232, 1392, True), ("exp25 dgrad", 76800, 384, 2304, True),
    ("exp18 dgrad", 76800, 136, 816, True),
]


def timeit(fn, iters):
    for _ in range(3):
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
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    ext = ops.load()
    print(f"{'shape':14s} {'M':>6s} {'N':>5s} {'K':>5s}  {'roof us':>8s} {'lib us':>8s} " +
          " ".join(f"cfg{c:d} us" for c in range(3)) + "  best")
    for name, M, N, K, nn in SHAPES:
        x = torch.randn(M, K, device="cuda").to(BF)
        w = (torch.randn(N, K, device="cuda") * 0.05).to(BF)
        b = w.t().contiguous() if nn else w
        roof = max((M * K + N * K + M * N) * 2 / 5.3e12, 2 * M * N * K / 2.3e15) * 1e6
        lib = timeit(lambda: torch.mm(x, b) if nn else torch.mm(x, w.t()), a.iters)
        ours = [timeit(lambda c=c: ext.gemm(x, b, nn, cfg=c), a.iters) for c in range(3)]
        best = min(range(3), key=lambda c: ours[c])
        print(f"{name:14s} {M:6d} {N:5d} {K:5d}  {roof:8.1f} {lib:8.1f} " + " ".join(f"{o:8.1f}" for o in ours) +
              f"  cfg{best} {lib / ours[best]:.2f}x", flush=True)
    fused_project(ext, a.iters)


def fused_project(ext, iters):
    """Project conv of blocks 19-23 / 25: the library path (bn_apply builds A = silu(bn2(y2)) * gate, GEMM, bn_stats of
    the output) against one gemm.hip launch with the operand prologue and the statistics epilogue."""
    for name, M, N, K in [("proj19", 76800, 232, 1392), ("proj25", 76800, 384, 2304), ("proj18", 76800, 232, 816)]:
        hw = 100 if M == 76800 else 361
        y = torch.randn(M, K, device="cuda").to(BF)
        sc, sh = torch.rand(K, device="cuda") + 0.5, torch.randn(K, device="cuda") * 0.3
        gate = torch.rand(M // hw, K, device="cuda")
        w = (torch.randn(N, K, device="cuda") * 0.05).to(BF)

        def lib():
            a = ext.bn_apply(y, sc, sh, 1, gate, hw)
            c = torch.mm(a, w.t())
            ext.bn_stats(c, 512)
        tl = timeit(lib, iters)
        ours = [timeit(lambda c=c: ext.gemm(y, w, False, None, sc, sh, gate, hw, stats=True, cfg=c), iters)
                for c in range(3)]
        best = min(range(3), key=lambda c: ours[c])
        print(f"{name} fused prologue+stats: library path {tl:.1f} us, gemm.hip " +
              " ".join(f"cfg{c} {o:.1f}" for c, o in enumerate(ours)) + f"  -> {tl / ours[best]:.2f}x", flush=True)


if __name__ == "__main__":
    main()
