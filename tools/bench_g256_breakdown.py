#!/usr/bin/env python3
"""Where a gemm256 tile's time goes: fixed per-tile cost (DMA prologue + epilogue) vs per-K-slab cost, from the time of
the same M x N output at K = 64 .. 768 (slope = per-slab, intercept = per-tile); and the project-GEMM prologue's cost
split (plain / +PRO / +stats / +store_a) on gemm.hip and gemm256.

  python tools/bench_g256_breakdown.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_rt1_for_distributed_training_amd import ops  # noqa: E402
from tools.bench_gemm256 import timeit  # noqa: E402

BF = torch.bfloat16


def main():
    ext = ops.load()
    M, N = 76800, 2304
    for bn in (256, 128):
        tiles = ((M + 255) // 256) * ((N + bn - 1) // bn)
        rounds = tiles / 256
        row = []
        for K in (64, 128, 256, 384, 768):
            x = torch.randn(M, K, device="cuda").to(BF)
            w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(BF)
            us = min(timeit(lambda: ext.gemm256(x, w, False, bn=bn), 20) for _ in range(3))
            row.append((K, us, us / rounds))
        print(f"bn={bn} tiles={tiles} (x{rounds:.1f} per CU): " +
              "  ".join(f"K={k}: {us:.1f} us ({pt:.2f} us/tile)" for k, us, pt in row), flush=True)
    K, N, hw = 1392, 232, 100
    y = torch.randn(M, K, device="cuda").to(BF)
    sc, sh = torch.rand(K, device="cuda") + 0.5, torch.randn(K, device="cuda") * 0.3
    gate = torch.rand(M // hw, K, device="cuda")
    w = (torch.randn(N, K, device="cuda") * 0.05).to(BF)
    for name, fn in [
        ("gemm plain", lambda: ext.gemm(y, w, False, cfg=1)),
        ("gemm PRO", lambda: ext.gemm(y, w, False, None, sc, sh, gate, hw, cfg=1)),
        ("gemm PRO+stats", lambda: ext.gemm(y, w, False, None, sc, sh, gate, hw, stats=True, cfg=1)),
        ("gemm PRO+stats+store_a", lambda: ext.gemm(y, w, False, None, sc, sh, gate, hw, stats=True, cfg=1, store_a=True)),
        ("g256 plain", lambda: ext.gemm256(y, w, False)),
        ("g256 PRO", lambda: ext.gemm256(y, w, False, None, sc, sh, gate, hw)),
        ("g256 PRO+stats", lambda: ext.gemm256(y, w, False, None, sc, sh, gate, hw, stats=True)),
        ("g256 PRO+stats+store_a", lambda: ext.gemm256(y, w, False, None, sc, sh, gate, hw, stats=True, store_a=True)),
        ("bn_apply", lambda: ext.bn_apply(y, sc, sh, 1, gate, hw)),
    ]:
        print(f"proj19 {name:24s} {min(timeit(fn, 20) for _ in range(3)):7.1f} us", flush=True)


if __name__ == "__main__":
    main()
