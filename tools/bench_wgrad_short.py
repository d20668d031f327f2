#!/usr/bin/env python3
"""Short-reduction weight gradients (the transformer's dW = dy^T x over T = B x S tokens, 8448 rows at b128): every
tile variant x row-split count of csrc/kernels/wgrad.hip (split partial sum included) against the library TN GEMM
with fp32 output, median us.

  python tools/bench_wgrad_short.py [--rows 8448]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_rt1_for_distributed_training_amd.ops import load  # noqa: E402
from tools.bench_dw_phases import timeit  # noqa: E402

SHAPES = [(3072, 512), (512, 1024), (512, 512), (1024, 512)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=8448)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    ext = load()
    M = a.rows
    for Co, Ci in SHAPES:
        dy = torch.randn(M, Co, device="cuda").to(torch.bfloat16)
        x = torch.randn(M, Ci, device="cuda").to(torch.bfloat16)
        ref = dy.float().t() @ x.float()
        lib = timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32), a.iters)
        auto = timeit(lambda: ext.wgrad(dy, x), a.iters)
        rows = []
        for v in range(6):
            for s in (1, 2, 3, 4, 6, 8, 12, 16):
                out = ext.wgrad(dy, x, variant=v, splits=s)
                err = float((out - ref).norm() / ref.norm())
                assert err < 1e-2, (Co, Ci, v, s, err)
                rows.append((timeit(lambda: ext.wgrad(dy, x, variant=v, splits=s), a.iters), v, s))
        rows.sort()
        best = " ".join(f"v{v}/s{s}:{t:.1f}" for t, v, s in rows[:5])
        print(f"Co={Co:5d} Ci={Ci:5d} M={M}: lib {lib:7.1f}  auto {auto:7.1f}  best {best}", flush=True)


if __name__ == "__main__":
    main()
