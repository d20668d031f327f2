#!/usr/bin/env python3
"""Split-K partial sums of the step's weight gradients: one colsum launch per gradient (reduce.hip colsum, the old
path) against the gather's multi_reduce_copy over all of them in one launch (parallel/flat.py deferred_sums), and
the achieved read bandwidth of each.

  python tools/bench_reduce.py
"""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_rt1_for_distributed_training_amd import ops  # noqa: E402
from tools.bench_tf_gemms import timeit  # noqa: E402

# (splits, Co, Ci, count): the transformer's Q/K/V, out, FF and embedding gradients at b128 and a few encoder ones
SHAPES = [(8, 3072, 512, 8), (12, 512, 1024, 8), (12, 512, 512, 9), (256, 144, 24, 2), (16, 1392, 232, 4),
          (64, 816, 136, 4), (24, 384, 1536, 2)]


def main():
    ext = ops.load()
    parts, dsts = [], []
    for S, Co, Ci, cnt in SHAPES:
        for _ in range(cnt):
            parts.append(torch.randn(S, Co, Ci, device="cuda"))
            dsts.append(torch.empty(Co, Ci, device="cuda"))
    nbytes = sum(p.numel() * 4 for p in parts)
    one = lambda: [ext.colsum(p) for p in parts]
    multi = lambda: ext.multi_reduce_copy_(dsts, [p[0] for p in parts], [p.shape[0] for p in parts],
                                           [p[0].numel() for p in parts])
    for name, fn in (("colsum each", one), ("multi_reduce", multi), ("colsum each", one), ("multi_reduce", multi)):
        us = timeit(fn, 20)
        print(f"{name:14s} {us:8.1f} us  {nbytes / us / 1e6:6.2f} TB/s over {nbytes / 1e6:.0f} MB of partials",
              flush=True)
    for S, Co, Ci, _ in SHAPES:
        p = torch.randn(S, Co, Ci, device="cuda")
        d = torch.empty(Co, Ci, device="cuda")
        t1 = timeit(lambda: ext.colsum(p), 50)
        t2 = timeit(lambda: ext.multi_reduce_copy_([d], [p[0]], [S], [p[0].numel()]), 50)
        mb = p.numel() * 4 / 1e6
        print(f"S={S:4d} [{Co:5d},{Ci:5d}] {mb:7.1f} MB: colsum {t1:7.1f} us ({mb / t1:5.2f} TB/s)  "
              f"multi_reduce {t2:7.1f} us ({mb / t2:5.2f} TB/s)", flush=True)


if __name__ == "__main__":
    main()
