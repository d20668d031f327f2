#!/usr/bin/env python3
"""The stem kernels alone at the bench shape (768 frames of 300x300 uint8, random shift): stem_fwd (MFMA conv + BN
partials) and stem_bwd_weight with the stem-BN backward prologue (block 0's StemLink), and their HBM rates.

  python tools/bench_stem.py [--frames 768] [--res 300]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_rt1_for_distributed_training_amd.ops import backbone, load  # noqa: E402
from tools.bench_dw_phases import timeit  # noqa: E402

BF = torch.bfloat16


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=768)
    ap.add_argument("--res", type=int, default=300)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    ext = load()
    N, H = a.frames, a.res
    Ho = (H - 1) // 2 + 1
    dev = "cuda"
    img = torch.randint(0, 256, (N, 3, H, H), device=dev, dtype=torch.uint8)
    w = torch.randn(40, 27, device=dev) * 0.3
    sh = torch.tensor([3, -5], dtype=torch.int32, device=dev)
    mb = backbone.MAX_BLOCKS
    t = timeit(lambda: ext.stem_fwd(img, sh, w, mb), a.iters)
    by = img.numel() + N * Ho * Ho * 40 * 2
    print(f"stem_fwd         {t:8.1f} us  {by / t / 1e6:5.2f} TB/s", flush=True)
    g = torch.randn(N, Ho, Ho, 40, device=dev).to(BF)
    x = torch.randn(N, Ho, Ho, 40, device=dev).to(BF)
    c = [torch.rand(40, device=dev) + 0.5 for _ in range(5)] + [torch.rand(40, device=dev) * 0.01 for _ in range(2)]
    t = timeit(lambda: ext.stem_bwd_weight(img, sh, g, mb, x, *c), a.iters)
    by = img.numel() + 2 * g.numel() * 2
    print(f"stem_bwd_weight  {t:8.1f} us  {by / t / 1e6:5.2f} TB/s  (BN-backward prologue)", flush=True)


if __name__ == "__main__":
    main()
