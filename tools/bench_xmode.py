#!/usr/bin/env python3
"""Block 2's x-mode depthwise kernels alone at the real shape (768 frames, 150x150 x 24 -> expand 144, k3 stride 2):
the forward (y1 recomputed on MFMA + BN1 + SiLU staging, dw_fwd_x) and the unified backward (dw_bwd_fused_x), against
the stored-y1 kernels they replace.  Run under rocprofv3 --pmc for counters of one kernel at a time.

  python tools/bench_xmode.py [--frames 768] [--iters 10] [--only fwd|bwd]
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
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="")
    ap.add_argument("--stored", action="store_true", help="also time the stored-y1 kernels")
    ap.add_argument("--blocks", default="", help="ignored (tools/gpu/pmc_dw.sh passes it)")
    a = ap.parse_args()
    ext = load()
    N, H, W, Cin, Ce, k, s = a.frames, 150, 150, 24, 144, 3, 2
    Ho, Wo = 75, 75
    dev = "cuda"
    x = (torch.randn(N, H, W, Cin, device=dev) + 0.3).to(BF)
    we = (torch.randn(Ce, Cin, device=dev) * Cin ** -0.5).to(BF)
    w = torch.randn(Ce, k * k, device=dev) * 0.3
    v = lambda: torch.rand(Ce, device=dev) + 0.5
    sc1, sh1, mu1, rs1 = v(), v() * 0.2, v() * 0.1, v()
    mb = backbone.MAX_BLOCKS
    if a.only in ("", "fwd"):
        t = timeit(lambda: ext.dw_fwd_x(x, we, w, sc1, sh1, k, s, mb), a.iters)
        print(f"dw_fwd_x        {t:8.1f} us  (in 150x150x{Ce} recomputed, out {Ho}x{Wo}x{Ce})", flush=True)
    if a.only in ("", "bwd"):
        dA = torch.randn(N, Ho, Wo, Ce, device=dev).to(BF)
        y2 = (torch.randn(N, Ho, Wo, Ce, device=dev) * 1.5).to(BF)
        gate, rb = torch.rand(N, Ce, device=dev), torch.randn(N, Ce, device=dev) * 0.1
        sc2, sh2, mu2, rs2, g2 = v(), v() * 0.2, v() * 0.1, v(), v()
        mdz2, mdzx2 = v() * 0.05, v() * 0.05
        t = timeit(lambda: ext.dw_bwd_fused_x(dA, y2, gate, rb, sc2, sh2, mu2, rs2, g2, mdz2, mdzx2, w, k, x, we, sc1,
                                              sh1, mu1, rs1, mb, True), a.iters)
        print(f"dw_bwd_fused_x  {t:8.1f} us", flush=True)
    if a.stored:
        y1 = (x.view(-1, Cin) @ we.t()).view(N, H, W, Ce)
        t = timeit(lambda: ext.dw_fwd(y1, w, sc1, sh1, 1, k, s, mb), a.iters)
        print(f"dw_fwd (y1)     {t:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
