#!/usr/bin/env python3
"""Per-block time and effective bandwidth of the per-frame reductions (csrc/kernels/block.hip) at the real RT-1
shapes (768 frames at 300x300): frame_pool with BN + SiLU (the SE squeeze), the same without the activation and
without BN (what the loads alone cost), se_bn_bwd_reduce and tail_bwd_reduce -- to tell VALU-bound from
load-latency-bound.

  python tools/bench_frame.py [--frames 768] [--res 300] [--blocks 6,14,19]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_rt1_for_distributed_training_amd.models.efficientnet import block_specs, conv_out_size  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.ops import load  # noqa: E402
from tools.bench_dw_phases import timeit  # noqa: E402

BF = torch.bfloat16
ACT_NONE, ACT_SILU = 0, 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=768)
    ap.add_argument("--res", type=int, default=300)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--blocks", default="")
    a = ap.parse_args()
    ext = load()
    N = a.frames
    H = W = conv_out_size(a.res, 3, 2)
    sel = {int(b) for b in a.blocks.split(",") if b}
    tot = [0.0] * 5
    print(f"{'blk':>3} {'C':>5} {'Co':>4} {'HW':>6} | {'pool':>7} {'pool_id':>7} {'pool_raw':>8} {'se_bn':>7} "
          f"{'tail':>7} | TB/s: {'pool':>5} {'raw':>5} {'se_bn':>5} {'tail':>5}")
    for sp in block_specs():
        C, Co, k, s = sp.expand_ch, sp.out_ch, sp.kernel, sp.stride
        H2, W2 = conv_out_size(H, k, s), conv_out_size(W, k, s)
        H, W = H2, W2
        if sel and sp.index not in sel:
            continue
        HW = H2 * W2
        dev = "cuda"
        y = torch.randn(N, HW, C, device=dev).to(BF)
        g = torch.randn(N, HW, C, device=dev).to(BF)
        v = lambda c: torch.rand(c, device=dev) + 0.5
        sc, sh, mu, rs = v(C), v(C), v(C), v(C)
        d3 = torch.randn(N, HW, Co, device=dev).to(BF)
        y3 = torch.randn(N, HW, Co, device=dev).to(BF)
        s3, h3, m3, r3 = v(Co), v(Co), v(Co), v(Co)
        fm = torch.rand(N, Co, device=dev)
        fns = [lambda: ext.frame_pool(y, None, sc, sh, ACT_SILU), lambda: ext.frame_pool(y, None, sc, sh, ACT_NONE),
               lambda: ext.frame_pool(y, None, None, None, ACT_NONE),
               lambda: ext.se_bn_bwd_reduce(g, y, sc, sh, mu, rs),
               lambda: ext.tail_bwd_reduce(d3, y3, s3, h3, m3, r3, None, None, fm)]
        t = [timeit(f, a.iters) for f in fns]
        for i in range(5):
            tot[i] += t[i]
        by = y.numel() * 2
        bw = lambda nbytes, us: nbytes / us / 1e6
        print(f"{sp.index:>3} {C:>5} {Co:>4} {HW:>6} | {t[0]:7.1f} {t[1]:7.1f} {t[2]:8.1f} {t[3]:7.1f} {t[4]:7.1f} | "
              f"      {bw(by, t[0]):5.2f} {bw(by, t[2]):5.2f} {bw(2 * by, t[3]):5.2f} {bw(2 * d3.numel() * 2, t[4]):5.2f}",
              flush=True)
        del y, g, d3, y3
        torch.cuda.empty_cache()
    print("total ms: pool %.3f  pool_id %.3f  pool_raw %.3f  se_bn %.3f  tail %.3f" % tuple(x / 1e3 for x in tot))


if __name__ == "__main__":
    main()
