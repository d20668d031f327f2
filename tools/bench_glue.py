#!/usr/bin/env python3
"""Per-block time and effective bandwidth of the flat elementwise glue passes (csrc/kernels/block.hip block_tail,
csrc/kernels/bn.hip bn_apply / bn_bwd_apply) at the real RT-1 shapes (768 frames at 300x300): the block tail
(BN3 + drop-path + residual + FiLM), the BN2 + SiLU + SE-gate apply of the project operand and the BN3 backward apply
with the FiLM row multiplier and drop-path keep.  ``RT1_HIP_SO`` selects another build for an A/B.

  python tools/bench_glue.py [--frames 768] [--res 300] [--blocks 8,14,19]
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
    tot = [0.0] * 3
    print(f"{'blk':>3} {'Ce':>5} {'Co':>4} {'HW':>6} | {'tail':>7} {'apply':>7} {'bwdapp':>7} | TB/s: {'tail':>5} "
          f"{'apply':>5} {'bwdapp':>6}")
    for sp in block_specs():
        C, Co, k, s = sp.expand_ch, sp.out_ch, sp.kernel, sp.stride
        H2, W2 = conv_out_size(H, k, s), conv_out_size(W, k, s)
        H, W = H2, W2
        if sel and sp.index not in sel:
            continue
        HW = H2 * W2
        dev = "cuda"
        v = lambda c: torch.rand(c, device=dev) + 0.5
        y3 = torch.randn(N, HW, Co, device=dev).to(BF)
        skip = torch.randn(N, HW, Co, device=dev).to(BF) if sp.has_skip else None
        keep = (torch.rand(N, device=dev) > 0.1).float() if sp.has_skip else None
        fm, fa = torch.rand(N, Co, device=dev), torch.rand(N, Co, device=dev)
        s3, h3, m3, r3, g3 = v(Co), v(Co), v(Co), v(Co), v(Co)
        y2 = torch.randn(N, H2, W2, C, device=dev).to(BF)
        s2, h2 = v(C), v(C)
        gate = torch.rand(N, C, device=dev)
        dout = torch.randn(N * HW, Co, device=dev).to(BF)
        fns = [lambda: ext.block_tail(y3, s3, h3, keep, skip, fm, fa),
               lambda: ext.bn_apply(y2, s2, h2, ACT_SILU, gate, HW),
               lambda: ext.bn_bwd_apply(dout, fm, None, HW, y3.view(N * HW, Co), s3, h3, m3, r3, g3, ACT_NONE, m3, r3,
                                        keep)]
        t = [timeit(f, a.iters) for f in fns]
        for i in range(3):
            tot[i] += t[i]
        b3 = y3.numel() * 2
        bw = lambda nbytes, us: nbytes / us / 1e6
        print(f"{sp.index:>3} {C:>5} {Co:>4} {HW:>6} | {t[0]:7.1f} {t[1]:7.1f} {t[2]:7.1f} | "
              f"      {bw(b3 * (3 if skip is not None else 2), t[0]):5.2f} {bw(y2.numel() * 4, t[1]):5.2f} "
              f"{bw(b3 * 3, t[2]):6.2f}", flush=True)
        del y3, skip, y2, dout
        torch.cuda.empty_cache()
    print("total ms: tail %.3f  apply %.3f  bwd_apply %.3f" % tuple(x / 1e3 for x in tot))


if __name__ == "__main__":
    main()
