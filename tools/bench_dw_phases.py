#!/usr/bin/env python3
"""Per-block time of the depthwise forward (dw_fwd) and the unified backward (dw_bwd_fused, variant 1) at the real
RT-1 shapes (768 frames at 300x300), for the phase split of the depthwise category: run it once per timing-only
build of the extension (build.py --variant <name> -D RT1_DW_TIMING=<mask>, loaded with RT1_HIP_SO=<.so>) and compare.

  python tools/bench_dw_phases.py [--frames 768] [--res 300] [--blocks 6,14,19] [--tag base]

Timing builds (csrc/kernels/dwconv.hip, RT1_DW_TIMING bit mask):
  2   no LDS staging of the input / dy tile (the tile holds stale data)
  4   no K x K tap loop (data and weight products)
  16  backward: no strip-centre x1 loads / BN1 + SiLU recompute
  8   no per-output epilogue (stores, BN statistics)
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_rt1_for_distributed_training_amd.models.efficientnet import block_specs, conv_out_size  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.ops import load  # noqa: E402

BF = torch.bfloat16


def timeit(fn, iters):
    for _ in range(2):
        fn()
    ts = []
    for _ in range(iters):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=768)
    ap.add_argument("--res", type=int, default=300)
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--blocks", default="")
    ap.add_argument("--tag", default=os.environ.get("RT1_HIP_SO", "default"))
    ap.add_argument("--fwd_only", action="store_true")
    a = ap.parse_args()
    ext = load()
    N = a.frames
    H = W = conv_out_size(a.res, 3, 2)
    sel = {int(b) for b in a.blocks.split(",") if b}
    tot_f = tot_b = 0.0
    print(f"[{a.tag}]")
    print(f"{'blk':>3} {'C':>5} {'k':>2} {'HxW':>7} | {'fwd us':>8} | {'bwd us':>8}")
    for sp in block_specs():
        C, k, s = sp.expand_ch, sp.kernel, sp.stride
        Ho, Wo = conv_out_size(H, k, s), conv_out_size(W, k, s)
        if s != 1 or (sel and sp.index not in sel):
            H, W = Ho, Wo
            continue
        dev = "cuda"
        expand = sp.expand_ch != sp.in_ch
        dA = torch.randn(N, Ho, Wo, C, device=dev).to(BF)
        y2 = torch.randn(N, Ho, Wo, C, device=dev).to(BF)
        x1 = torch.randn(N, H, W, C, device=dev).to(BF)
        gate, rb = torch.rand(N, C, device=dev), torch.randn(N, C, device=dev) * 1e-3
        v = lambda: torch.rand(C, device=dev) + 0.5
        sc2, sh2, mu2, rs2, g2, mdz, mdzx = v(), v(), v(), v(), v(), v() * 0.01, v() * 0.01
        sc1, sh1, mu1, rs1 = (v(), v(), v(), v()) if expand else (None, None, None, None)
        act = 1 if expand else 0
        w = torch.randn(C, k * k, device=dev) * 0.2
        fwd = lambda: ext.dw_fwd(x1, w, sc1, sh1, act, k, s, 2048)
        bwd = lambda: ext.dw_bwd_fused(dA, y2, gate, rb, sc2, sh2, mu2, rs2, g2, mdz, mdzx, w, k, x1, sc1, sh1, act,
                                       mu1, rs1, 2048, 1)
        tf, tb = timeit(fwd, a.iters), (0.0 if a.fwd_only else timeit(bwd, a.iters))
        tot_f += tf
        tot_b += tb
        print(f"{sp.index:>3} {C:>5} {k:>2} {H:>3}x{W:<3} | {tf:8.1f} | {tb:8.1f}", flush=True)
        H, W = Ho, Wo
        del dA, y2, x1
        torch.cuda.empty_cache()
    print(f"total stride-1: fwd {tot_f / 1e3:.3f} ms, bwd {tot_b / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
