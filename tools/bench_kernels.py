#!/usr/bin/env python3
"""Per-layer microbenchmark of the fused encoder kernels at the real RT-1 shapes.

For every MBConv block of FiLM-EfficientNet-B3 at the given frame count and
resolution, times (HIP events, median of --iters) the depthwise forward,
backward-data and backward-weight kernels and the BN/frame kernels, and
reports the effective HBM bandwidth (compulsory bytes / time).

  python tools/bench_kernels.py --frames 768 --res 300 [--only dw]
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
    ts = []
    for _ in range(3):
        fn()
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
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="")
    ap.add_argument("--blocks", default="", help="comma-separated block indices (default: all)")
    ap.add_argument("--wgrad_blocks", type=int, default=1024, help="max_blocks of the depthwise weight-grad grid")
    ap.add_argument("--fwd_blocks", type=int, default=2048, help="max_blocks of the depthwise fwd / bwd-data grids")
    a = ap.parse_args()
    ext = load()
    N = a.frames
    H = W = conv_out_size(a.res, 3, 2)
    tot = {"fwd": 0.0, "bwd_data": 0.0, "bwd_w": 0.0, "bn_bwd_apply": 0.0, "bn_apply": 0.0, "bn_stats": 0.0, "frame_pool": 0.0, "se_bn_red": 0.0}
    print(f"{'blk':>3} {'C':>5} {'k':>2} {'s':>2} {'HxW':>9} | {'fwd us':>8} {'GB/s':>6} | {'bwdD us':>8} {'GB/s':>6} |"
          f" {'bwdW us':>8} {'GB/s':>6} | {'bnBwdAp':>8} {'GB/s':>6} | {'bnFwdAp':>8} {'GB/s':>6} | {'bnStat':>7} {'GB/s':>6} | {'seRed':>7} {'GB/s':>6}")
    sel = {int(b) for b in a.blocks.split(",") if b}
    for sp in block_specs():
        C, k, s = sp.expand_ch, sp.kernel, sp.stride
        Ho, Wo = conv_out_size(H, k, s), conv_out_size(W, k, s)
        if sel and sp.index not in sel:
            H, W = Ho, Wo
            continue
        x = torch.randn(N, H, W, C, device="cuda").to(BF)
        w = torch.randn(C, k * k, device="cuda") * 0.2
        sc = torch.rand(C, device="cuda") + 0.5
        sh = torch.randn(C, device="cuda") * 0.1
        mu = torch.zeros(C, device="cuda")
        rs = torch.ones(C, device="cuda")
        dy = torch.randn(N, Ho, Wo, C, device="cuda").to(BF)
        in_b, out_b = x.numel() * 2, dy.numel() * 2
        t_f = timeit(lambda: ext.dw_fwd(x, w, sc, sh, 1, k, s, a.fwd_blocks), a.iters)
        t_d = timeit(lambda: ext.dw_bwd_data(dy, w, H, W, k, s, x, sc, sh, mu, rs, a.fwd_blocks), a.iters)
        t_w = timeit(lambda: ext.dw_bwd_weight(dy, x, sc, sh, 1, k, s, a.wgrad_blocks), a.iters)
        gate = torch.rand(N, C, device="cuda")
        rb = torch.randn(N, C, device="cuda") * 1e-3
        y2 = dy
        t_a = timeit(lambda: ext.bn_bwd_apply(dy, gate, rb, Ho * Wo, y2, sc, sh, mu, rs, sc, 1, mu, mu), a.iters)
        t_p = timeit(lambda: ext.bn_apply(y2, sc, sh, 1, gate, Ho * Wo), a.iters)
        y2f = y2.view(-1, C)
        t_s = timeit(lambda: ext.bn_stats(y2f, int(max(1, min(1024, (y2f.shape[0] + 255) // 256)))), a.iters)
        t_r = timeit(lambda: ext.se_bn_bwd_reduce(dy.view(N, Ho * Wo, C), y2.view(N, Ho * Wo, C), sc, sh, mu, rs),
                     a.iters)
        tot["fwd"] += t_f
        tot["bwd_data"] += t_d
        tot["bwd_w"] += t_w
        tot["bn_bwd_apply"] += t_a
        tot["bn_apply"] += t_p
        tot["bn_stats"] += t_s
        tot["frame_pool"] += timeit(lambda: ext.frame_pool(y2.view(N, Ho * Wo, C), None, sc, sh, 1), a.iters)
        tot["se_bn_red"] += t_r
        gb = lambda b, t: b / t / 1e3
        print(f"{sp.index:>3} {C:>5} {k:>2} {s:>2} {H:>4}x{W:<4} | {t_f:8.1f} {gb(in_b + out_b, t_f):6.0f} | "
              f"{t_d:8.1f} {gb(2 * in_b + out_b, t_d):6.0f} | {t_w:8.1f} {gb(in_b + out_b, t_w):6.0f} | "
              f"{t_a:8.1f} {gb(3 * out_b, t_a):6.0f} | {t_p:8.1f} {gb(2 * out_b, t_p):6.0f} | {t_s:7.1f} {gb(out_b, t_s):6.0f} | {t_r:7.1f} {gb(2 * out_b, t_r):6.0f}", flush=True)
        H, W = Ho, Wo
        del x, dy
        torch.cuda.empty_cache()
    print("totals (ms):", {k: round(v / 1e3, 2) for k, v in tot.items()})


if __name__ == "__main__":
    main()
