#!/usr/bin/env python3
"""Per-layer timing of the encoder's 1x1-conv GEMMs (hipBLASLt through torch) at the real RT-1 shapes,
against the HBM / MFMA roofline of each shape.

For every MBConv expand/project conv of FiLM-EfficientNet-B3 at --frames x --res, times (HIP events,
median) the forward GEMM, the backward-data GEMM and the split-K weight-gradient GEMM exactly as
``ops/backbone.py`` issues them.

  python tools/bench_gemms.py --frames 768 --res 300 [--use-ext]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_rt1_for_distributed_training_amd.models.efficientnet import block_specs, conv_out_size  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.ops import backbone as bb  # noqa: E402

BF = torch.bfloat16
HBM = 5.5e12      # sustained bytes/s used for the roofline
MFMA = 2.3e15     # dense bf16 flop/s


def timeit(fn, iters):
    for _ in range(3):
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


def roof_us(M, K, N, out_bytes=2):
    return max(2 * M * K * N / MFMA, (2 * M * K + out_bytes * M * N) / HBM) * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=768)
    ap.add_argument("--res", type=int, default=300)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--use-ext", action="store_true", help="time the HIP GEMM path of ops.backbone when present")
    a = ap.parse_args()
    N = a.frames
    H = W = conv_out_size(a.res, 3, 2)
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0, "roof": 0.0}
    print(f"{'blk':>3} {'conv':>4} {'M':>9} {'K':>5} {'N':>5} | {'fwd us':>8} {'%roof':>5} | {'dgrad':>8} {'%roof':>5} |"
          f" {'wgrad':>8} {'%roof':>5}")
    for sp in block_specs():
        Ho, Wo = conv_out_size(H, sp.kernel, sp.stride), conv_out_size(W, sp.kernel, sp.stride)
        convs = []
        if sp.expand_ch != sp.in_ch:
            convs.append(("exp", N * H * W, sp.in_ch, sp.expand_ch))
        convs.append(("proj", N * Ho * Wo, sp.expand_ch, sp.out_ch))
        for name, M, K, Nn in convs:
            x = torch.randn(M, K, device="cuda").to(BF)
            w = (torch.randn(Nn, K, device="cuda") * 0.1).to(BF)
            dy = torch.randn(M, Nn, device="cuda").to(BF)
            wt = w.t()
            t_f = timeit(lambda: bb._mm(x, wt), a.iters)
            t_d = timeit(lambda: bb._mm(dy, w), a.iters)
            t_w = timeit(lambda: bb.wgrad(dy, x), a.iters)
            r_f, r_d = roof_us(M, K, Nn), roof_us(M, Nn, K)
            if a.use_ext:
                from pytorch_rt1_for_distributed_training_amd.ops import load
                ext = load()
                wT = w.t().contiguous()
                if ext.pw_gemm_supported(K, Nn):
                    t_f = min(t_f, timeit(lambda: ext.pw_gemm(x, w, 2048), a.iters))
                if ext.pw_gemm_supported(Nn, K):
                    t_d = min(t_d, timeit(lambda: ext.pw_gemm(dy, wT, 2048), a.iters))
            r_w = max(2 * M * K * Nn / MFMA, 2 * (M * K + M * Nn) / HBM) * 1e6
            tot["fwd"] += t_f
            tot["dgrad"] += t_d
            tot["wgrad"] += t_w
            tot["roof"] += r_f + r_d + r_w
            print(f"{sp.index:>3} {name:>4} {M:>9} {K:>5} {Nn:>5} | {t_f:8.1f} {100 * r_f / t_f:5.0f} | "
                  f"{t_d:8.1f} {100 * r_d / t_d:5.0f} | {t_w:8.1f} {100 * r_w / t_w:5.0f}", flush=True)
            del x, dy
        H, W = Ho, Wo
        torch.cuda.empty_cache()
    print("totals (ms):", {k: round(v / 1e3, 2) for k, v in tot.items()})


if __name__ == "__main__":
    main()
