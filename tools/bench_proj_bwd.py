#!/usr/bin/env python3
"""Project-conv backward of the skinny blocks (0-7) at 768 frames: projbwd.hip (ext.proj_bwd: SE/BN2 sums + dWp from
(dy3, y2) per frame) vs the previous pair wgrad(dy3, A) + se_bn_bwd_reduce(dA, y2), median us and the compulsory-byte
rate of the new kernel.

  python tools/bench_proj_bwd.py [--frames 768 --res 300]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_rt1_for_distributed_training_amd.models.efficientnet import block_specs, conv_out_size  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.ops import backbone, load  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=768)
    ap.add_argument("--res", type=int, default=300)
    a = ap.parse_args()
    ext = load()
    N = a.frames
    H = W = conv_out_size(a.res, 3, 2)
    print(f"{'blk':>4} {'Cout':>5} {'Ce':>5} {'HxW':>8} | {'old us':>8} {'new us':>8} {'new GB/s':>9}")
    tot_o = tot_n = 0.0
    for sp in block_specs():
        Ho, Wo = conv_out_size(H, sp.kernel, sp.stride), conv_out_size(W, sp.kernel, sp.stride)
        H, W = Ho, Wo
        Ce, Cout, HW = sp.expand_ch, sp.out_ch, Ho * Wo
        if not ext.proj_bwd_supported(Cout, Ce) or not backbone.project_fused(Ce, Cout, HW):
            continue
        M = N * HW
        dy3 = (torch.randn(M, Cout, device="cuda") * 0.1).to(torch.bfloat16)
        y2 = torch.randn(M, Ce, device="cuda").to(torch.bfloat16)
        A = torch.randn(M, Ce, device="cuda").to(torch.bfloat16)
        dA = torch.randn(M, Ce, device="cuda").to(torch.bfloat16)
        Wp = (torch.randn(Cout, Ce, device="cuda") * 0.1).to(torch.bfloat16)
        gate = torch.rand(N, Ce, device="cuda")
        sc, sh, mu, rs = (torch.rand(Ce, device="cuda") + 0.5 for _ in range(4))
        t_old = timeit(lambda: (backbone.wgrad(dy3, A), ext.se_bn_bwd_reduce(dA.view(N, HW, Ce), y2.view(N, HW, Ce),
                                                                             sc, sh, mu, rs)))
        t_new = timeit(lambda: ext.proj_bwd(dy3, y2.view(N, HW, Ce), Wp, gate, sc, sh, mu, rs))
        gbs = M * (Ce + Cout) * 2 / t_new / 1e3
        tot_o += t_old
        tot_n += t_new
        print(f"{sp.index:>4} {Cout:>5} {Ce:>5} {Ho:>4}x{Wo:<3} | {t_old:8.1f} {t_new:8.1f} {gbs:9.0f}", flush=True)
        del dy3, y2, A, dA
        torch.cuda.empty_cache()
    print(f"total: old {tot_o / 1e3:.2f} ms (+ the forward's operand store), new {tot_n / 1e3:.2f} ms")


if __name__ == "__main__":
    main()
