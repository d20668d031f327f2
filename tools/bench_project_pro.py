#!/usr/bin/env python3
"""Project-conv operand prologue (pw_gemm with scale/shift/gate, ops/backbone.py project_fused) vs bn_apply + pw_gemm,
at the real RT-1 shapes of the skinny-GEMM blocks, forward (GEMM + BN3 stats) and backward weight gradient
(wgrad with the same prologue vs wgrad on the materialised A).

  python tools/bench_project_pro.py [--frames 768] [--res 300]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_rt1_for_distributed_training_amd.models.efficientnet import block_specs, conv_out_size  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.ops import backbone, load  # noqa: E402

BF = torch.bfloat16


def timeit(fn, iters=10):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=768)
    ap.add_argument("--res", type=int, default=300)
    a = ap.parse_args()
    ext = load()
    N = a.frames
    H = W = conv_out_size(a.res, 3, 2)
    print(f"{'blk':>3} {'Ce':>5} {'Cout':>4} {'HxW':>9} | {'fwd unf':>8} {'fwd pro':>8} {'pro+st':>8} | {'wg unf':>8} "
          f"{'wg pro':>8}")
    tu = tp = 0.0
    fs_tot = [0.0]
    for sp in block_specs():
        Ce, Cout = sp.expand_ch, sp.out_ch
        H2, W2 = conv_out_size(H, sp.kernel, sp.stride), conv_out_size(W, sp.kernel, sp.stride)
        H, W = H2, W2
        if not ext.pw_gemm_supported(Ce, Cout):
            continue
        hw = H2 * W2
        M2 = N * hw
        y2 = torch.randn(M2, Ce, device="cuda").to(BF)
        wp = (torch.randn(Cout, Ce, device="cuda") * 0.1).to(BF)
        sc, sh = torch.rand(Ce, device="cuda") + 0.5, torch.randn(Ce, device="cuda") * 0.2
        gate = torch.rand(N, Ce, device="cuda")
        dy3 = torch.randn(M2, Cout, device="cuda").to(BF)
        A = ext.bn_apply(y2, sc, sh, 1, gate, hw)
        f_u = timeit(lambda: ext.pw_gemm(ext.bn_apply(y2, sc, sh, 1, gate, hw), wp, 2048, True))
        f_p = timeit(lambda: ext.pw_gemm(y2, wp, 2048, True, sc, sh, gate, hw))
        f_s = timeit(lambda: ext.pw_gemm(y2, wp, 2048, True, sc, sh, gate, hw, True))
        w_u = timeit(lambda: backbone.wgrad(dy3, A))
        w_p = timeit(lambda: backbone.wgrad(dy3, y2, prologue=(sc, sh, gate, 1, hw)))
        fs_tot[0] += f_s + w_u
        tu += f_u + w_u
        tp += f_p + w_p
        print(f"{sp.index:>3} {Ce:>5} {Cout:>4} {H2:>4}x{W2:<4} | {f_u:8.1f} {f_p:8.1f} {f_s:8.1f} | {w_u:8.1f} "
              f"{w_p:8.1f}", flush=True)
        del y2, dy3, A
        torch.cuda.empty_cache()
    print(f"total (fwd + wgrad): unfused {tu / 1e3:.2f} ms, prologue in both {tp / 1e3:.2f} ms, "
          f"prologue + stored operand {fs_tot[0] / 1e3:.2f} ms")


if __name__ == "__main__":
    main()
