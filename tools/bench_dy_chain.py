#!/usr/bin/env python3
"""Per-block time of the project-dgrad -> SE / BN2 backward sums -> depthwise backward chain of the wide blocks
(the ones without projbwd), staging path vs the dy-ready two-GEMM path, at the real RT-1 shapes (768 frames at
300x300):

  staging : dA = dY3 @ Wp (the backbone's dgrad) -> se_bn_bwd_reduce(dA, y2) -> dw_bwd_fused (BN2 backward in staging)
  dy-ready: gemm_se SE_RED (sums, dA never stored) -> gemm_se SE_BWD (dy2 stored) -> dw_bwd_fused(dy_ready=True)
            (the gemm_se columns are the best of the four tile configurations, listed per shape at the end)

The projbwd blocks (0-7) are listed too: pw_gemm dA + staging vs pw_gemm_bn2bwd dy2 + copy staging.

  python tools/bench_dy_chain.py [--frames 768] [--res 300] [--blocks 9,14,19]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_rt1_for_distributed_training_amd.models.efficientnet import block_specs, conv_out_size  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.ops import backbone, load  # noqa: E402
from tools.bench_dw_phases import timeit  # noqa: E402

BF = torch.bfloat16


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=768)
    ap.add_argument("--res", type=int, default=300)
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--blocks", default="")
    a = ap.parse_args()
    ext = load()
    N = a.frames
    H = W = conv_out_size(a.res, 3, 2)
    sel = {int(b) for b in a.blocks.split(",") if b}
    tot_old = tot_new = 0.0
    best_red, best_bwd = {}, {}
    print(f"{'blk':>3} {'Ce':>5} {'Co':>4} {'k':>2} {'s':>2} {'H2xW2':>7} | {'dgrad':>7} {'reduce':>7} {'dw':>7} "
          f"{'old':>7} | {'se_red':>7} {'se_bwd':>7} {'dw_rdy':>7} {'new':>7} | {'gain':>6}")
    for sp in block_specs():
        Ce, Co, k, s = sp.expand_ch, sp.out_ch, sp.kernel, sp.stride
        H2, W2 = conv_out_size(H, k, s), conv_out_size(W, k, s)
        HW2 = H2 * W2
        xmode = sp.expand_ch != sp.in_ch and backbone.x_mode_preferred(sp.in_ch, Ce, k, s, H2, W2)
        pbf = backbone.proj_bwd_fused(Ce, Co, HW2)
        skip = (sel and sp.index not in sel) or xmode or not backbone._dw_copy_staging(k, H2, W2, s, False) \
            or (pbf and not ext.pw_gemm_supported(Co, Ce))
        if skip:
            H, W = H2, W2
            continue
        dev = "cuda"
        M2 = N * HW2
        expand = sp.expand_ch != sp.in_ch
        zout = expand and backbone.pw_bwd_z_preferred(Ce, sp.in_ch, k, H2, W2, s)
        dy3 = torch.randn(M2, Co, device=dev).to(BF)
        Wp = (torch.randn(Co, Ce, device=dev) * Co ** -0.5).to(BF)
        y2 = torch.randn(N, H2, W2, Ce, device=dev).to(BF)
        x1 = torch.randn(N, H, W, Ce, device=dev).to(BF)
        gate, rb = torch.rand(N, Ce, device=dev), torch.randn(N, Ce, device=dev) * 1e-3
        v = lambda: torch.rand(Ce, device=dev) + 0.5
        sc2, sh2, mu2, rs2, g2, mdz, mdzx = v(), v(), v(), v(), v(), v() * 0.01, v() * 0.01
        sc1, sh1, mu1, rs1 = (v(), v(), v(), v()) if expand else (None, None, None, None)
        act = 1 if expand else 0
        w = torch.randn(Ce, k * k, device=dev) * 0.2
        if (Ce, Co) in backbone.GEMM_PROJ_DGRAD:
            dgrad = lambda: ext.gemm(dy3, Wp, True, cfg=backbone.GEMM_PROJ_DGRAD[(Ce, Co)])[0]
        else:
            dgrad = lambda: backbone._lin(dy3, Wp.t())
        dA = dgrad()
        reduce = lambda: ext.se_bn_bwd_reduce(dA.view(N, HW2, Ce), y2.view(N, HW2, Ce), sc2, sh2, mu2, rs2)
        dw_args = lambda d, rdy: ext.dw_bwd_fused(d.view(N, H2, W2, Ce), y2, gate, rb, sc2, sh2, mu2, rs2, g2, mdz, mdzx,
                                                  w, k, x1, sc1, sh1, act, mu1, rs1, backbone.MAX_BLOCKS,
                                                  backbone.DW_VARIANT, zout, dy_ready=rdy)
        se_red = lambda c: ext.gemm_se(dy3, Wp, y2.view(M2, Ce), HW2, sc2, sh2, mu2, rs2, cfg=c)
        se_bwd = lambda c: ext.gemm_se(dy3, Wp, y2.view(M2, Ce), HW2, sc2, sh2, mu2, rs2, gate, rb, g2, mdz, mdzx,
                                       cfg=c)
        if pbf:
            # projbwd blocks: the dgrad is the skinny pw_gemm (dA) vs pw_gemm_bn2bwd (dy2); the sums come from projbwd
            # in both paths (not timed)
            WpT = Wp.t().contiguous()
            dgrad = lambda: ext.pw_gemm(dy3, WpT, backbone.PW_BLOCKS)[0]
            bn2bwd = lambda: ext.pw_gemm_bn2bwd(dy3, WpT, y2.view(M2, Ce), gate, rb, HW2, sc2, sh2, mu2, rs2, g2, mdz,
                                                mdzx, backbone.PW_BLOCKS)
            dA, dy2 = dgrad(), bn2bwd()
            t = [timeit(f, a.iters) for f in (dgrad, lambda: dw_args(dA, False), bn2bwd, lambda: dw_args(dy2, True))]
            old, new = t[0] + t[1], t[2] + t[3]
            tot_old += old
            tot_new += new
            print(f"{sp.index:>3} {Ce:>5} {Co:>4} {k:>2} {s:>2} {H2:>3}x{W2:<3} | {t[0]:7.1f} {'-':>7} {t[1]:7.1f} "
                  f"{old:7.1f} | {'-':>7} {t[2]:7.1f} {t[3]:7.1f} {new:7.1f} | {old - new:6.1f}  (pw_gemm / bn2bwd)",
                  flush=True)
            H, W = H2, W2
            del dA, dy2, y2, x1, dy3
            torch.cuda.empty_cache()
            continue
        dy2 = se_bwd(0)
        t_red = [timeit(lambda: se_red(c), a.iters) for c in range(4)]
        t_bwd = [timeit(lambda: se_bwd(c), a.iters) for c in range(4)]
        best_red[(Ce, Co, HW2)] = (min(range(4), key=lambda c: t_red[c]), [round(x, 1) for x in t_red])
        best_bwd[(Ce, Co, HW2)] = (min(range(4), key=lambda c: t_bwd[c]), [round(x, 1) for x in t_bwd])
        t = [timeit(f, a.iters) for f in (dgrad, reduce, lambda: dw_args(dA, False))]
        t += [min(t_red), min(t_bwd), timeit(lambda: dw_args(dy2, True), a.iters)]
        old, new = t[0] + t[1] + t[2], t[3] + t[4] + t[5]
        tot_old += old
        tot_new += new
        print(f"{sp.index:>3} {Ce:>5} {Co:>4} {k:>2} {s:>2} {H2:>3}x{W2:<3} | {t[0]:7.1f} {t[1]:7.1f} {t[2]:7.1f} "
              f"{old:7.1f} | {t[3]:7.1f} {t[4]:7.1f} {t[5]:7.1f} {new:7.1f} | {old - new:6.1f}", flush=True)
        H, W = H2, W2
        del dA, dy2, y2, x1, dy3
        torch.cuda.empty_cache()
    print(f"total: staging {tot_old / 1e3:.3f} ms, dy-ready {tot_new / 1e3:.3f} ms, gain {(tot_old - tot_new) / 1e3:.3f} ms")
    print("gemm_se tile config per (Ce, Cout, HW2) -- best, us for cfg 0..3:")
    for key in best_red:
        print(f"  {key}: red {best_red[key]}  bwd {best_bwd[key]}")


if __name__ == "__main__":
    main()
