#!/usr/bin/env python3
"""The project conv of the wide blocks (8-25) at the real shapes (768 frames at 300x300): how much of each kernel is
its BN2 + SiLU + gate operand prologue.  Per block: the operand pass bn_apply (y2 -> A), the GEMM on the stored A, and
the GEMM with the prologue rebuilding A from y2 -- on the kernel the block uses (pw_tall for N <= 144, gemm.hip for
blocks 18-23, hipBLASLt otherwise), all with the BN3 statistics where the step takes them.

  python tools/bench_proj_prologue.py [--frames 768] [--res 300] [--blocks 9,14,19]
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
ACT_SILU = 1


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
    print(f"{'blk':>3} {'Ce':>5} {'Co':>4} {'HW':>4} {'kernel':>8} | {'bn_apply':>8} {'gemm(A)':>8} {'gemm(pro)':>9} "
          f"| pro - plain")
    for sp in block_specs():
        Ce, Co, k, s = sp.expand_ch, sp.out_ch, sp.kernel, sp.stride
        H2, W2 = conv_out_size(H, k, s), conv_out_size(W, k, s)
        H, W = H2, W2
        HW2 = H2 * W2
        if sp.index < 8 or (sel and sp.index not in sel):
            continue
        dev = "cuda"
        M2 = N * HW2
        y2 = torch.randn(M2, Ce, device=dev).to(BF)
        wp = (torch.randn(Co, Ce, device=dev) * Ce ** -0.5).to(BF)
        sc, sh = torch.rand(Ce, device=dev) + 0.5, torch.randn(Ce, device=dev) * 0.2
        gate = torch.rand(N, Ce, device=dev)
        A = ext.bn_apply(y2, sc, sh, ACT_SILU, gate, HW2)
        t_apply = timeit(lambda: ext.bn_apply(y2, sc, sh, ACT_SILU, gate, HW2), a.iters)
        if (Ce, Co) in backbone.GEMM_PROJ:
            kind, cfg = "gemm.hip", backbone.GEMM_PROJ[(Ce, Co)]
            plain = lambda: ext.gemm(A, wp, False, None, stats=True, cfg=cfg)
            pro = lambda: ext.gemm(y2, wp, False, None, sc, sh, gate, HW2, stats=True, cfg=cfg)
        elif ext.pw_tall_preferred(Ce, Co):
            kind = "pw_tall"
            plain = lambda: ext.pw_tall(A, wp)
            pro = lambda: ext.pw_tall(y2, wp, sc, sh, gate, HW2, False)
        else:
            kind = "library"
            plain = lambda: torch.mm(A, wp.t())
            pro = None
        t_plain = timeit(plain, a.iters)
        t_pro = timeit(pro, a.iters) if pro is not None else float("nan")
        extra = ""
        if kind == "pw_tall":
            # the weight gradient dWp = dy3^T A: on the stored A, or with A rebuilt from y2 in the wgrad kernel
            dy3 = torch.randn(M2, Co, device=dev).to(BF)
            t_store = timeit(lambda: ext.pw_tall(y2, wp, sc, sh, gate, HW2, True), a.iters)
            t_wg = timeit(lambda: backbone.wgrad(dy3, A), a.iters)
            t_wgp = timeit(lambda: backbone.wgrad(dy3, y2, prologue=(sc, sh, gate, ACT_SILU, HW2)), a.iters)
            extra = (f" | pro+store {t_store:6.1f}  wgrad(A) {t_wg:6.1f}  wgrad(pro) {t_wgp:6.1f} | now "
                     f"{t_apply + t_plain + t_wg:6.1f}  pro+store {t_store + t_wg:6.1f}  pro+wgrad(pro) "
                     f"{t_pro + t_wgp:6.1f}")
            del dy3
        print(f"{sp.index:>3} {Ce:>5} {Co:>4} {HW2:>4} {kind:>8} | {t_apply:8.1f} {t_plain:8.1f} {t_pro:9.1f} | "
              f"{t_pro - t_plain:7.1f}{extra}", flush=True)
        del y2, A
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
