#!/usr/bin/env python3
"""1x1-conv weight gradients at the encoder's real shapes: the MFMA streaming kernel (csrc/kernels/wgrad.hip)
vs the previous split-K torch.bmm (hipBLASLt) + column-sum path, per shape (median us) and achieved GB/s.

  python tools/bench_wgrad.py --frames 768 --res 300
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
    ap.add_argument("--variants", action="store_true", help="also time every tile variant of the MFMA kernel")
    a = ap.parse_args()
    ext = load()
    N = a.frames
    H = W = conv_out_size(a.res, 3, 2)
    shapes = []
    for sp in block_specs():
        Ho, Wo = conv_out_size(H, sp.kernel, sp.stride), conv_out_size(W, sp.kernel, sp.stride)
        shapes.append((f"blk{sp.index} project", N * Ho * Wo, sp.out_ch, sp.expand_ch))
        if sp.expand_ch != sp.in_ch:
            shapes.append((f"blk{sp.index} expand", N * H * W, sp.expand_ch, sp.in_ch))
        H, W = Ho, Wo
    shapes += [("top 384->1536", N * H * W, 1536, 384), ("conv1x1 1536->512", N * H * W, 512, 1536)]
    tot_new = tot_old = 0.0
    NV = 6
    vh = "".join(f" {'v' + str(i):>7}" for i in range(NV)) if a.variants else ""
    print(f"{'site':22s} {'M':>9} {'Co':>5} {'Ci':>5} | {'bmm us':>8} {'new us':>8} {'new GB/s':>8} |{vh}")
    for name, M, Co, Ci in shapes:
        dy = torch.randn(M, Co, device="cuda").to(torch.bfloat16)
        x = torch.randn(M, Ci, device="cuda").to(torch.bfloat16)
        t_old = timeit(lambda: backbone.wgrad_bmm(dy, x))
        t_new = timeit(lambda: ext.wgrad(dy, x))
        tot_old += t_old
        tot_new += t_new
        gbs = (M * (Co + Ci) * 2) / t_new / 1e3
        vs = ""
        if a.variants:
            ref = backbone.wgrad_bmm(dy, x)
            for v in range(NV):
                out = ext.wgrad(dy, x, variant=v)
                err = (out - ref).abs().max().item() / max(ref.abs().max().item(), 1e-6)
                assert err < 2e-2, (name, v, err)
                vs += f" {timeit(lambda: ext.wgrad(dy, x, variant=v)):7.1f}"
        print(f"{name:22s} {M:>9} {Co:>5} {Ci:>5} | {t_old:8.1f} {t_new:8.1f} {gbs:8.0f} |{vs}", flush=True)
        del dy, x
        torch.cuda.empty_cache()
    print(f"total: bmm {tot_old / 1e3:.2f} ms, new {tot_new / 1e3:.2f} ms")


if __name__ == "__main__":
    main()
