#!/usr/bin/env python3
"""Squeeze-excitation MLP forward / backward per MBConv block shape: fused se.hip kernels vs the torch-op path.

  python tools/bench_se.py [--frames 768] [--ab <other build .so>]

``--ab`` times the fused forward / backward of this build against a second build of the extension loaded into the
same process (launches interleaved, identical inputs) and prints the outputs' relative difference.
"""
from __future__ import annotations

import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_rt1_for_distributed_training_amd.models.efficientnet import block_specs  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.ops import load  # noqa: E402


def timeit(fn, iters=20):
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
    ts.sort()
    return ts[len(ts) // 2]


def timeab(fa, fb, iters=30):
    for _ in range(3):
        fa(), fb()
    ts = [[], []]
    for _ in range(iters):
        for k, f in enumerate((fa, fb)):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            f()
            b.record()
            b.synchronize()
            ts[k].append(a.elapsed_time(b) * 1e3)
    return [sorted(t)[len(t) // 2] for t in ts]


def _rel(x, y):
    return max(float((p.float() - q.float()).norm() / (q.float().norm() + 1e-12)) for p, q in zip(x, y)
               if isinstance(p, torch.Tensor))


def main_ab(a):
    from tools.bench_dw_replay import load_other
    ext, other = load(), load_other(a.ab)
    N, dev = a.frames, "cuda"
    tot = [0.0, 0.0, 0.0, 0.0]
    print(f"{'blk':>3} {'C':>5} {'S':>3} | {'fwd':>8} {'other':>8} | {'bwd':>8} {'other':>8} | rel diff fwd / bwd")
    for sp in block_specs():
        C, S, HW = sp.expand_ch, sp.se_ch, 100
        g = torch.Generator(device=dev).manual_seed(sp.index)
        ps = torch.randn(N, C, device=dev, generator=g)
        w1, b1 = torch.randn(S, C, device=dev, generator=g) * 0.1, torch.randn(S, device=dev, generator=g)
        w2, b2 = torch.randn(C, S, device=dev, generator=g) * 0.1, torch.randn(C, device=dev, generator=g)
        red = torch.randn(5, N, C, device=dev, generator=g)
        fo = ext.se_fwd(ps, 1.0 / HW, w1, b1, w2, b2)
        pool, h, gate = fo
        fw = timeab(lambda: ext.se_fwd(ps, 1.0 / HW, w1, b1, w2, b2),
                    lambda: other.se_fwd(ps, 1.0 / HW, w1, b1, w2, b2))
        bw = timeab(lambda: ext.se_bwd(red, gate, h, pool, 1.0 / HW, w1, w2, float(N * HW)),
                    lambda: other.se_bwd(red, gate, h, pool, 1.0 / HW, w1, w2, float(N * HW)))
        df = _rel(ext.se_fwd(ps, 1.0 / HW, w1, b1, w2, b2), other.se_fwd(ps, 1.0 / HW, w1, b1, w2, b2))
        db = _rel(ext.se_bwd(red, gate, h, pool, 1.0 / HW, w1, w2, float(N * HW)),
                  other.se_bwd(red, gate, h, pool, 1.0 / HW, w1, w2, float(N * HW)))
        for k, v in enumerate(fw + bw):
            tot[k] += v
        print(f"{sp.index:>3} {C:>5} {S:>3} | {fw[0]:8.1f} {fw[1]:8.1f} | {bw[0]:8.1f} {bw[1]:8.1f} | {df:.1e} {db:.1e}",
              flush=True)
    print(f"total us (x1 per block): fwd {tot[0]:.0f} vs {tot[1]:.0f}, bwd {tot[2]:.0f} vs {tot[3]:.0f}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=768)
    ap.add_argument("--ab", default="")
    a = ap.parse_args()
    if a.ab:
        return main_ab(a)
    ext = load()
    N, dev = a.frames, "cuda"
    print(f"{'blk':>3} {'C':>5} {'S':>3} | {'fwd old':>8} {'fwd new':>8} | {'bwd old':>8} {'bwd new':>8}")
    to = tn = 0.0
    for sp in block_specs():
        C, S, HW = sp.expand_ch, sp.se_ch, 100
        ps = torch.randn(N, C, device=dev)
        w1, b1 = torch.randn(S, C, device=dev), torch.randn(S, device=dev)
        w2, b2 = torch.randn(C, S, device=dev), torch.randn(C, device=dev)
        red = torch.randn(5, N, C, device=dev)

        def fwd_old():
            pool = ps / HW
            h = torch.addmm(b1, pool, w1.t())
            hs = F.silu(h)
            return pool, h, hs, torch.sigmoid(torch.addmm(b2, hs, w2.t())).contiguous()

        pool, h, hs, gate = fwd_old()

        def bwd_old():
            dz, df2b = ext.se_bwd_dz(red[0], gate)
            dz.t() @ hs
            dh, df1b = ext.se_bwd_dh(dz @ w2, h)
            dh.t() @ pool
            ext.se_bwd_bnsum(red, gate, dh @ w1, 1.0 / HW, float(N * HW))

        f_o = timeit(fwd_old)
        f_n = timeit(lambda: ext.se_fwd(ps, 1.0 / HW, w1, b1, w2, b2))
        b_o = timeit(bwd_old)
        b_n = timeit(lambda: ext.se_bwd(red, gate, h, pool, 1.0 / HW, w1, w2, float(N * HW)))
        to += f_o + b_o
        tn += f_n + b_n
        print(f"{sp.index:>3} {C:>5} {S:>3} | {f_o:8.1f} {f_n:8.1f} | {b_o:8.1f} {b_n:8.1f}", flush=True)
    print(f"total us: old {to:.0f}, fused {tn:.0f}")


if __name__ == "__main__":
    main()
