#!/usr/bin/env python3
"""FiLM projection kernels at the bench shape (768 frames, the encoder's 27 FiLM layers): gemm.hip tile configs of the
column-mapped forward and the row splits of the column-mapped weight gradient, median of interleaved rounds.

  python tools/bench_film.py [--frames 768]
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_rt1_for_distributed_training_amd import ops  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.config import RT1Config  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.models import build_rt1  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.ops import backbone  # noqa: E402
from tools.bench_tf_gemms import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=768)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    ext = ops.load()
    model = build_rt1(RT1Config(backend="hip"))
    enc = model._image_tokenizer._tokenizer
    ws, bs, sizes = backbone.film_params(enc.net, enc)
    M, N = a.frames, sum(sizes)
    xe = torch.randn(M, 512, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, 512, device="cuda") * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device="cuda") * 0.05
    cmap, _ = backbone._film_layout(sizes, M, xe.device)
    g = torch.randn(M * N, device="cuda")
    cands = {f"fwd cfg{c}": (lambda c=c: ext.film_fwd(xe, 512, w, b, cmap, M * N, c)) for c in range(5)}
    cands.update({f"wgrad t{t}s{s}": (lambda s=s, t=t: ext.film_wgrad(g, cmap, xe, 512, s, t))
                  for t in (0, 1) for s in (1, 2)})
    times = {k: [] for k in cands}
    for _ in range(a.rounds):
        for k, fn in cands.items():
            times[k].append(timeit(fn, a.iters))
    floor_f = (M * 512 * 2 + N * 512 * 2 + M * N * 4) / 5e12 * 1e6
    print(f"M={M} N={N}: forward byte floor {floor_f:.1f} us")
    for k, v in times.items():
        print(f"{k:10s} {statistics.median(v):7.1f} us", flush=True)


if __name__ == "__main__":
    main()
