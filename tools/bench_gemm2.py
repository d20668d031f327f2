#!/usr/bin/env python3
"""gemm.hip v2 (persistent LDS-DMA ring, csrc/kernels/gemm2.hip) against the library (torch.mm on hipBLASLt, with the
recorded TunableOp solutions the step uses) and gemm.hip v1, on the step's library-GEMM shapes (same box, same
inputs).  Data gradients C = dY W run on v2 as NT with the weight transposed once (the transpose is timed too).

  python tools/bench_gemm2.py [--iters 30]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_rt1_for_distributed_training_amd.utils.tuned_gemms import enable_tuned_gemms  # noqa: E402

TUNED = enable_tuned_gemms()
import torch  # noqa: E402
from pytorch_rt1_for_distributed_training_amd import ops  # noqa: E402

BF = torch.bfloat16
# (name, M, N, K, nn)
SHAPES = [
    ("qkv fwd", 8448, 3072, 512, False), ("out fwd", 8448, 512, 1024, False), ("ff fwd", 8448, 512, 512, False),
    ("qkv dgrad", 8448, 512, 3072, True), ("out dgrad", 8448, 1024, 512, True), ("ff dgrad", 8448, 512, 512, True),
    ("proj25 fwd", 76800, 384, 2304, False), ("conv1x1 fwd", 76800, 512, 1536, False),
    ("top fwd", 76800, 1536, 384, False), ("exp25 fwd", 76800, 2304, 384, False),
    ("proj25 dgrad", 76800, 2304, 384, True), ("conv1x1 dgrad", 76800, 1536, 512, True),
    ("top dgrad", 76800, 384, 1536, True), ("exp25 dgrad", 76800, 384, 2304, True),
]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    ext = ops.load()
    print(f"tuned library GEMMs: {TUNED}")
    print(f"{'shape':14s} {'M':>6s} {'N':>5s} {'K':>5s}  {'roof us':>8s} {'lib us':>8s} {'v1 us':>8s} " +
          " ".join(f"{'v2.' + str(v) + ' us':>8s}" for v in range(4)) + f" {'best+T':>8s}  best/lib  maxrel", flush=True)
    wins = 0
    for name, M, N, K, nn in SHAPES:
        x = torch.randn(M, K, device="cuda").to(BF)
        w = (torch.randn(N, K, device="cuda") * 0.05).to(BF)         # the NT operand [N, K]
        b = w.t().contiguous()                                        # NN: the weight as the library sees it, [K, N]
        roof = max((M * K + N * K + M * N) * 2 / 5.3e12, 2 * M * N * K / 2.3e15) * 1e6
        if nn:
            lib = timeit(lambda: torch.mm(x, b), a.iters)
            v1 = timeit(lambda: ext.gemm(x, b, True, cfg=0), a.iters)
        else:
            lib = timeit(lambda: torch.mm(x, w.t()), a.iters)
            v1 = timeit(lambda: ext.gemm(x, w, False, cfg=0), a.iters)
        v2 = [timeit(lambda v=v: ext.gemm2(x, w, variant=v), a.iters) for v in range(4)]
        best = min(range(4), key=lambda v: v2[v])
        v2t = timeit(lambda: ext.gemm2(x, b.t().contiguous(), variant=best), a.iters) if nn else v2[best]
        ref = x.float() @ w.float().t()
        err = max(float(((ext.gemm2(x, w, variant=v)[0].float() - ref).abs().max() / ref.abs().max()))
                  for v in range(4))
        wins += lib / v2t >= 1.0
        print(f"{name:14s} {M:6d} {N:5d} {K:5d}  {roof:8.1f} {lib:8.1f} {v1:8.1f} " +
              " ".join(f"{t:8.1f}" for t in v2) + f" {v2t:8.1f}  v{best} {lib / v2t:5.2f}x  {err:.1e}", flush=True)
    print(f"v2 (incl. the weight transpose on data gradients) >= library on {wins}/{len(SHAPES)} shapes", flush=True)


if __name__ == "__main__":
    main()
