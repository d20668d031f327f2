"""fp8 (OCP e4m3fn) support: the activation quantiser only.  The fp8 forward-GEMM path is retired.

Round 1-3 ran BASELINE config 5 ("456x456 + fp8 weights") with the hipBLASLt-sized forward products as e4m3fn x e4m3fn
``torch._scaled_mm`` calls behind a one-pass activation quantiser (``csrc/kernels/fp8.hip``, delayed per-tensor
scaling) and a per-step weight quantisation.  It never paid: those GEMMs are HBM-bound at this model's shapes, so the
extra quantisation passes cost more than the faster fp8 MFMA saves -- 2.2 % slower than bf16 at 456x456, b128, in
rounds 2 and 3 (``profiles/r3_bench_b456_fp8.log`` vs ``profiles/r3_bench_b456_bf16.log``; round 2:
``profiles/r2_bench_456_fp8.log``).  It would only pay with every producer kernel emitting e4m3 directly (activations
stored in fp8 end to end), which this framework does not do.  The quantiser stays (tested, reusable); ``enable(True)``
refuses with this explanation, and config 5 runs in bf16 (``bench.py --height 456 --width 456``).
"""
from __future__ import annotations

import torch

from ._ext import load

E4M3 = torch.float8_e4m3fn
RETIRED = ("the fp8 forward-GEMM path is retired: it measured 2.2 % slower than bf16 at 456x456 "
           "(profiles/r3_bench_b456_fp8.log vs profiles/r3_bench_b456_bf16.log); run config 5 in bf16")


def enable(flag: bool = True):
    if flag:
        raise ValueError(RETIRED)


def enabled() -> bool:
    return False


def quantize(a: torch.Tensor, amax_prev: torch.Tensor, amax_next: torch.Tensor):
    """a bf16 -> (e4m3fn tensor, fp32 scale) with the scale from ``amax_prev``; this call's amax is recorded into
    ``amax_next`` (int32 bits, integer atomicMax: reproducible) -- csrc/kernels/fp8.hip."""
    return load().fp8_quant(a.contiguous(), amax_prev, amax_next)


def maybe_fp8_mm(a: torch.Tensor, w: torch.Tensor, key):
    """Kept for call-site compatibility: always None (bf16 product)."""
    return None
