"""fp8 (OCP e4m3fn) forward GEMMs with delayed per-tensor scaling -- BASELINE config 5 ("fp8 weights").

Forward products of the hipBLASLt-sized GEMMs (mid/low-resolution 1x1 convs of the encoder, the top conv,
conv1x1, and the transformer QKV / out / FF projections) run as fp8 x fp8 -> bf16 on CDNA4's fp8 MFMA via
``torch._scaled_mm`` (hipBLASLt).  Activations are quantised by ``csrc/kernels/fp8.hip`` in one pass with the
scale recorded at the previous call of the same site (the pass also records this call's amax, integer atomicMax:
reproducible); weights are quantised every step with their exact amax.  Backward products stay bf16 on the
saved bf16 operands (the usual fp8-forward training recipe), so only the forward numerics change.
"""
from __future__ import annotations

from typing import Dict

import torch

from ._ext import load

E4M3 = torch.float8_e4m3fn
_ENABLED = False


class _Site:
    __slots__ = ("amax_prev", "amax_next", "w_scratch")

    def __init__(self, a: torch.Tensor):
        first = a.detach().abs().amax().float().clamp(min=1e-12).reshape(1)
        self.amax_prev = torch.empty(1, dtype=torch.float32, device=a.device)
        self.amax_next = first.view(torch.int32).clone()
        self.w_scratch = torch.zeros(1, dtype=torch.int32, device=a.device)


_SITES: Dict[object, _Site] = {}


def enable(flag: bool = True):
    global _ENABLED
    _ENABLED = bool(flag)


def enabled() -> bool:
    return _ENABLED


def supported(M: int, K: int, N: int) -> bool:
    return K % 16 == 0 and N % 16 == 0 and M % 16 == 0


def fp8_mm(a: torch.Tensor, w: torch.Tensor, key) -> torch.Tensor:
    """a [M, K] bf16 @ w[N, K]^T bf16 -> [M, N] bf16 through e4m3fn operands (forward only)."""
    ext = load()
    a = a.contiguous()
    site = _SITES.get(key)
    if site is None:
        site = _SITES[key] = _Site(a)
    site.amax_prev.copy_(site.amax_next.view(torch.float32))
    site.amax_next.zero_()
    a8, sa = ext.fp8_quant(a, site.amax_prev, site.amax_next)
    wc = w.contiguous()
    wmax = wc.abs().amax().float().clamp(min=1e-12).reshape(1)
    w8, sw = ext.fp8_quant(wc, wmax, site.w_scratch)
    return torch._scaled_mm(a8, w8.t(), scale_a=sa, scale_b=sw, out_dtype=torch.bfloat16)


def maybe_fp8_mm(a: torch.Tensor, w: torch.Tensor, key):
    """fp8 product when enabled and the shape qualifies, else None (caller runs bf16)."""
    if not _ENABLED or key is None:
        return None
    M, K = a.shape
    if not supported(M, K, w.shape[0]):
        return None
    return fp8_mm(a, w, key)
