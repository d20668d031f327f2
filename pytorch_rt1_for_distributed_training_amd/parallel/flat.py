"""Flat parameter / gradient storage.

Every trainable parameter is a view into ONE fp32 buffer and its ``.grad`` a
view into ONE fp32 gradient buffer, laid out in gradient-ready order.  This is
what makes the rest of the MI355X design cheap:

* data-parallel buckets are contiguous slices of the gradient buffer, so a
  bucket all-reduce is a single RCCL call with no pack/unpack copy;
* the optimizer is one fused kernel launch over the whole buffer
  (``ops.adam``), instead of 572 per-tensor launches;
* zeroing gradients is one memset; the 1/world averaging is folded into the
  optimizer kernel.

Per-parameter gradient accumulation is avoided: ``zero_grad(set_to_none=True)``
memsets the buffer and releases every ``.grad``, so autograd's AccumulateGrad
*steals* the tensor each backward produces (no ``grad += g`` kernel per
parameter, ~570 launches per RT-1 step).  ``gather_grads`` then lands the stolen
tensors in the flat buffer with one multi-tensor copy (per DP bucket, or for
everything before the optimizer) and re-points ``.grad`` at the flat views.

Segments are padded to 64 elements (256 B) so every parameter starts on a
16-B-vectorisable boundary.
"""
from __future__ import annotations

import bisect
from typing import Dict, List, Optional, Sequence

import torch
import torch.nn as nn

from ..ops import switches

ALIGN = 64
MULTI_COPY = switches.on("multi_copy")     # one-launch gradient gather (ops/switches.py)


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


# Split-K weight gradients whose fixed-order sum is deferred into the gather (``defer_partials``): the wgrad kernels
# leave [splits, Co, Ci] fp32 partials, autograd steals the first split's [Co, Ci] view as the parameter's gradient,
# and gather_grads sums the splits on their way into the flat buffer (csrc/kernels/reduce.hip multi_reduce_copy: one
# launch per bucket instead of one colsum launch per weight gradient).  first-split data_ptr -> (partials, bytes).
_PENDING: Dict[int, tuple] = {}
_DEFER = [0]
# Only partial sets up to this size wait for the gather: a bigger one (the transformer's Q/K/V gradient: 8 x 6.3 MB) is
# summed right after its kernel while it is still in the 256 MB last-level cache -- deferred to the end of the
# backward it came back from HBM and the gather's reduce cost what the colsum launches saved (tools/bench_reduce.py,
# profiles/r6_defer_trace.md)
DEFER_MAX_BYTES = 24 << 20


class deferred_sums:
    """Context of one backward whose parameter gradients the flat gather collects: weight-gradient sites may return
    unsummed split partials (``defer_partials``).  Not for gradient accumulation over several backwards (a second
    backward's AccumulateGrad would add only its first split)."""

    def __init__(self, enabled: bool = True):
        self.enabled = enabled

    def __enter__(self):
        if self.enabled:
            _DEFER[0] += 1
        return self

    def __exit__(self, *exc):
        if self.enabled:
            _DEFER[0] -= 1
        return False


def defer_partials(part: torch.Tensor, ok: bool = True) -> torch.Tensor:
    """Parameter gradient from split partials ``part`` [S, ...] (fp32): inside ``deferred_sums``, the first split's
    view with the sum left to the flat gather; otherwise the fixed-order sum now.  ``ok``: every slice of the result
    becomes a gradient of a parameter that requires one (a dropped slice would leave the entry pending)."""
    if part.shape[0] == 1:
        return part[0]
    if (ok and _DEFER[0] and part.is_cuda and part.dtype == torch.float32 and part.is_contiguous()
            and part.numel() * 4 <= DEFER_MAX_BYTES):
        g = part[0]
        _PENDING[g.data_ptr()] = [part, g.numel() * 4, g.numel() * 4]     # partials, bytes, bytes not yet gathered
        _BASES.clear()
        return g
    if not part.is_cuda:
        return part.sum(0)
    from ..ops import load
    return load().colsum(part)


_BASES: List[int] = []      # sorted keys of _PENDING (rebuilt lazily after a registration)


def _pending_of(g: torch.Tensor):
    """(base, splits, split stride in elements) when ``g`` is (a row slice of) a deferred first split, else None."""
    if not _PENDING:
        return None
    if len(_BASES) != len(_PENDING):
        _BASES[:] = sorted(_PENDING)
    ptr = g.data_ptr()
    i = bisect.bisect_right(_BASES, ptr) - 1
    if i < 0:
        return None
    base = _BASES[i]
    ent = _PENDING.get(base)
    if ent is None or ptr >= base + ent[1]:
        return None
    if ptr + g.numel() * 4 > base + ent[1]:
        raise RuntimeError("a gradient straddles a deferred split-K partial")
    return base, ent[0].shape[0], ent[0][0].numel()


def _copy_many(dst: List[torch.Tensor], src: List[torch.Tensor]):
    """dst[i].copy_(src[i]): on the GPU through the extension's multi-copy kernel (32 tensors per launch instead of
    one blit per tensor), else ``torch._foreach_copy_``."""
    if dst[0].is_cuda and MULTI_COPY:
        from ..ops import available, load
        if available():
            ok = [d.dtype == torch.float32 and s.dtype == torch.float32 and s.is_contiguous() and s.device == d.device
                  for d, s in zip(dst, src)]
            fast = [i for i, k in enumerate(ok) if k]
            if fast:
                load().multi_copy_([dst[i] for i in fast], [src[i] for i in fast])
            rest = [i for i, k in enumerate(ok) if not k]
            if rest:
                torch._foreach_copy_([dst[i] for i in rest], [src[i] for i in rest])
            return
    torch._foreach_copy_(dst, src)


class FlatParameters:
    def __init__(self, params: Sequence[nn.Parameter], device=None, dtype=torch.float32):
        params = list(params)
        if not params:
            raise ValueError("no parameters")
        device = device or params[0].device
        self.params: List[nn.Parameter] = params
        self.offsets: List[int] = []
        off = 0
        for p in params:
            self.offsets.append(off)
            off += _align(p.numel())
        self.numel = off
        self.data = torch.zeros(off, device=device, dtype=dtype)
        self.grad = torch.zeros(off, device=device, dtype=dtype)
        with torch.no_grad():
            for p, o in zip(params, self.offsets):
                n = p.numel()
                view = self.data[o:o + n].view_as(p)
                view.copy_(p.data)
                p.data = view
                p.grad = self.grad[o:o + n].view_as(p)
        self.index: Dict[int, int] = {id(p): i for i, p in enumerate(params)}
        self.views: List[torch.Tensor] = [p.grad for p in params]
        self._loose = False   # some .grad may not be a flat view (released by zero_grad(set_to_none=True))

    def zero_grad(self, set_to_none: bool = False):
        self.grad.zero_()
        if set_to_none:
            for p in self.params:
                p.grad = None
            self._loose = True

    def gather_grads(self, indices: Optional[Sequence[int]] = None):
        """Copy gradients that autograd stored outside the flat buffer into it (one ``_foreach_copy_``)
        and point ``.grad`` back at the flat views.  Parameters without a gradient keep the zeros of
        the last ``zero_grad``."""
        if not self._loose:
            self._check_pending(indices)
            return
        dst, src, red = [], [], []
        used = set()
        for i in (range(len(self.params)) if indices is None else indices):
            p, v = self.params[i], self.views[i]
            g = p.grad
            if g is not None and g.data_ptr() != v.data_ptr():
                pend = _pending_of(g) if g.is_cuda else None
                if pend is not None:
                    if v.dtype != torch.float32 or not g.is_contiguous():
                        raise RuntimeError("deferred split-K gradient needs an fp32 flat buffer")
                    _PENDING[pend[0]][2] -= g.numel() * 4
                    used.add(pend[0])
                    red.append((v, g, pend[1], pend[2]))
                else:
                    dst.append(v)
                    src.append(g)
            p.grad = v
        if red:
            from ..ops import load
            load().multi_reduce_copy_([r[0] for r in red], [r[1] for r in red], [r[2] for r in red],
                                      [r[3] for r in red])
        if dst:
            _copy_many(dst, src)
        for b in used:
            if _PENDING[b][2] <= 0:
                del _PENDING[b]
                _BASES.clear()
        if indices is None:
            self._loose = False
        self._check_pending(indices)

    def _check_pending(self, indices):
        if indices is None and _PENDING:
            n = len(_PENDING)
            _PENDING.clear()
            _BASES.clear()
            raise RuntimeError(f"{n} deferred split-K gradient(s) never reached the flat gather (a gradient was "
                               "modified or accumulated after its weight-gradient kernel)")

    def reattach_grads(self):
        """Re-point ``.grad`` at the flat buffer (after something replaced it)."""
        self._loose = True
        self.gather_grads()

    def segment(self, i: int):
        return self.offsets[i], self.params[i].numel()

    def state_tensors(self) -> List[torch.Tensor]:
        return [p.data for p in self.params]


def flatten_buffers(module: nn.Module, device=None) -> Optional[torch.Tensor]:
    """Move every floating-point buffer (BN running stats) into one flat tensor
    so it can be broadcast with one collective (DDP ``broadcast_buffers``)."""
    bufs = [(m, n, b) for m in module.modules() for n, b in m.named_buffers(recurse=False)
            if b is not None and b.is_floating_point() and n in ("running_mean", "running_var")]
    if not bufs:
        return None
    total = sum(_align(b.numel()) for _, _, b in bufs)
    flat = torch.zeros(total, device=device or bufs[0][2].device, dtype=torch.float32)
    off = 0
    for m, n, b in bufs:
        view = flat[off:off + b.numel()].view_as(b)
        view.copy_(b)
        setattr(m, n, view)
        m._buffers[n] = view
        off += _align(b.numel())
    return flat
