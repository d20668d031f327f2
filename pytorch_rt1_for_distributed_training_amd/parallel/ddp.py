"""Data parallelism: bucketed gradient all-reduce overlapped with backward.

Replaces the reference's ``DDPStrategy(find_unused_parameters=True)``
(``distribute_train.py:235``; collectives C1-C5 in SURVEY §2.8) with an
explicit MI355X-oriented design:

* C1 parameter broadcast: ONE broadcast of the flat parameter buffer;
* C2 gradient all-reduce: the flat gradient buffer (``parallel.flat``) is cut
  into contiguous buckets in gradient-ready order; a post-accumulate-grad hook
  counts arrivals and launches the bucket's all-reduce (SUM) as soon as its
  last gradient lands, so RCCL traffic over xGMI overlaps the rest of the
  backward.  The 1/world average is folded into the optimizer kernel.
  Buckets default to 32 MB: large enough that RCCL spreads each one over
  channels on all 7 xGMI links, small enough (≈5 buckets for RT-1's 141 MB of
  fp32 gradients) to leave only the tail bucket exposed;
* C3 unused-parameter search: none; unused parameters (``_action_token_emb``)
  are frozen statically, and any bucket not complete at ``finish()`` is
  flushed then (so a conditional branch can never deadlock);
* C4 buffer broadcast: optional coalesced broadcast of the flat BN-buffer
  region from rank 0 before each forward (DDP ``broadcast_buffers`` parity);
* C5 loss logging: callers reduce on device only at the log interval.

The collective backend is pluggable: ``torch`` (torch.distributed process
group = RCCL for GPU / gloo for CPU) or ``native`` (the C++ ``rt1_comm``
RCCL communicator with its own HIP comm stream, ``parallel.native_comm``).
"""
from __future__ import annotations

import contextlib
from typing import Callable, List, Optional, Sequence

import os

import torch
import torch.distributed as dist
import torch.nn as nn

from .dist import pg_world1
from .flat import FlatParameters, flatten_buffers


_DEBUG_SYNC_LAUNCH = os.environ.get("RT1_DDP_SYNC_LAUNCH", "0") == "1"


class _Bucket:
    __slots__ = ("index", "start", "end", "members", "pending", "work", "launched")

    def __init__(self, index: int, start: int, end: int, members: List[int]):
        self.index = index
        self.start, self.end, self.members = start, end, members
        self.pending = len(members)
        self.work = None
        self.launched = False


class DataParallel:
    def __init__(self, module: nn.Module, flat: FlatParameters, bucket_cap_mb: float = 32.0,
                 broadcast_buffers: bool = True, process_group=None, comm=None,
                 grad_comm_dtype: torch.dtype = torch.float32):
        self.module = module
        self.flat = flat
        self.pg = process_group
        self.comm = comm  # optional native communicator with all_reduce_(tensor) / broadcast_(tensor, root)
        if comm is not None:
            # the communicator defines the group; a world-1 communicator (NativeComm.single) still runs the whole
            # bucketed path (hooks, RCCL on the comm stream, graph segments) -- the one-GPU rehearsal of it
            self.world = comm.world
            self.enabled = True
        else:
            self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
            self.enabled = self.world > 1 or (dist.is_initialized() and pg_world1())
        self.broadcast_buffers = broadcast_buffers and self.enabled
        self.grad_comm_dtype = grad_comm_dtype
        self._sync = True
        self.launch_log: List[int] = []   # bucket indices in the order their all-reduce was issued (last step)
        self._capture = None   # SegmentedCapture while a hipGraph DP step is being captured (engine/graphs.py)
        self.buffers = flatten_buffers(module) if self.enabled else None
        cap = int(bucket_cap_mb * 1024 * 1024 / flat.grad.element_size())
        self.buckets: List[_Bucket] = []
        self._param_bucket: List[int] = []
        cur: List[int] = []
        start = 0
        nparams = len(flat.params)
        for i in range(nparams):
            end = flat.offsets[i + 1] if i + 1 < nparams else flat.numel
            cur.append(i)
            if end - start >= cap or i + 1 == nparams:
                self.buckets.append(_Bucket(len(self.buckets), start, end, cur))
                cur, start = [], end
        self._param_bucket = [0] * nparams
        for bi, b in enumerate(self.buckets):
            for i in b.members:
                self._param_bucket[i] = bi
        self._hooks = []
        if self.enabled:
            for i, p in enumerate(flat.params):
                self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))
            self.broadcast_parameters()

    # ------------------------------------------------------------------ collectives
    def _all_reduce(self, t: torch.Tensor):
        if self.comm is not None:
            return self.comm.all_reduce_(t)
        if self.grad_comm_dtype != t.dtype:
            # compressed path: reduce a low-precision copy, write back (2x fewer xGMI bytes)
            low = t.to(self.grad_comm_dtype)
            work = dist.all_reduce(low, group=self.pg, async_op=True)
            return _CopyBack(work, low, t)
        return dist.all_reduce(t, group=self.pg, async_op=True)

    def broadcast_parameters(self):
        if not self.enabled:
            return
        in_flat = {id(p) for p in self.flat.params}
        frozen = [p.data for p in self.module.parameters() if id(p) not in in_flat]
        for t in [self.flat.data] + frozen:
            if self.comm is not None:
                self.comm.broadcast_(t, 0)
            else:
                dist.broadcast(t, 0, group=self.pg)
        self.sync_buffers()

    def sync_buffers(self):
        if self.broadcast_buffers and self.buffers is not None:
            if self.comm is not None:
                self.comm.broadcast_(self.buffers, 0)
            else:
                dist.broadcast(self.buffers, 0, group=self.pg)

    # ------------------------------------------------------------------ hooks
    def _make_hook(self, i: int) -> Callable:
        def hook(_p):
            if self._capture is not None:
                b = self.buckets[self._param_bucket[i]]
                b.pending -= 1
                if b.pending == 0 and not b.launched:
                    # captured: land the bucket's gradients in the flat buffer, then end the current graph
                    # segment so this bucket's all-reduce can be issued right after that segment replays
                    b.launched = True
                    if self.flat.grad.is_cuda and torch.cuda.current_stream() != self._capture.stream:
                        raise RuntimeError("gradient hook ran off the capture stream; segmented capture impossible")
                    self.flat.gather_grads(b.members)
                    self._capture.bucket_ready(b.index)
                return
            if not self._sync:
                return
            b = self.buckets[self._param_bucket[i]]
            b.pending -= 1
            if b.pending == 0 and not b.launched:
                self._launch(b)
        return hook

    def _launch(self, b: _Bucket):
        b.launched = True
        self.launch_log.append(b.index)
        self.flat.gather_grads(b.members)
        b.work = self._all_reduce(self.flat.grad[b.start:b.end])
        if _DEBUG_SYNC_LAUNCH:      # debug: no overlap of a bucket's all-reduce with the rest of the backward
            b.work.wait()
            torch.cuda.synchronize()
            b.work = None

    # ------------------------------------------------------------------ step protocol
    def prepare(self):
        """Call before forward: reset bucket state, broadcast BN buffers."""
        for b in self.buckets:
            b.pending = len(b.members)
            b.launched = False
            b.work = None
        self.launch_log = []
        if self._sync:
            self.sync_buffers()

    def finish(self):
        """Call after backward: flush incomplete buckets and wait (stream-wise) for all."""
        if not self.enabled or not self._sync:
            if self._sync:
                self.flat.gather_grads()
            return
        for b in self.buckets:
            if not b.launched:
                self._launch(b)
        for b in self.buckets:
            if b.work is not None:
                b.work.wait()
                b.work = None
        self.flat.gather_grads()   # clears the 'loose' flag (every bucket already gathered its members)

    def all_reduce_grads(self):
        """Sum the whole (already gathered) flat gradient across ranks, bucket by bucket, all in flight at once,
        with no overlap (tools / tests; the training paths overlap buckets with backward)."""
        if not self.enabled:
            return
        works = [self._all_reduce(self.flat.grad[b.start:b.end]) for b in self.buckets]
        for w in works:
            if w is not None:
                w.wait()

    def launch_bucket(self, index: int):
        """Start the all-reduce of one (already gathered) bucket; returns the work handle (or None)."""
        b = self.buckets[index]
        return self._all_reduce(self.flat.grad[b.start:b.end])

    @staticmethod
    def wait_all(works):
        for w in works:
            if w is not None:
                w.wait()

    @contextlib.contextmanager
    def capture_cuts(self, capture):
        """While capturing a DP step as graph segments: gradient hooks gather each completed bucket and tell
        ``capture`` (``engine.graphs.SegmentedCapture``) to cut the graph there.  No collective is captured."""
        for b in self.buckets:
            b.pending = len(b.members)
            b.launched = False
            b.work = None
        prev, self._capture = self._capture, capture
        try:
            yield
        finally:
            self._capture = prev

    def unlaunched_buckets(self) -> List[int]:
        return [b.index for b in self.buckets if not b.launched]

    @property
    def grad_scale(self) -> float:
        """Multiply summed gradients by this to get the data-parallel mean."""
        return 1.0 / self.world if self.enabled else 1.0

    @contextlib.contextmanager
    def no_sync(self):
        prev, self._sync = self._sync, False
        try:
            yield
        finally:
            self._sync = prev


class _CopyBack:
    def __init__(self, work, low, dst):
        self.work, self.low, self.dst = work, low, dst

    def wait(self):
        self.work.wait()
        self.dst.copy_(self.low)


def gradient_ready_order(model: nn.Module, run_backward: Callable[[], None],
                         params: Optional[Sequence[nn.Parameter]] = None) -> List[nn.Parameter]:
    """Order in which gradients become ready during one backward (like DDP's
    bucket rebuild).  ``run_backward`` must run a forward+backward; BN running
    statistics touched by it are restored afterwards."""
    params = [p for p in (params or model.parameters()) if p.requires_grad]
    saved = {k: v.clone() for k, v in model.state_dict().items() if not k.endswith("weight") and not k.endswith("bias")}
    order: List[nn.Parameter] = []
    seen = set()
    hooks = []
    for p in params:
        def h(pp, _p=p):
            if id(_p) not in seen:
                seen.add(id(_p))
                order.append(_p)
        hooks.append(p.register_post_accumulate_grad_hook(h))
    try:
        run_backward()
    finally:
        for hk in hooks:
            hk.remove()
        with torch.no_grad():
            sd = model.state_dict()
            for k, v in saved.items():
                sd[k].copy_(v)
        for p in params:
            p.grad = None
    order += [p for p in params if id(p) not in seen]
    return order
