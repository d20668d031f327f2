"""hipGraph capture of a data-parallel step as a chain of graph segments cut at gradient-bucket boundaries.

The reference overlaps its gradient all-reduce with backward through DDP's autograd hooks
(``/root/reference/distribute_train.py:235``).  A single captured hipGraph of forward+backward cannot do that
without capturing the collectives themselves, and RCCL kernels inside a replayed graph are a hang risk we do not
take.  Instead the forward+backward is captured as K graphs sharing ONE memory pool:

    segment 0 = forward + backward up to the moment bucket b0's last gradient lands (+ its gather copy)
    segment 1 = backward until bucket b1 completes (+ gather) ...
    segment K-1 = the rest of backward + the remaining gathers

A replay runs ``seg_0.replay(); all_reduce(b0) on the comm stream; seg_1.replay(); all_reduce(b1); ...`` so each
bucket's RCCL ring runs on its own stream while the next segment's backward kernels run on the compute stream:
the same overlap DDP gets, with every compute kernel still replayed from a graph (about 10-15 us of host
overhead per segment; RT-1 has ~5 buckets of 32 MB).

The cut happens inside the post-accumulate-grad hook that completes a bucket (``parallel.ddp`` capture mode):
the hook runs on autograd's device thread, so the segments are captured in ``relaxed`` mode (a capture may end on
a different thread than the one that began it) and always on the one side stream the whole capture uses.
Segments must be replayed in capture order (they share the pool) -- :meth:`replay_with` is the only way in.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Tuple

import torch

_LEAKED: List = []


class SegmentedCapture:
    def __init__(self, stream: torch.cuda.Stream, mode: str = "relaxed"):
        self.stream = stream
        self.mode = mode
        self.pool = None
        self.segments: List[Tuple[torch.cuda.CUDAGraph, List[int]]] = []
        self._cur: Optional[torch.cuda.CUDAGraph] = None
        self._ready: List[int] = []
        self.expected_last: Optional[int] = None   # number of buckets; the final one is not cut (no empty tail)
        self._done = 0

    # -- capture side ------------------------------------------------------------------------------------------
    def begin(self):
        if self.pool is None:
            self.pool = torch.cuda.graph_pool_handle()     # one private pool shared by every segment
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(self.stream):
            g.capture_begin(pool=self.pool, capture_error_mode=self.mode)
        self._cur = g
        self._ready = []

    def bucket_ready(self, index: int):
        """Called (from a gradient hook) once bucket ``index`` is gathered: close the segment here."""
        self._ready.append(index)
        self._done += 1
        if self.expected_last is not None and self._done >= self.expected_last:
            return            # last bucket: keep capturing; it is issued after the final segment
        self._close()
        self.begin()

    def _close(self):
        with torch.cuda.stream(self.stream):
            self._cur.capture_end()
        self.segments.append((self._cur, self._ready))
        self._cur = None
        self._ready = []

    def end(self, extra_buckets: Optional[List[int]] = None):
        if self._cur is None:
            return
        self._ready += [b for b in (extra_buckets or []) if b not in self._ready]
        self._close()

    def abort(self):
        """Best effort after an exception mid-capture: end the open capture so the stream is usable again."""
        if self._cur is not None:
            try:
                with torch.cuda.stream(self.stream):
                    self._cur.capture_end()
            except Exception:
                # never let a half-captured graph's destructor run (it aborts the process): keep it alive
                _LEAKED.append(self._cur)
            self._cur = None

    # -- replay side -------------------------------------------------------------------------------------------
    def replay_with(self, on_buckets: Callable[[List[int]], None]):
        for g, buckets in self.segments:
            g.replay()
            if buckets:
                on_buckets(buckets)

    @property
    def num_segments(self) -> int:
        return len(self.segments)
