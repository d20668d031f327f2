"""Double-buffered host->HBM batch prefetch on a dedicated HIP stream.

The next batch's pinned host tensors are copied with ``hipMemcpyAsync`` on a
side stream while the current step computes; the compute stream waits on an
event only when it consumes the batch, and the consumer's stream is recorded on
the buffers so the caching allocator never recycles them early.  With uint8
frames a 128-sample 300x300 window batch is 207 MB, i.e. ~4 ms of PCIe Gen5
that is fully hidden behind a step.
"""
from __future__ import annotations

from typing import Dict, Iterable, Iterator, Optional

import torch


def _map(batch, fn):
    if isinstance(batch, dict):
        return {k: _map(v, fn) for k, v in batch.items()}
    if isinstance(batch, torch.Tensor):
        return fn(batch)
    return batch


class DevicePrefetcher:
    def __init__(self, loader: Iterable[Dict], device: torch.device, depth: int = 2, transform=None):
        """``transform(batch) -> batch`` runs on the device batch right after the copy, on the prefetch stream
        (e.g. ``data.shards.decode_on_device``: GPU crop + resize of raw frames), overlapping the current step."""
        self.loader = loader
        self.transform = transform
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.stream = torch.cuda.Stream(device=self.device) if self.cuda else None
        self.depth = max(1, depth)

    def __iter__(self) -> Iterator[Dict]:
        it = iter(self.loader)
        queue = []

        def issue():
            try:
                host = next(it)
            except StopIteration:
                return False
            if not self.cuda:
                queue.append((self.transform(host) if self.transform else host, None))
                return True
            with torch.cuda.stream(self.stream):
                dev = _map(host, lambda t: t.to(self.device, non_blocking=True))
                if self.transform is not None:
                    dev = self.transform(dev)
                ev = torch.cuda.Event()
                ev.record(self.stream)
            queue.append((dev, ev))
            return True

        for _ in range(self.depth):
            if not issue():
                break
        while queue:
            batch, ev = queue.pop(0)
            if ev is not None:
                cur = torch.cuda.current_stream(self.device)
                cur.wait_event(ev)
                _map(batch, lambda t: t.record_stream(cur))
            issue()
            yield batch

    def __len__(self):
        return len(self.loader)  # type: ignore[arg-type]
