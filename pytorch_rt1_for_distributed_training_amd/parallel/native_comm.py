"""Native RCCL communicator (``csrc/comm.cpp``) for the data-parallel gradient path.

``torch.distributed`` is used only to bootstrap: rank 0 creates the RCCL unique id and broadcasts it
over the existing process group; afterwards every bucket all-reduce / parameter broadcast goes
straight to RCCL on the communicator's own pooled HIP stream (default priority; ``RT1_COMM_STREAM=high``
for a high-priority one) (one process per MI355X,
xGMI transport picked by RCCL).  Collectives are ordered after the work already queued on the
caller's stream and their ``Work.wait()`` is a stream-level wait, so the host never blocks.

A watchdog thread in the C++ layer aborts the communicator (``ncclCommAbort``) and exits the process with code 75
when a collective stays pending longer than ``timeout_s`` (env ``RT1_COMM_TIMEOUT``, default 600 s) or RCCL
reports an asynchronous error, so a dead peer ends the job instead of hanging every rank.

Select with ``TrainEngine(..., comm="native")`` / ``distribute_train.py --comm native`` /
``bench.py --comm native``; the default stays ``torch`` (ProcessGroup over the same RCCL).
"""
from __future__ import annotations

from typing import Optional

import os

import torch
import torch.distributed as dist


def _timeout(t):
    return float(os.environ.get("RT1_COMM_TIMEOUT", 600.0)) if t is None else float(t)


class NativeComm:
    def __init__(self, process_group=None, device: Optional[int] = None, timeout_s: Optional[float] = None):
        from ..ops import load
        ext = load()
        if not dist.is_initialized():
            raise RuntimeError("NativeComm needs an initialised torch.distributed process group to bootstrap")
        self.rank = dist.get_rank(process_group)
        self.world = dist.get_world_size(process_group)
        dev = torch.cuda.current_device() if device is None else int(device)
        uid = [ext.comm.unique_id() if self.rank == 0 else None]
        dist.broadcast_object_list(uid, src=0, group=process_group)
        self._c = ext.comm.Communicator(uid[0], self.world, self.rank, dev, _timeout(timeout_s))

    @classmethod
    def single(cls, device: int = 0, timeout_s: Optional[float] = None) -> "NativeComm":
        """world = 1 communicator without a process group (self-test / single-GPU runs)."""
        from ..ops import load
        ext = load()
        self = cls.__new__(cls)
        self.rank, self.world = 0, 1
        self._c = ext.comm.Communicator(ext.comm.unique_id(), 1, 0, int(device), _timeout(timeout_s))
        return self

    @property
    def timed_out(self) -> bool:
        return self._c.timed_out()

    def all_reduce_(self, t: torch.Tensor, op: str = "sum"):
        return self._c.all_reduce_(t, op)

    def all_reduce_coalesced_(self, ts, op: str = "sum"):
        return self._c.all_reduce_coalesced_(list(ts), op)

    def broadcast_(self, t: torch.Tensor, root: int = 0):
        w = self._c.broadcast_(t, root)
        w.wait()       # later compute on the caller's stream reads t: order it after the broadcast
        return w

    def destroy(self):
        self._c.destroy()
