"""Process-group bootstrap: one process per GPU, RCCL over xGMI.

The reference delegates all of this to Lightning's ``DDPStrategy`` which
re-executes the script per GPU (``distribute_train.py:231-238``).  Here the
launcher is ``torchrun`` (or any launcher that exports RANK / WORLD_SIZE /
LOCAL_RANK / MASTER_ADDR / MASTER_PORT); on ROCm the ``nccl`` backend of
torch.distributed *is* RCCL.  CPU runs (tests) use ``gloo``.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: Optional[str] = None

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world_size > 1


_CTX = DistContext()


def context() -> DistContext:
    return _CTX


def default_device() -> torch.device:
    """The initialised context's device, else cuda:current if a GPU is visible, else CPU."""
    if _CTX.device.type != "cpu" or _CTX.backend is not None:
        return _CTX.device
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return _CTX.device


def env_world() -> tuple:
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", 0))))


def pg_world1() -> bool:
    """``RT1_PG_WORLD1=1``: create the torch process group (RCCL on a GPU) even for ONE rank and run the bucketed DP
    path on it.  The one-GPU rehearsal of exactly what ``bench.py --gpus N`` runs for N > 1 (ProcessGroup all-reduces
    between graph-segment replays), not only of the native communicator."""
    return os.environ.get("RT1_PG_WORLD1") == "1"


def init_distributed(device: str = "auto", backend: Optional[str] = None, timeout_s: int = 600) -> DistContext:
    """Initialise (idempotently) from the launcher's environment.

    device: ``auto`` (GPU if visible), ``gpu``/``cuda`` or ``cpu``.
    """
    global _CTX
    rank, world, local = env_world()
    want_gpu = device in ("gpu", "cuda") or (device == "auto" and torch.cuda.is_available())
    if want_gpu:
        torch.cuda.set_device(local % max(torch.cuda.device_count(), 1))
        dev = torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    if (world > 1 or pg_world1()) and not dist.is_initialized():
        # RT1_DIST_BACKEND=gloo lets several ranks share one GPU (RCCL needs one device per rank): used to
        # rehearse the multi-rank bench / trainer paths on a one-GPU box
        backend = backend or os.environ.get("RT1_DIST_BACKEND") or ("nccl" if dev.type == "cuda" else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(**kw)
    _CTX = DistContext(rank, world, local, dev, backend if dist.is_initialized() else None)
    return _CTX


def barrier():
    if dist.is_initialized():
        if _CTX.backend == "nccl":
            dist.barrier(device_ids=[_CTX.device.index])
        else:
            dist.barrier()


def all_reduce_mean(t: torch.Tensor) -> torch.Tensor:
    if dist.is_initialized() and dist.get_world_size() > 1:
        t = t.clone()
        dist.all_reduce(t)
        t /= dist.get_world_size()
    return t


def all_reduce_max(x: float) -> float:
    if dist.is_initialized() and dist.get_world_size() > 1:
        t = torch.tensor([float(x)], device=_CTX.device if _CTX.backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())
    return float(x)


def all_gather_floats(xs) -> list:
    """Every rank's list of floats (same length on all ranks) -> [world][len] on every rank."""
    xs = [float(x) for x in xs]
    if dist.is_initialized() and dist.get_world_size() > 1:
        dev = _CTX.device if _CTX.backend == "nccl" else "cpu"
        t = torch.tensor(xs, device=dev, dtype=torch.float64)
        out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(out, t)
        return [o.cpu().tolist() for o in out]
    return [xs]


def all_gather_objects(obj) -> list:
    """Every rank's picklable ``obj`` -> [world] on every rank (host-side metadata, e.g. device identities)."""
    if dist.is_initialized() and dist.get_world_size() > 1:
        out = [None] * dist.get_world_size()
        dist.all_gather_object(out, obj)
        return out
    return [obj]


def all_true(flag: bool) -> bool:
    """Logical AND of a per-rank flag over all ranks."""
    if dist.is_initialized() and dist.get_world_size() > 1:
        dev = _CTX.device if _CTX.backend == "nccl" else "cpu"
        t = torch.tensor([0.0 if flag else 1.0], device=dev, dtype=torch.float64)
        dist.all_reduce(t)
        return float(t.item()) == 0.0
    return bool(flag)


def broadcast_object(obj, src: int = 0):
    if dist.is_initialized() and dist.get_world_size() > 1:
        lst = [obj]
        dist.broadcast_object_list(lst, src=src, device=_CTX.device if _CTX.backend == "nccl" else None)
        return lst[0]
    return obj


def shutdown():
    if dist.is_initialized():
        dist.destroy_process_group()
