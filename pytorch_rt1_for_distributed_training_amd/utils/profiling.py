"""Tracing helpers: roctx ranges (visible in rocprofv3 ``--marker-trace``) and
device-accurate step timers.  The reference has no tracing on its RT-1 path
(SURVEY §5); these are additive.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import time
from typing import Dict, List, Optional

import torch

_ROCTX = None


def _roctx():
    global _ROCTX
    if _ROCTX is None:
        _ROCTX = False
        for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                _ROCTX = lib
                break
            except OSError:
                continue
    return _ROCTX


@contextlib.contextmanager
def range_push(name: str):
    lib = _roctx() if os.environ.get("RT1_ROCTX", "0") == "1" else None
    if lib:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib:
            lib.roctxRangePop()


class StepTimer:
    """Wall-clock per step with device synchronisation at the edges only."""

    def __init__(self, device: torch.device):
        self.device = device
        self.times: List[float] = []
        self._t0: Optional[float] = None

    def _sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def start(self):
        self._sync()
        self._t0 = time.perf_counter()

    def stop(self) -> float:
        self._sync()
        dt = time.perf_counter() - self._t0
        self.times.append(dt)
        return dt

    def summary(self) -> Dict[str, float]:
        if not self.times:
            return {}
        ts = sorted(self.times)
        return {"mean_ms": 1e3 * sum(ts) / len(ts), "median_ms": 1e3 * ts[len(ts) // 2], "min_ms": 1e3 * ts[0]}
