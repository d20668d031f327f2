"""Graph-replayable dropout seeds for the HIP kernels.

Every dropout kernel (``attention.hip``, ``transformer.hip``) hashes ``salt + counter * golden``: the
salt is a host constant per call site (the i-th dropout of a forward pass), the counter an int32 on the
device that ``begin_forward`` advances with a device op.  A captured hipGraph therefore replays a
different mask on every step, and the backward regenerates exactly the forward's mask (same salt, same
counter value).  Replaces the reference's stateful ``nn.Dropout`` RNG (``transformer.py:57,117``).
"""
from __future__ import annotations

from typing import Dict

import torch

_COUNTERS: Dict[torch.device, torch.Tensor] = {}
_salt = 0


def counter(device) -> torch.Tensor:
    device = torch.device(device)
    t = _COUNTERS.get(device)
    if t is None:
        start = int(torch.randint(0, 2 ** 30, (1,)).item())   # host RNG: follows torch.manual_seed
        t = torch.full((1,), start, dtype=torch.int32, device=device)
        _COUNTERS[device] = t
    return t


def begin_forward(device):
    """Start a forward pass: advance the device counter (a captured op) and restart the salt sequence."""
    global _salt
    _salt = 0
    counter(device).add_(1)


def next_salt() -> int:
    global _salt
    _salt += 1
    return (_salt * 0x2545F491) & 0x7FFFFFFF
