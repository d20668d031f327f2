"""Minimal observation/action space types (gym is not a dependency).

The reference describes observations, actions and the inference-time
``network_state`` with ``gym.spaces`` (``distribute_train.py:28-40``,
``pytorch_robotics_transformer/transformer_network.py:105-123``).  Only a small
part of that API is used: ``shape``, ``low``/``high``, ``n``, ``nvec``,
``sample()``, ordered ``keys()`` and item access.  This module provides exactly
that surface, so the framework runs without gym while keeping the same
constructor signatures (``Box(low, high, shape, dtype)``, ``Discrete(n)``,
``MultiDiscrete(nvec)``, ``Dict(mapping)``).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict as _TDict, Mapping, Optional, Sequence, Union

import numpy as np

__all__ = ["Space", "Box", "Discrete", "MultiDiscrete", "Dict", "batched_space_sampler", "np_to_tensor"]

_rng = np.random.default_rng()


class Space:
    shape: tuple = ()
    dtype = None

    def sample(self):  # pragma: no cover - abstract
        raise NotImplementedError

    def contains(self, x) -> bool:  # pragma: no cover - abstract
        raise NotImplementedError


class Box(Space):
    """A (possibly unbounded) box in R^n."""

    def __init__(self, low, high, shape: Optional[Sequence[int]] = None, dtype=np.float32):
        self.dtype = np.dtype(dtype)
        if shape is None:
            shape = np.broadcast(np.asarray(low), np.asarray(high)).shape
        self.shape = tuple(int(s) for s in shape)
        self.low = np.broadcast_to(np.asarray(low, dtype=self.dtype), self.shape).copy()
        self.high = np.broadcast_to(np.asarray(high, dtype=self.dtype), self.shape).copy()

    def sample(self):
        lo, hi = self.low.astype(np.float64), self.high.astype(np.float64)
        bounded_lo, bounded_hi = np.isfinite(lo), np.isfinite(hi)
        out = np.empty(self.shape, dtype=np.float64)
        both = bounded_lo & bounded_hi
        out[both] = _rng.uniform(lo[both], hi[both])
        unb = ~bounded_lo & ~bounded_hi
        out[unb] = _rng.normal(size=int(unb.sum()))
        lo_only = bounded_lo & ~bounded_hi
        out[lo_only] = lo[lo_only] + _rng.exponential(size=int(lo_only.sum()))
        hi_only = ~bounded_lo & bounded_hi
        out[hi_only] = hi[hi_only] - _rng.exponential(size=int(hi_only.sum()))
        return out.astype(self.dtype)

    def contains(self, x) -> bool:
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self):
        return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"


class Discrete(Space):
    def __init__(self, n: int):
        self.n = int(n)
        self.shape = ()
        self.dtype = np.dtype(np.int64)

    def sample(self):
        return np.int64(_rng.integers(0, self.n))

    def contains(self, x) -> bool:
        return 0 <= int(x) < self.n

    def __repr__(self):
        return f"Discrete({self.n})"


class MultiDiscrete(Space):
    def __init__(self, nvec):
        self.nvec = np.asarray(nvec, dtype=np.int64)
        self.shape = self.nvec.shape
        self.dtype = np.dtype(np.int64)

    def sample(self):
        return (_rng.random(self.shape) * self.nvec).astype(np.int64)

    def contains(self, x) -> bool:
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= 0) and np.all(x < self.nvec))

    def __repr__(self):
        return f"MultiDiscrete({self.nvec.tolist()})"


class Dict(Space):
    """Ordered mapping of spaces.  Like gym, a plain dict is sorted by key
    unless it is an ``OrderedDict`` (the reference relies on OrderedDict to fix
    the action-token order, ``distribute_train.py:35-40``)."""

    def __init__(self, spaces: Union[Mapping[str, Space], None] = None, **kwargs):
        if spaces is None:
            spaces = kwargs
        if isinstance(spaces, OrderedDict):
            self.spaces = OrderedDict(spaces)
        else:
            self.spaces = OrderedDict(sorted(spaces.items()))
        self.shape = None

    def keys(self):
        return self.spaces.keys()

    def items(self):
        return self.spaces.items()

    def values(self):
        return self.spaces.values()

    def __getitem__(self, k):
        return self.spaces[k]

    def __contains__(self, k):
        return k in self.spaces

    def __iter__(self):
        return iter(self.spaces)

    def __len__(self):
        return len(self.spaces)

    def sample(self):
        return OrderedDict((k, s.sample()) for k, s in self.spaces.items())

    def contains(self, x) -> bool:
        return all(k in x and s.contains(x[k]) for k, s in self.spaces.items())

    def __repr__(self):
        return "Dict(" + ", ".join(f"{k}: {v}" for k, v in self.spaces.items()) + ")"


def batched_space_sampler(space: Dict, batch_size: int) -> _TDict[str, np.ndarray]:
    """Stack ``batch_size`` samples of every entry of ``space``
    (same contract as ``tokenizers/utils.py:8-17`` in the reference)."""
    samples = [space.sample() for _ in range(batch_size)]
    return {k: np.stack([s[k] for s in samples], axis=0) for k in samples[0].keys()}


def np_to_tensor(sample_dict, device="cpu"):
    """Move every value of ``sample_dict`` to a torch tensor on ``device``
    (``tokenizers/utils.py:20-26``; the device defaults to CPU here)."""
    import torch

    return {k: torch.as_tensor(np.asarray(v)).to(device) for k, v in sample_dict.items()}
