"""Dataset statistics and normalisers for behaviour cloning.

Reference: ``language_table/train/normalization.py:28-330`` -- Chan's parallel mean/variance over sampled
batches (``ChanRunningStatistics``), per-dimension action min/max, and Std / MinMax (de)normalisers applied to
the non-image observation keys and the actions.  Process 0 computes the statistics and the others wait for them
(``input_pipeline_rlds.py:195-234``); here :func:`broadcast_stats` shares rank 0's numbers over the process group.
"""
from __future__ import annotations

from typing import Dict, Iterable, Optional

import numpy as np


class ChanStats:
    """Running mean / M2 over the last dimension, merged batch by batch (Chan et al. parallel algorithm)."""

    def __init__(self):
        self.n = 0
        self.mean = None
        self.m2 = None

    def update(self, sample: np.ndarray):
        x = np.asarray(sample, np.float64).reshape(-1, np.asarray(sample).shape[-1])
        nb = x.shape[0]
        mb = x.mean(0)
        m2b = ((x - mb) ** 2).sum(0)
        if self.n == 0:
            self.n, self.mean, self.m2 = nb, mb, m2b
            return
        n = self.n + nb
        delta = mb - self.mean
        self.mean = self.mean + delta * nb / n
        self.m2 = self.m2 + m2b + delta ** 2 * self.n * nb / n
        self.n = n

    @property
    def variance(self) -> np.ndarray:
        return self.m2 / max(self.n, 1)

    @property
    def std(self) -> np.ndarray:
        return np.sqrt(self.variance)


def compute_dataset_statistics(batches: Iterable, num_samples: int, skip_keys=("rgb", "instruction",
                                                                                "instruction_embedding")) -> Dict:
    """batches yield (obs dict, action array); returns {obs: {key: {mean, std}}, action: {mean, std, min, max}}."""
    obs_stats: Dict[str, ChanStats] = {}
    act = ChanStats()
    amin = amax = None
    seen = 0
    for obs, action in batches:
        for k, v in obs.items():
            if k in skip_keys:
                continue
            obs_stats.setdefault(k, ChanStats()).update(v)
        a = np.asarray(action, np.float64).reshape(-1, np.asarray(action).shape[-1])
        act.update(a)
        amin = a.min(0) if amin is None else np.minimum(amin, a.min(0))
        amax = a.max(0) if amax is None else np.maximum(amax, a.max(0))
        seen += a.shape[0]
        if seen >= num_samples:
            break
    return {"obs": {k: {"mean": s.mean.astype(np.float32), "std": s.std.astype(np.float32)}
                    for k, s in obs_stats.items()},
            "action": {"mean": act.mean.astype(np.float32), "std": act.std.astype(np.float32),
                       "min": amin.astype(np.float32), "max": amax.astype(np.float32)}}


class StdNormalizer:
    def __init__(self, mean, std, eps: float = 1e-6):
        self.mean, self.std, self.eps = np.asarray(mean, np.float32), np.asarray(std, np.float32), eps

    def normalize(self, x):
        return (x - self._like(self.mean, x)) / (self._like(self.std, x) + self.eps)

    def denormalize(self, x):
        return x * (self._like(self.std, x) + self.eps) + self._like(self.mean, x)

    @staticmethod
    def _like(v, x):
        try:
            import torch
            if isinstance(x, torch.Tensor):
                return torch.as_tensor(v, dtype=x.dtype, device=x.device)
        except ImportError:  # pragma: no cover
            pass
        return v


class MinMaxNormalizer(StdNormalizer):
    """Maps [min, max] to [-1, 1]."""

    def __init__(self, vmin, vmax, eps: float = 1e-6):
        vmin, vmax = np.asarray(vmin, np.float32), np.asarray(vmax, np.float32)
        super().__init__((vmax + vmin) / 2.0, (vmax - vmin) / 2.0, eps)


def broadcast_stats(stats: Optional[Dict], src: int = 0) -> Dict:
    """Rank ``src`` computes the statistics, every rank returns the same dict."""
    from ..parallel import dist as pdist
    return pdist.broadcast_object(stats, src)
