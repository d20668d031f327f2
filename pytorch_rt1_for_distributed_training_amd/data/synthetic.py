"""Synthetic RT-1 batches of the real shapes (no dataset / network access).

A sample is one T-frame window exactly as ``EmbodiedIntelligenceDataset``
emits it (``load_np_dataset.py:106-116``): images (T,3,H,W), a 512-d sentence
embedding per frame, ``terminate_episode`` (T,) in {0,1} and a 2-d action
(T,2) in [-0.1, 0.1].  Frames are kept as uint8 (what the Language-Table
dataset stores and what the reference's PIL transform produces before /255),
so host->device traffic is 4x smaller than float32; the /255 happens inside
the fused stem.
"""
from __future__ import annotations

from typing import Dict, Iterator, Optional

import torch


def make_batch(batch_size: int, seq_len: int, height: int, width: int, device="cpu", uint8: bool = True,
               generator: Optional[torch.Generator] = None, pin: bool = False) -> Dict:
    g = generator
    if uint8:
        img = torch.randint(0, 256, (batch_size, seq_len, 3, height, width), dtype=torch.uint8, generator=g)
    else:
        img = torch.rand(batch_size, seq_len, 3, height, width, generator=g)
    emb = torch.randn(batch_size, 1, 512, generator=g).expand(batch_size, seq_len, 512).contiguous()
    term = torch.zeros(batch_size, seq_len, dtype=torch.long)
    term[:, -1] = torch.randint(0, 2, (batch_size,), generator=g)
    act = (torch.rand(batch_size, seq_len, 2, generator=g) * 0.2 - 0.1)
    batch = {"train_observation": {"image": img, "natural_language_embedding": emb},
             "action_label": {"terminate_episode": term, "action": act}}
    if pin:
        batch = _apply(batch, lambda t: t.pin_memory())
    if str(device) != "cpu":
        batch = _apply(batch, lambda t: t.to(device, non_blocking=True))
    return batch


def _apply(batch, fn):
    if isinstance(batch, dict):
        return {k: _apply(v, fn) for k, v in batch.items()}
    return fn(batch)


class SyntheticDataset(torch.utils.data.Dataset):
    """Deterministic per-index synthetic windows (for DataLoader / sampler tests)."""

    def __init__(self, length: int, seq_len: int, height: int, width: int, seed: int = 0, uint8: bool = False):
        self.length, self.seq_len, self.h, self.w, self.seed, self.uint8 = length, seq_len, height, width, seed, uint8

    def __len__(self):
        return self.length

    def __getitem__(self, idx):
        g = torch.Generator().manual_seed(self.seed * 1000003 + idx)
        b = make_batch(1, self.seq_len, self.h, self.w, uint8=self.uint8, generator=g)
        return _apply(b, lambda t: t[0])


class SyntheticStream:
    """Infinite stream of pinned host batches, a small ring re-used (content
    does not matter for throughput; the H2D copy still happens every step)."""

    def __init__(self, batch_size, seq_len, height, width, ring: int = 2, uint8: bool = True, seed: int = 0):
        g = torch.Generator().manual_seed(seed)
        pin = torch.cuda.is_available()
        self.ring = [make_batch(batch_size, seq_len, height, width, uint8=uint8, generator=g, pin=pin)
                     for _ in range(ring)]
        self.i = 0

    def __iter__(self) -> Iterator[Dict]:
        return self

    def __next__(self) -> Dict:
        b = self.ring[self.i % len(self.ring)]
        self.i += 1
        return b
