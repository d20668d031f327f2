"""HBM-resident training frames: the input path with no per-step frame traffic over PCIe.

The host-gather path (``data.shards.ShardBatchLoader``) copies every frame of a batch from the page cache into pinned
memory and over PCIe each step: at the bench config (128 windows x 6 frames of 360x640x3) that is 531 MB per batch,
~10 ms of H2D per rank and, on an 8-GPU node, ~42 GB/s of host memcpy for all ranks together
(``profiles/r3_realdata_shard_train_300_b128.log``, ``profiles/r4_loader_8rank_cpu.log``).  An MI355X holds 288 GB of
HBM3E and RT-1 trains in a fraction of it, so this path keeps the frames where the model reads them:

* **Assign** -- each rank owns a seeded random subset of episodes, balanced by frame count (:func:`assign_episodes`:
  shuffle, then longest-first greedy onto the least-loaded rank).  Episodes of a Language-Table shard are stored in
  collection order; a contiguous split would give rank 0 (whose BN running statistics are the ones broadcast, kept in
  checkpoints and used at eval) one end of that order.  A random deal gives every rank an i.i.d. sample of episodes.
  The block-to-block split (8,000 episodes, ~343k frames of 360x640, ~237 GB raw; ``SURVEY.md`` §2.2 D1) is ~30 GB
  per rank on 8 GPUs.
* **Load once** -- :class:`ResidentShard` streams the rank's episodes (runs of consecutive owned episodes are read as
  one range) from the memory-mapped shard into one ``[F, h, w, 3]`` uint8 device tensor through two pinned staging buffers (the H2D of one chunk overlaps the read of the
  next), plus the per-frame instruction embedding / action / terminal flag.
* **Per step** -- :class:`ResidentBatchLoader` only plans a batch on the host: window -> frame rows (left-padded at the
  episode start exactly like ``EmbodiedIntelligenceDataset``, ``/root/reference/load_np_dataset.py:49-74``) and one
  random crop box per frame (``DecodeAndRandomResizedCrop``, ``:8-39``).  ~18 KB per batch cross PCIe.  On the device,
  :func:`decode_resident` gathers and crops+resizes the frames in ONE kernel (``crop_resize_gather_u8``,
  ``csrc/kernels/imgproc.hip``: Pillow-exact bilinear) and gathers the per-frame vectors with ``index_select``.

Sampling: every epoch visits each of the rank's windows once in a fresh random order (seeded by ``seed + epoch``), and
all ranks run the same number of batches (the minimum over ranks, computed from the shard metadata alone, so no
collective is needed).  Versus ``DistributedSampler`` (global shuffle, then a split) the assignment of windows to
ranks is fixed for the run (re-dealing it per epoch would re-upload ~30 GB per rank); each epoch still covers the
whole dataset once across ranks, and the deal itself is random (``seed``), not the shard's storage order.
"""
from __future__ import annotations

import time
from typing import Dict, Iterator, List, Optional, Tuple

import numpy as np
import torch

from .shards import Shard, crop_boxes, _pil_crop_resize, gpu_crop_supported


def partition_episodes(lengths: np.ndarray, world: int) -> List[Tuple[int, int]]:
    """Contiguous episode ranges ``[e_lo, e_hi)`` per rank with about ``total / world`` frames each (cuts at the episode
    boundary nearest each ideal cut).  Every rank gets at least one episode when there are enough.  Kept for tools that
    want storage-order ranges; the training path uses :func:`assign_episodes`."""
    lengths = np.asarray(lengths, np.int64)
    E = len(lengths)
    if world <= 1:
        return [(0, E)]
    if E < world:
        raise ValueError(f"{E} episodes cannot be split over {world} ranks")
    cum = np.concatenate([[0], np.cumsum(lengths)])
    total = cum[-1]
    cuts = [0]
    for r in range(1, world):
        ideal = total * r / world
        e = int(np.argmin(np.abs(cum - ideal)))
        e = max(e, cuts[-1] + 1)                       # at least one episode per rank
        e = min(e, E - (world - r))                    # leave one for each later rank
        cuts.append(e)
    cuts.append(E)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def assign_episodes(lengths: np.ndarray, world: int, seed: int = 0) -> List[np.ndarray]:
    """Sorted episode indices per rank: a seeded random deal balanced by frame count.

    The episodes are shuffled with ``seed``, then dealt longest first (stable, so equal lengths keep the shuffled
    order) onto the rank with the fewest frames so far (ties: the lowest rank).  Deterministic from (lengths, world,
    seed) alone, so every rank computes the same deal without a collective.  Raises ValueError when there are fewer
    episodes than ranks (callers in 'auto' mode fall back to the host path)."""
    lengths = np.asarray(lengths, np.int64)
    E = len(lengths)
    if world <= 1:
        return [np.arange(E, dtype=np.int64)]
    if E < world:
        raise ValueError(f"{E} episodes cannot be split over {world} ranks")
    perm = np.random.default_rng(int(seed) * 2_654_435_761 % (2 ** 32) + 17).permutation(E)
    order = perm[np.argsort(-lengths[perm], kind="stable")]
    load = np.zeros(world, np.int64)
    owner = np.empty(E, np.int64)
    for e in order:
        r = int(np.argmin(load))
        owner[e] = r
        load[r] += lengths[e]
    return [np.nonzero(owner == r)[0].astype(np.int64) for r in range(world)]


def _runs(eps: np.ndarray) -> List[Tuple[int, int]]:
    """Maximal runs [a, b) of consecutive values in a sorted index array."""
    if len(eps) == 0:
        return []
    brk = np.nonzero(np.diff(eps) != 1)[0]
    starts = np.concatenate([[0], brk + 1])
    ends = np.concatenate([brk + 1, [len(eps)]])
    return [(int(eps[a]), int(eps[b - 1]) + 1) for a, b in zip(starts, ends)]


class ResidentShard:
    """One rank's episodes of a packed shard, resident on ``device`` (frames + per-frame vectors).

    ``seed`` picks the episode deal (:func:`assign_episodes`); every rank must pass the same one."""

    def __init__(self, path: str, device, rank: int = 0, world: int = 1, chunk_mb: float = 256.0,
                 max_gb: Optional[float] = None, seed: int = 0):
        self.shard = Shard(path)
        self.device = torch.device(device)
        self.rank, self.world = rank, world
        off, ln = self.shard.offsets, self.shard.lengths
        self.assignment = assign_episodes(ln, world, seed)
        self.episodes = self.assignment[rank]
        # global frame ranges [f_a, f_b) of the rank's runs of consecutive episodes, in storage order
        self.frame_runs = [(int(off[a]), int(off[b - 1] + ln[b - 1])) for a, b in _runs(self.episodes)]
        F = sum(b - a for a, b in self.frame_runs)
        # global frame row -> row of the resident table (-1: another rank's frame)
        self.row_map = np.full(int(ln.sum()), -1, np.int64)
        pos = 0
        for a, b in self.frame_runs:
            self.row_map[a:b] = np.arange(pos, pos + b - a)
            pos += b - a
        fshape = self.shard.frame_shape
        self.frame_bytes = int(np.prod(fshape))
        need_gb = F * self.frame_bytes / 2 ** 30
        if max_gb is not None and need_gb > max_gb:
            raise MemoryError(f"rank {rank}: {F} frames = {need_gb:.1f} GB exceed the HBM data budget {max_gb} GB")
        t0 = time.perf_counter()
        self.frames = torch.empty((F,) + fshape, dtype=torch.uint8, device=self.device)
        if self.device.type != "meta":          # meta: planning only (tools/loader_bench.py host-side timing)
            self._load_frames(chunk_mb)
        rows = np.concatenate([np.arange(a, b) for a, b in self.frame_runs]) if self.frame_runs else np.zeros(0, int)
        self.instruction = torch.from_numpy(np.ascontiguousarray(self.shard.instruction[rows])).to(self.device)
        self.action = torch.from_numpy(np.ascontiguousarray(self.shard.action[rows])).to(self.device)
        self.is_terminal = torch.from_numpy(self.shard.is_terminal[rows].astype(np.int64)).to(self.device)
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        self.load_s = time.perf_counter() - t0
        owned = np.zeros(len(ln), bool)
        owned[self.episodes] = True
        self.window_ids = np.nonzero(owned[self.shard.windows[:, 0]])[0]
        # windows per rank, from the metadata alone (identical on every rank)
        self.windows_per_rank = [int(np.sum(ln[eps])) for eps in self.assignment]

    def _chunks(self, per: int):
        """(table row, global frame row, count) pieces of at most ``per`` frames, run by run."""
        pos = 0
        for a, b in self.frame_runs:
            for s in range(a, b, per):
                n = min(per, b - s)
                yield pos + (s - a), s, n
            pos += b - a

    def _load_frames(self, chunk_mb: float):
        fr = self.shard.frames
        per = max(1, int(chunk_mb * 2 ** 20) // self.frame_bytes)
        if self.device.type != "cuda":
            for dst, src, n in self._chunks(per):
                self.frames[dst:dst + n].copy_(torch.from_numpy(np.array(fr[src:src + n])))
            return
        # two pinned staging buffers: the H2D of chunk i runs on a side stream while chunk i+1 is read from disk
        stage = [torch.empty((per,) + tuple(fr.shape[1:]), dtype=torch.uint8, pin_memory=True) for _ in range(2)]
        done = [None, None]
        st = torch.cuda.Stream(self.device)
        for i, (dst, src, n) in enumerate(self._chunks(per)):
            k = i % 2
            if done[k] is not None:
                done[k].synchronize()
            np.copyto(stage[k].numpy()[:n], fr[src:src + n])
            with torch.cuda.stream(st):
                self.frames[dst:dst + n].copy_(stage[k][:n], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(st)
            done[k] = ev
        st.synchronize()

    @property
    def nbytes(self) -> int:
        return self.frames.numel() + 4 * (self.instruction.numel() + self.action.numel()) + 8 * self.is_terminal.numel()

    def global_rows(self, local: np.ndarray) -> np.ndarray:
        """Resident-table rows -> the shard's global frame rows (tests / tools)."""
        inv = np.concatenate([np.arange(a, b) for a, b in self.frame_runs])
        return inv[local]

    def local_rows(self, widx: np.ndarray, T: int) -> np.ndarray:
        """[len(widx), T] frame rows of windows, in this rank's resident table."""
        rows = self.row_map[self.shard.frame_index(widx, T)]
        if rows.size and rows.min() < 0:
            raise IndexError("window outside this rank's resident episodes")
        return rows


class ResidentBatchLoader:
    """Per-batch plans over a :class:`ResidentShard`: ``{"plan_rows": [B, T] int64, "crop_boxes": [B, T, 4] int32}``
    (pinned when CUDA is present); :func:`decode_resident` turns a plan into the model's batch on the device."""

    def __init__(self, resident: ResidentShard, batch_size: int, seq_len: int, crop_factor: Optional[float] = 0.95,
                 shuffle: bool = True, seed: int = 0, drop_last: bool = True, pin: Optional[bool] = None):
        self.res = resident
        self.B, self.T = int(batch_size), int(seq_len)
        self.factor = crop_factor
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.pin = (resident.device.type == "cuda") if pin is None else pin
        self.epoch = 0
        self.stats = {"batches": 0, "fill_s": 0.0, "gather_s": 0.0, "wait_s": 0.0}

    def set_epoch(self, epoch: int):
        self.epoch = int(epoch)

    def __len__(self):
        # the same count on every rank (collectives run per step): the smallest rank's share
        n = min(self.res.windows_per_rank)
        return n // self.B if self.drop_last else -(-n // self.B)

    def __iter__(self) -> Iterator[Dict]:
        ids = self.res.window_ids
        if self.shuffle:
            ids = ids[np.random.default_rng((self.seed + self.epoch) * 7919 + self.res.rank).permutation(len(ids))]
        rng = np.random.default_rng((self.seed + 1) * 1_000_003 + self.epoch * 7919 + self.res.rank)
        h0, w0 = self.res.shard.frame_shape[:2]
        st = self.stats = {"batches": 0, "fill_s": 0.0, "gather_s": 0.0, "wait_s": 0.0}
        for i in range(len(self)):
            t0 = time.perf_counter()
            widx = ids[i * self.B:(i + 1) * self.B]
            if len(widx) < self.B and not self.drop_last:     # short last batch: wrap (DistributedSampler-style)
                widx = np.concatenate([widx, ids[:self.B - len(widx)]])
            b = len(widx)
            rows = torch.empty((b, self.T), dtype=torch.int64, pin_memory=self.pin)
            boxes = torch.empty((b, self.T, 4), dtype=torch.int32, pin_memory=self.pin)
            rows.numpy()[:] = self.res.local_rows(widx, self.T)
            boxes.numpy()[:] = crop_boxes(rng, b * self.T, h0, w0, self.factor).reshape(b, self.T, 4)
            st["fill_s"] += time.perf_counter() - t0
            st["batches"] += 1
            yield {"plan_rows": rows, "crop_boxes": boxes}


def decode_resident(res: ResidentShard, batch: Dict, H: int, W: int) -> Dict:
    """Plan -> the model's batch (``image`` [B, T, 3, H, W] uint8, embeddings, action labels) from the resident
    tables; other batches pass through unchanged."""
    if "plan_rows" not in batch:
        return batch
    rows, boxes = batch["plan_rows"], batch["crop_boxes"]
    B, T = rows.shape
    flat = rows.reshape(-1).to(res.device)
    bx = boxes.reshape(-1, 4).to(res.device)
    if res.frames.is_cuda and gpu_crop_supported(res.frames.shape[1], res.frames.shape[2], H, W):
        from ..ops import load
        img = load().crop_resize_gather_u8(res.frames, flat.contiguous(), bx.contiguous(), H, W)
    else:
        img = _pil_crop_resize(res.frames.index_select(0, flat.cpu() if not res.frames.is_cuda else flat), bx, H, W)
        img = img.to(res.device)
    return {"action_label": {"terminate_episode": res.is_terminal.index_select(0, flat).view(B, T),
                             "action": res.action.index_select(0, flat).view(B, T, 2)},
            "train_observation": {"image": img.view(B, T, 3, H, W),
                                  "natural_language_embedding": res.instruction.index_select(0, flat).view(B, T, -1)}}
