"""Packed episode shards + a batch loader that feeds raw frames to the GPU.

The reference's input path (``/root/reference/load_np_dataset.py:41-116``) re-loads a whole pickled episode per
sample and runs 6 PIL crop+resizes per sample on the CPU; at MI355X step rates (~1000 windows/s per GPU, 6 frames
each) that cannot keep up.  This path is laid out for the accelerator instead:

* **Storage** -- one shard per split: ``frames.u8`` (every frame of every episode, raw HWC uint8, back to back;
  memory-mapped, so a window is a plain slice served from the page cache) and ``meta.npz`` (episode offsets /
  lengths, per-step 512-d instruction embedding, action, terminal flag; no pickle).  ``pack_shard`` converts the
  per-episode ``.npz`` format (``data.episodes``) into it.
* **Host side** -- :class:`ShardBatchLoader` builds whole batches: window -> frame indices (left-padded with the
  episode's first step exactly like ``EmbodiedIntelligenceDataset``), one random crop box per frame (the
  ``DecodeAndRandomResizedCrop`` draw, Python rounding as Pillow's ``crop`` does), and a gather of the raw frames
  straight into a pinned buffer with a thread pool (numpy copies release the GIL).  Two batches are kept in
  flight.  Sharding across ranks and per-epoch shuffling follow ``DistributedSampler``.
* **Device side** -- :func:`decode_on_device` runs the Pillow-exact crop+bilinear-resize kernel
  (``csrc/kernels/imgproc.hip``) on the prefetch stream right after the H2D copy, producing the ``(B, T, 3, H,
  W)`` uint8 image tensor the stem reads.  On CPU it falls back to Pillow itself.
"""
from __future__ import annotations

import concurrent.futures as cf
import math
import os
import queue
import threading
import time
from typing import Dict, Iterator, List, Optional, Sequence

import numpy as np
import torch

FRAMES = "frames.u8"
META = "meta.npz"


def is_shard(path: str) -> bool:
    return os.path.exists(os.path.join(path, FRAMES)) and os.path.exists(os.path.join(path, META))


def pack_shard(src_dir: str, ids: Sequence[int], dst_dir: str) -> int:
    """Pack ``episode_{id}.npz`` files into one shard; returns the number of frames written."""
    os.makedirs(dst_dir, exist_ok=True)
    offsets, lengths, instr, action, term = [], [], [], [], []
    shape = None
    total = 0
    with open(os.path.join(dst_dir, FRAMES), "wb") as f:
        for eid in ids:
            with np.load(os.path.join(src_dir, f"episode_{eid}.npz"), allow_pickle=False) as z:
                rgb = np.ascontiguousarray(z["rgb"], dtype=np.uint8)
                if shape is None:
                    shape = rgb.shape[1:]
                elif rgb.shape[1:] != shape:
                    raise ValueError(f"episode {eid}: frame shape {rgb.shape[1:]} != {shape}")
                f.write(rgb.tobytes())
                offsets.append(total)
                lengths.append(rgb.shape[0])
                total += rgb.shape[0]
                instr.append(np.asarray(z["instruction"], np.float32))
                action.append(np.asarray(z["action"], np.float32))
                term.append(np.asarray(z["is_terminal"], bool))
    np.savez(os.path.join(dst_dir, META), offsets=np.asarray(offsets, np.int64),
             lengths=np.asarray(lengths, np.int64), episode_ids=np.asarray(list(ids), np.int64),
             instruction=np.concatenate(instr), action=np.concatenate(action), is_terminal=np.concatenate(term),
             frame_shape=np.asarray(shape, np.int64))
    return total


class Shard:
    """Read side of a packed shard (memory-mapped frames)."""

    def __init__(self, path: str):
        with np.load(os.path.join(path, META), allow_pickle=False) as z:
            meta = {k: z[k] for k in z.files}
        self.offsets = meta["offsets"]
        self.lengths = meta["lengths"]
        self.instruction = meta["instruction"]
        self.action = meta["action"]
        self.is_terminal = meta["is_terminal"]
        self.frame_shape = tuple(int(v) for v in meta["frame_shape"])
        n = int(self.lengths.sum())
        self.frames = np.memmap(os.path.join(path, FRAMES), dtype=np.uint8, mode="r", shape=(n,) + self.frame_shape)
        # one window per step of every episode, in episode order (load_np_dataset.py:49-74)
        self.windows = np.concatenate([np.stack([np.full(l, e), np.arange(l)], 1)
                                       for e, l in enumerate(self.lengths)]).astype(np.int64)

    def __len__(self):
        return len(self.windows)

    def frame_index(self, widx: np.ndarray, T: int) -> np.ndarray:
        """Global frame rows [len(widx), T] of windows: steps start-T+1 .. start, clamped at the episode's step 0."""
        ep, start = self.windows[widx, 0], self.windows[widx, 1]
        steps = start[:, None] + np.arange(T)[None, :] - (T - 1)
        steps = np.maximum(steps, 0)
        return self.offsets[ep][:, None] + steps


def crop_boxes(rng: np.random.Generator, n: int, h0: int, w0: int, factor: Optional[float]) -> np.ndarray:
    """[n, 4] int32 (x0, y0, x1, y1): ``DecodeAndRandomResizedCrop``'s draw with Pillow's crop rounding."""
    if factor is None:
        return np.tile(np.asarray([[0, 0, w0, h0]], np.int32), (n, 1))
    sh, sw = h0 * factor, w0 * factor
    oy = rng.integers(0, int(h0 - sh + 1), size=n)
    ox = rng.integers(0, int(w0 - sw + 1), size=n)
    x1 = np.round(ox + sw)            # round-half-to-even, like Python's round() in Image.crop
    y1 = np.round(oy + sh)
    return np.stack([ox, oy, x1, y1], 1).astype(np.int32)


class ShardBatchLoader:
    """Whole-batch loader over a shard: yields dicts with raw frames + crop boxes (pinned when CUDA is present).

    ``len()`` = batches per epoch for this rank; ``set_epoch`` reseeds the shuffle like DistributedSampler."""

    def __init__(self, path: str, batch_size: int, seq_len: int, crop_factor: Optional[float] = 0.95,
                 shuffle: bool = True, rank: int = 0, world: int = 1, seed: int = 0, drop_last: bool = True,
                 threads: int = 8, pin: Optional[bool] = None, prefetch: int = 2, reuse_buffers: int = 0):
        self.shard = Shard(path)
        self.B, self.T = int(batch_size), int(seq_len)
        self.factor = crop_factor
        self.shuffle, self.rank, self.world, self.seed = shuffle, rank, world, seed
        self.drop_last = drop_last
        self.threads = max(1, threads)
        self.pin = torch.cuda.is_available() if pin is None else pin
        self.prefetch = max(1, prefetch)
        # reuse_buffers = k > 0: a ring of k batch buffers instead of a fresh allocation per batch (a yielded batch
        # is then overwritten k - prefetch - 1 batches later).  Pinned buffers come from torch's caching host
        # allocator, which already recycles them safely; a fresh PAGEABLE 531 MB buffer per batch costs ~0.6 s of
        # page faults (tools/loader_bench.py models the pinned reuse on a CPU-only box with this).
        self.reuse_buffers = int(reuse_buffers)
        self._ring: List[Dict[str, torch.Tensor]] = []
        self._ring_i = 0
        self.epoch = 0
        # per-iteration input-path timing (seconds): producer fill time (gather + metadata, on the loader thread) and
        # consumer time blocked waiting for a filled batch; reset at every __iter__
        self.stats = {"batches": 0, "fill_s": 0.0, "gather_s": 0.0, "wait_s": 0.0}

    def set_epoch(self, epoch: int):
        self.epoch = int(epoch)

    def _indices(self) -> np.ndarray:
        n = len(self.shard)
        if self.shuffle:
            order = np.random.default_rng(self.seed + self.epoch).permutation(n)
        else:
            order = np.arange(n)
        per = n // self.world if self.drop_last else -(-n // self.world)
        if not self.drop_last and per * self.world > n:           # pad by wrapping, like DistributedSampler
            order = np.concatenate([order, order[: per * self.world - n]])
        return order[self.rank * per:(self.rank + 1) * per] if self.world > 1 else order[:per * self.world]

    def __len__(self):
        n = len(self._indices())
        return n // self.B if self.drop_last else -(-n // self.B)

    def _alloc(self, b: int) -> Dict[str, torch.Tensor]:
        if self.reuse_buffers > 0:
            if len(self._ring) < self.reuse_buffers:
                self._ring.append(self._new(b))
            buf = self._ring[self._ring_i % len(self._ring)]
            self._ring_i += 1
            if buf["raw"].shape[0] == b:
                return buf
        return self._new(b)

    def _new(self, b: int) -> Dict[str, torch.Tensor]:
        h, w, c = self.shard.frame_shape
        mk = lambda shape, dt: torch.empty(shape, dtype=dt, pin_memory=self.pin)
        return {"raw": mk((b, self.T, h, w, c), torch.uint8), "boxes": mk((b, self.T, 4), torch.int32),
                "emb": mk((b, self.T, 512), torch.float32), "act": mk((b, self.T, 2), torch.float32),
                "term": mk((b, self.T), torch.long)}

    def _fill(self, pool, widx: np.ndarray, rng: np.random.Generator) -> Dict:
        b = len(widx)
        buf = self._alloc(b)
        rows = self.shard.frame_index(widx, self.T)                       # [b, T]
        raw = buf["raw"].numpy()
        frames = self.shard.frames

        src = np.asarray(frames)            # plain ndarray view of the memmap (no subclass overhead)
        dst = raw.reshape((-1,) + frames.shape[1:])
        flat_rows = rows.reshape(-1)

        def gather(lo, hi):
            # one frame-sized memcpy per row: numpy releases the GIL for these, so the pool's threads copy in
            # parallel (~26 GB/s with 8 threads vs ~1.7 GB/s for np.take on the memmap, tools/loader_bench.py)
            for i in range(lo * self.T, hi * self.T):
                dst[i] = src[flat_rows[i]]

        step = max(1, -(-b // self.threads))
        tg = time.perf_counter()
        futs = [pool.submit(gather, lo, min(b, lo + step)) for lo in range(0, b, step)]
        h0, w0 = self.shard.frame_shape[:2]
        buf["boxes"].numpy()[:] = crop_boxes(rng, b * self.T, h0, w0, self.factor).reshape(b, self.T, 4)
        buf["emb"].numpy()[:] = self.shard.instruction[rows]
        buf["act"].numpy()[:] = self.shard.action[rows]
        buf["term"].numpy()[:] = self.shard.is_terminal[rows].astype(np.int64)
        for f in futs:
            f.result()
        self.stats["gather_s"] += time.perf_counter() - tg
        return {"action_label": {"terminate_episode": buf["term"], "action": buf["act"]},
                "train_observation": {"raw_frames": buf["raw"], "crop_boxes": buf["boxes"],
                                      "natural_language_embedding": buf["emb"]}}

    def __iter__(self) -> Iterator[Dict]:
        idx = self._indices()
        nb = len(self)
        rng = np.random.default_rng((self.seed + 1) * 1_000_003 + self.epoch * 7919 + self.rank)
        q: "queue.Queue" = queue.Queue(maxsize=self.prefetch)
        stop = threading.Event()
        st = self.stats = {"batches": 0, "fill_s": 0.0, "gather_s": 0.0, "wait_s": 0.0}

        def produce():
            try:
                with cf.ThreadPoolExecutor(self.threads) as pool:
                    for i in range(nb):
                        if stop.is_set():
                            return
                        t0 = time.perf_counter()
                        item = self._fill(pool, idx[i * self.B:(i + 1) * self.B], rng)
                        st["fill_s"] += time.perf_counter() - t0
                        st["batches"] += 1
                        q.put(item)
            except BaseException as e:     # surface loader errors in the consumer
                q.put(e)
                return
            q.put(None)

        th = threading.Thread(target=produce, daemon=True)
        th.start()
        try:
            while True:
                t0 = time.perf_counter()
                item = q.get()
                st["wait_s"] += time.perf_counter() - t0
                if item is None:
                    return
                if isinstance(item, BaseException):
                    raise item
                yield item
        finally:
            stop.set()
            while th.is_alive():
                try:
                    q.get_nowait()
                except queue.Empty:
                    th.join(timeout=0.05)


def _pil_crop_resize(raw: torch.Tensor, boxes: torch.Tensor, H: int, W: int) -> torch.Tensor:
    from PIL import Image
    r = raw.reshape((-1,) + tuple(raw.shape[-3:])).cpu().numpy()
    bx = boxes.reshape(-1, 4).cpu().numpy()
    out = np.empty((r.shape[0], 3, H, W), np.uint8)
    for i in range(r.shape[0]):
        img = Image.fromarray(r[i]).crop(tuple(int(v) for v in bx[i])).resize((W, H), Image.BILINEAR)
        out[i] = np.asarray(img).transpose(2, 0, 1)
    return torch.from_numpy(out)


CROP_MAX_TAPS = 16   # csrc/kernels/imgproc.hip MAXK: filter taps per axis of the GPU resize


def gpu_crop_supported(h0: int, w0: int, H: int, W: int) -> bool:
    """True when every crop of an [h0, w0] frame resized to [H, W] fits the GPU kernel's tap budget.  Pillow's
    bilinear filter spans ceil(2 * max(crop / out, 1)) + 1 source pixels per axis; a crop is at most the frame."""
    def taps(src, dst):
        return math.ceil(2.0 * max(src / dst, 1.0)) + 1
    return taps(h0, H) <= CROP_MAX_TAPS and taps(w0, W) <= CROP_MAX_TAPS


def decode_on_device(batch: Dict, H: int, W: int) -> Dict:
    """Replace ``raw_frames`` + ``crop_boxes`` by the cropped, resized ``image`` [B, T, 3, H, W] uint8 (on the
    batch's device: the HIP kernel on GPU, Pillow on CPU).  Other batches pass through unchanged."""
    obs = batch.get("train_observation", {})
    if "raw_frames" not in obs:
        return batch
    raw, boxes = obs["raw_frames"], obs["crop_boxes"]
    B, T = raw.shape[:2]
    if raw.is_cuda and gpu_crop_supported(raw.shape[2], raw.shape[3], H, W):
        from ..ops import load
        img = load().crop_resize_u8(raw.reshape((B * T,) + tuple(raw.shape[2:])), boxes.reshape(B * T, 4), H, W)
    else:
        # CPU batches, and downscales past the GPU kernel's tap budget (> ~7x): Pillow, exact by construction
        img = _pil_crop_resize(raw, boxes, H, W).to(raw.device)
    obs2 = {k: v for k, v in obs.items() if k not in ("raw_frames", "crop_boxes")}
    obs2["image"] = img.view(B, T, 3, H, W)
    out = dict(batch)
    out["train_observation"] = obs2
    return out
