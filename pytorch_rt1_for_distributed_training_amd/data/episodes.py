"""Language-Table episode windows (reference D1-D5, ``load_np_dataset.py``).

Semantics kept from ``EmbodiedIntelligenceDataset`` (``load_np_dataset.py:41-116``):
each episode is left-padded with ``window-1`` copies of its first step and
yields one sample per window start; a sample is ``{action_label:
{terminate_episode (T,), action (T,2)}, train_observation: {image (T,3,H,W),
natural_language_embedding (T,512)}}``.  ``DecodeAndRandomResizedCrop``
(``:8-39``) crops ``factor*size`` at a random offset and bilinearly resizes to
(W, H).

Storage differs on purpose.  The reference keeps every episode as a pickled
object array and re-loads the WHOLE episode file for every sample (``:80-83``,
SURVEY §2.10 item 9).  Here an episode is an ``.npz`` of plain arrays
(``rgb`` uint8 (S,h,w,3), ``instruction`` f32 (S,512), ``action`` f32 (S,2),
``is_terminal`` bool (S,)) loaded with ``allow_pickle=False``; the index is
built from array headers only, and each worker keeps a small LRU of decoded
episodes so consecutive windows of one episode hit memory.
``convert_reference_episodes`` translates the reference's ``.npy`` format
(which needs ``allow_pickle=True`` and therefore an explicit opt-in).
"""
from __future__ import annotations

import collections
import glob
import os
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

try:
    from PIL import Image
except ImportError:  # pragma: no cover
    Image = None


class DecodeAndRandomResizedCrop:
    def __init__(self, random_crop_factor: Optional[float] = None, resize_size=(456, 256), as_uint8: bool = False,
                 rng: Optional[np.random.Generator] = None):
        self.random_crop_factor = random_crop_factor
        self.resize_size = tuple(resize_size)  # (W, H) like PIL
        self.as_uint8 = as_uint8
        self.rng = rng or np.random.default_rng()

    def __call__(self, image) -> torch.Tensor:
        if not isinstance(image, Image.Image):
            image = Image.fromarray(np.asarray(image))
        w0, h0 = image.size
        if self.random_crop_factor is None:
            box = (0, 0, w0, h0)
        else:
            sh, sw = h0 * self.random_crop_factor, w0 * self.random_crop_factor
            oy = int(self.rng.integers(0, int(h0 - sh + 1)))
            ox = int(self.rng.integers(0, int(w0 - sw + 1)))
            box = (ox, oy, ox + sw, oy + sh)
        img = np.array(image.crop(box).resize(self.resize_size, Image.BILINEAR))
        t = torch.from_numpy(np.ascontiguousarray(img)).permute(2, 0, 1)
        return t.contiguous() if self.as_uint8 else t.float().div_(255.0)


def _npz_len(path: str) -> int:
    with np.load(path, allow_pickle=False) as z:
        return int(z["action"].shape[0])


class EpisodeWindowDataset(torch.utils.data.Dataset):
    def __init__(self, data_dir: str, ids: Sequence[int], window_length: int, transform=None, cache_episodes: int = 4):
        self.data_dir = data_dir
        self.ids = list(ids)
        self.window = int(window_length)
        self.transform = transform
        self._cache: "collections.OrderedDict[int, Dict[str, np.ndarray]]" = collections.OrderedDict()
        self._cache_n = cache_episodes
        self.samples: List[tuple] = []
        for eid in self.ids:
            n = _npz_len(self._path(eid))
            # padded length = n + window - 1  ->  n windows per episode
            self.samples.extend((eid, i) for i in range(n))

    def _path(self, eid: int) -> str:
        return os.path.join(self.data_dir, f"episode_{eid}.npz")

    def _episode(self, eid: int) -> Dict[str, np.ndarray]:
        ep = self._cache.get(eid)
        if ep is None:
            with np.load(self._path(eid), allow_pickle=False) as z:
                ep = {k: z[k] for k in z.files}
            self._cache[eid] = ep
            if len(self._cache) > self._cache_n:
                self._cache.popitem(last=False)
        else:
            self._cache.move_to_end(eid)
        return ep

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, idx):
        eid, start = self.samples[idx]
        ep = self._episode(eid)
        steps = [max(0, j - (self.window - 1)) for j in range(start, start + self.window)]
        imgs = []
        for s in steps:
            frame = ep["rgb"][s]
            if self.transform is not None:
                imgs.append(self.transform(frame))
            else:
                imgs.append(torch.from_numpy(np.ascontiguousarray(frame)).permute(2, 0, 1).float() / 255.0)
        term = torch.tensor([1 if bool(ep["is_terminal"][s]) else 0 for s in steps], dtype=torch.long)
        return {"action_label": {"terminate_episode": term,
                                 "action": torch.from_numpy(ep["action"][steps].astype(np.float32))},
                "train_observation": {"image": torch.stack(imgs),
                                      "natural_language_embedding":
                                          torch.from_numpy(ep["instruction"][steps].astype(np.float32))}}


def collate_fn(batch: List[Dict]) -> Dict:
    """Stack nested sample dicts into (B, T, ...) (``load_np_dataset.py:131-146``)."""
    def stack(items):
        first = items[0]
        if isinstance(first, dict):
            return {k: stack([it[k] for it in items]) for k in first}
        return torch.stack(items)
    return stack(batch)


def write_episode(path: str, rgb, instruction, action, is_terminal, is_first=None):
    rgb = np.asarray(rgb, dtype=np.uint8)
    arrays = dict(rgb=rgb, instruction=np.asarray(instruction, np.float32), action=np.asarray(action, np.float32),
                  is_terminal=np.asarray(is_terminal, bool))
    if is_first is not None:
        arrays["is_first"] = np.asarray(is_first, bool)
    np.savez(path, **arrays)


def convert_reference_episodes(src_dir: str, dst_dir: str, trust_pickle: bool = False) -> int:
    """Convert the reference's ``episode_{id}.npy`` (object arrays of step dicts,
    written by ``rlds_np_convert.py``) into ``.npz`` episodes.  Loading those
    files executes pickle, so it must be explicitly allowed for files you trust."""
    if not trust_pickle:
        raise PermissionError("reference .npy episodes are pickled object arrays; pass trust_pickle=True "
                              "only for files you produced yourself")
    os.makedirs(dst_dir, exist_ok=True)
    n = 0
    for path in sorted(glob.glob(os.path.join(src_dir, "episode_*.npy"))):
        steps = np.load(path, allow_pickle=True)
        write_episode(os.path.join(dst_dir, os.path.basename(path)[:-4] + ".npz"),
                      np.stack([s["rgb"] for s in steps]), np.stack([s["instruction"] for s in steps]),
                      np.stack([s["action"] for s in steps]), [bool(s["is_terminal"]) for s in steps],
                      [bool(s.get("is_first", False)) for s in steps])
        n += 1
    return n


def make_fake_episodes(dst_dir: str, num_episodes: int, steps: int = 10, height: int = 64, width: int = 96,
                       seed: int = 0) -> List[int]:
    """Tiny random episodes in the on-disk format (tests / smoke runs)."""
    rng = np.random.default_rng(seed)
    os.makedirs(dst_dir, exist_ok=True)
    for e in range(num_episodes):
        term = np.zeros(steps, bool)
        term[-1] = True
        write_episode(os.path.join(dst_dir, f"episode_{e}.npz"),
                      rng.integers(0, 256, (steps, height, width, 3), dtype=np.uint8),
                      np.repeat(rng.standard_normal((1, 512)).astype(np.float32), steps, 0),
                      rng.uniform(-0.1, 0.1, (steps, 2)).astype(np.float32), term,
                      np.arange(steps) == 0)
    return list(range(num_episodes))
