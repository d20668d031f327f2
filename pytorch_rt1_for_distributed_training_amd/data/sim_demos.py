"""Scripted demonstrations from the in-tree Language-Table board, windowed for sequence BC (SURVEY J3 role).

The reference trains LAVA on the RLDS Language-Table datasets through a tf.data pipeline that pads each
episode at the front, cuts fixed-length windows, and normalises (``input_pipeline_rlds.py:105-153``).  Without
network access the demonstrations here come from the scripted push oracle on ``sim.LanguageTable``: each
episode's (rgb, instruction embedding, action) steps are front-padded with copies of step 0 and cut into
``sequence_length`` windows whose label is the action of the last step.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
import torch


def collect_episodes(num_episodes: int, reward: str = "block2block", block_mode: str = "BLOCK_8", seed: int = 0,
                     max_steps: int = 60, encoder=None, action_noise: float = 0.0,
                     oracle: str = "push") -> List[Dict[str, np.ndarray]]:
    """Scripted demonstrations on the in-tree board; ``oracle="rrt"`` uses the obstacle-aware RRT* oracle
    (the reference's data came from its RRT oracle family)."""
    from ..sim import REWARDS, BlockMode, HashedTextEncoder, LanguageTable, PushOracle, RRTPushOracle
    oracle_cls = {"push": PushOracle, "rrt": RRTPushOracle}[oracle]
    enc = encoder or HashedTextEncoder()
    env = LanguageTable(BlockMode[block_mode], reward_factory=REWARDS[reward], seed=seed)
    episodes = []
    for ep in range(num_episodes):
        obs = env.reset()
        policy = oracle_cls(env, action_noise_std=action_noise, seed=seed + ep)
        emb = enc(env.instruction_str or "")
        rgb, acts, done = [], [], False
        for _ in range(max_steps):
            a = policy.action()
            rgb.append(obs["rgb"])
            acts.append(a)
            obs, _, done, _ = env.step(a)
            if done:
                break
        episodes.append({"rgb": np.stack(rgb), "instruction_embedding": np.repeat(emb[None], len(rgb), 0),
                         "action": np.stack(acts).astype(np.float32), "success": np.array(done)})
    return episodes


class WindowDataset(torch.utils.data.Dataset):
    """One sample per step: the window of ``sequence_length`` steps ending there (front-padded with step 0)."""

    def __init__(self, episodes: List[Dict[str, np.ndarray]], sequence_length: int = 4):
        self.episodes = episodes
        self.T = sequence_length
        self.index = [(e, s) for e, ep in enumerate(episodes) for s in range(len(ep["action"]))]

    def __len__(self):
        return len(self.index)

    def __getitem__(self, i):
        e, s = self.index[i]
        ep = self.episodes[e]
        steps = [max(0, s - self.T + 1 + k) for k in range(self.T)]
        return {"observation": {"rgb": torch.from_numpy(ep["rgb"][steps]),
                                "instruction_embedding": torch.from_numpy(ep["instruction_embedding"][steps])},
                "action": torch.from_numpy(ep["action"][s])}


def collate(samples):
    return {"observation": {k: torch.stack([s["observation"][k] for s in samples])
                            for k in samples[0]["observation"]},
            "action": torch.stack([s["action"] for s in samples])}


def to_device(batch, device):
    if isinstance(batch, dict):
        return {k: to_device(v, device) for k, v in batch.items()}
    return batch.to(device, non_blocking=True)


def action_batches(dataset: WindowDataset, batch_size: int = 64, seed: int = 0):
    """(obs, action) numpy batches for normalisation statistics."""
    rng = np.random.default_rng(seed)
    idx = rng.permutation(len(dataset))
    for i in range(0, len(idx), batch_size):
        acts = np.stack([dataset.episodes[dataset.index[j][0]]["action"][dataset.index[j][1]]
                         for j in idx[i:i + batch_size]])
        yield {}, acts


def rlds_episodes(builder_dir: str, encoder=None, rank: int = 0, world_size: int = 1, limit: int = 0,
                  split: str = "train") -> List[Dict[str, np.ndarray]]:
    """Episodes of a Language-Table RLDS builder directory (the reference's ``input_pipeline_rlds.py`` source),
    read without TensorFlow (``data/tfrecord.py``); episode i goes to rank i % world_size, the instruction bytes
    are embedded with ``encoder`` (text -> [512]; default the hashed stand-in)."""
    from ..sim import HashedTextEncoder
    from .tfrecord import read_rlds_episodes
    enc = encoder or HashedTextEncoder()
    if limit and limit < world_size:
        raise ValueError(f"rlds_episodes: limit {limit} < world_size {world_size} leaves some ranks without episodes")
    out = []
    # the rank's records are chosen before parsing: the other ranks' episodes are never decoded here
    for ep in read_rlds_episodes(builder_dir, split, select=lambda i: i % world_size == rank, limit=limit):
        st = ep["steps"]
        obs = st.get("observation", {})
        rgb = np.asarray(obs["rgb"], np.uint8)
        codes = np.asarray(obs["instruction"]).reshape(len(rgb), -1)
        texts = [bytes(c[c != 0].astype(np.uint8).tolist()).decode("utf-8", errors="ignore") for c in codes]
        out.append({"rgb": rgb, "instruction_embedding": np.stack([enc(t) for t in texts]).astype(np.float32),
                    "action": np.asarray(st["action"], np.float32).reshape(len(rgb), -1)[:, :2],
                    "success": np.array(bool(np.asarray(st.get("is_terminal", [False]))[-1]))})
    if not out:
        raise ValueError(f"rlds_episodes: rank {rank} of {world_size} got no episodes from {builder_dir} ({split})")
    return out


def synthetic_episodes(num: int, steps: int = 10, height: int = 180, width: int = 320,
                       seed: int = 0) -> List[Dict[str, np.ndarray]]:
    rng = np.random.default_rng(seed)
    return [{"rgb": rng.integers(0, 256, (steps, height, width, 3), dtype=np.uint8),
             "instruction_embedding": rng.standard_normal((steps, 512)).astype(np.float32),
             "action": rng.uniform(-0.03, 0.03, (steps, 2)).astype(np.float32), "success": np.array(False)}
            for _ in range(num)]
