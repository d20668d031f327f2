"""Closed-loop evaluation loop (reference ``language_table/eval/main_rt1.py:100-201``).

Per episode: zero the policy state, reset the env, feed the centrally cropped
frame + instruction embedding, step until the env reports success or
``max_episode_steps`` is exceeded (the reference breaks once ``episode_steps >
80``, i.e. after at most 81 policy steps), record rendered frames and count
successes.  Videos are written as animated GIF (PIL) instead of mp4 (imageio is
not a dependency).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import numpy as np

from .envs import CentralCropResize, History

try:
    from PIL import Image
except ImportError:  # pragma: no cover
    Image = None


def save_gif(frames: List[np.ndarray], path: str, fps: int = 10):
    imgs = [Image.fromarray(np.asarray(f, dtype=np.uint8)) for f in frames]
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    imgs[0].save(path, save_all=True, append_images=imgs[1:], duration=int(1000 / fps), loop=0)


def evaluate(policy, env, episodes: int = 10, max_episode_steps: int = 80, crop: Optional[CentralCropResize] = None,
             history_length: int = 6, video_dir: Optional[str] = None, name: str = "blocktoblock") -> Dict[str, float]:
    crop = crop or CentralCropResize()
    hist = History(history_length)
    successes = 0
    lengths = []
    for ep in range(episodes):
        policy.reset()
        obs = env.reset()
        frames = [env.render()]
        h = hist.reset({"rgb": crop(obs["rgb"]), "emb": obs["instruction_embedding"]})
        steps = 0
        done = False
        while not done:
            action = policy.action(h["rgb"], h["emb"])
            obs, _, done, _ = env.step(action)
            frames.append(env.render())
            h = hist.push({"rgb": crop(obs["rgb"]), "emb": obs["instruction_embedding"]})
            steps += 1
            if steps > max_episode_steps:
                break
        ok = bool(env.succeeded)
        successes += int(ok)
        lengths.append(steps)
        if video_dir:
            save_gif(frames, os.path.join(video_dir, f"{name}_{ep}_{'success' if ok else 'failure'}.gif"))
    return {name: successes, "episodes": episodes, "success_rate": successes / max(episodes, 1),
            "mean_steps": float(np.mean(lengths)) if lengths else 0.0}
