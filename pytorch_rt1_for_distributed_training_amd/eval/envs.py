"""Evaluation environments and observation wrappers.

The reference evaluates in Google's pybullet Language-Table simulator
(``language_table/environments``) wrapped by ``UseTokenWrapper``
(instruction -> Universal-Sentence-Encoder embedding), ``CentralCropImageWrapper``
(central crop consistent with the training random-crop factor, resize to
456x256) and a 6-step ``HistoryWrapper`` (``language_table/eval/wrappers.py``,
``main_rt1.py:130-142``).

* ``make_language_table_env`` builds that stack when ``language_table`` +
  ``pybullet`` + an instruction encoder are importable (they are optional; not
  present in this image) and raises a clear error otherwise.
* ``CentralCropResize`` and ``History`` re-implement the two image/history
  wrappers without TensorFlow.
* ``ToyPushEnv`` is a dependency-free 2-D block-pushing task with the same
  observation/step interface, so the full rollout loop (policy, wrappers,
  success accounting, video frames) runs and is tested anywhere.
* ``make_sim_env`` is the in-tree Language-Table board (``sim``: the reference's block sets, task rewards,
  instruction language and camera on a planar pushing world) behind the same interface, with the
  reference eval's "reject boards the oracle cannot solve" reset (``main_rt1.py:162-172``).
"""
from __future__ import annotations

import collections
from typing import Callable, Dict, Optional, Tuple

import numpy as np

try:
    from PIL import Image
except ImportError:  # pragma: no cover
    Image = None


class CentralCropResize:
    """Central crop of ``factor`` (matching the training random crop) then bilinear resize to (W, H)."""

    def __init__(self, target_width: int = 456, target_height: int = 256, random_crop_factor: float = 0.95):
        self.w, self.h, self.f = target_width, target_height, random_crop_factor

    def __call__(self, rgb: np.ndarray) -> np.ndarray:
        h0, w0 = rgb.shape[:2]
        ch, cw = int(h0 * self.f), int(w0 * self.f)
        oy, ox = (h0 - ch) // 2, (w0 - cw) // 2
        img = Image.fromarray(np.asarray(rgb, dtype=np.uint8)[oy:oy + ch, ox:ox + cw])
        return np.array(img.resize((self.w, self.h), Image.BILINEAR))


class History:
    """Fixed-length observation history, first observation tiled (``tile_first_step_obs=True``)."""

    def __init__(self, length: int = 6):
        self.length = length
        self.buf: Dict[str, collections.deque] = {}

    def reset(self, obs: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
        self.buf = {k: collections.deque([v] * self.length, maxlen=self.length) for k, v in obs.items()}
        return self.stacked()

    def push(self, obs: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
        for k, v in obs.items():
            self.buf[k].append(v)
        return self.stacked()

    def stacked(self) -> Dict[str, np.ndarray]:
        return {k: np.stack(list(d)) for k, d in self.buf.items()}


class ToyPushEnv:
    """Push a block to a target with 2-D delta actions in [-0.1, 0.1] (Language-Table action space).

    Observation: ``rgb`` (180, 320, 3) uint8 top-down render (Language-Table
    camera size, ``environments/constants.py:46-47``) and
    ``instruction_embedding`` (512,) — a fixed random vector per target colour.
    """

    H, W = 180, 320

    def __init__(self, seed: int = 0, success_radius: float = 0.05):
        self.rng = np.random.default_rng(seed)
        self.success_radius = success_radius
        self.embeddings = {c: np.random.default_rng(100 + i).standard_normal(512).astype(np.float32)
                           for i, c in enumerate(("red", "blue", "green", "yellow"))}
        self.reset()

    def reset(self):
        self.effector = self.rng.uniform(-0.3, 0.3, 2)
        self.block = self.rng.uniform(-0.3, 0.3, 2)
        self.target = self.rng.uniform(-0.3, 0.3, 2)
        self.color = self.rng.choice(list(self.embeddings))
        self.steps = 0
        return self._obs()

    @property
    def succeeded(self) -> bool:
        return float(np.linalg.norm(self.block - self.target)) < self.success_radius

    def step(self, action) -> Tuple[Dict[str, np.ndarray], float, bool, dict]:
        a = np.clip(np.asarray(action, dtype=np.float64), -0.1, 0.1)
        self.effector = np.clip(self.effector + a, -0.5, 0.5)
        if np.linalg.norm(self.effector - self.block) < 0.05:
            self.block = np.clip(self.block + a, -0.5, 0.5)
        self.steps += 1
        done = self.succeeded
        return self._obs(), float(done), done, {}

    def render(self) -> np.ndarray:
        img = np.full((self.H, self.W, 3), 235, np.uint8)

        def dot(p, color, r):
            cy = int((p[1] + 0.5) * (self.H - 1))
            cx = int((p[0] + 0.5) * (self.W - 1))
            y0, y1, x0, x1 = max(cy - r, 0), min(cy + r, self.H), max(cx - r, 0), min(cx + r, self.W)
            img[y0:y1, x0:x1] = color
        dot(self.target, (40, 40, 40), 6)
        dot(self.block, (200, 30, 30), 8)
        dot(self.effector, (30, 30, 200), 4)
        return img

    def _obs(self):
        return {"rgb": self.render(), "instruction_embedding": self.embeddings[self.color]}


def make_language_table_env(seed: int = 0, instruction_encoder: Optional[Callable[[str], np.ndarray]] = None):
    """The reference BlockToBlock / BLOCK_8 environment (requires pybullet + language_table)."""
    try:
        from language_table.environments import blocks, language_table  # type: ignore
        from language_table.environments.rewards import block2block  # type: ignore
    except ImportError as e:
        raise RuntimeError("the Language-Table simulator (pybullet + language_table package) is not installed; "
                           "use --env toy for a dependency-free rollout") from e
    if instruction_encoder is None:
        raise RuntimeError("an instruction encoder (text -> 512-d USE embedding) is required for Language-Table")
    env = language_table.LanguageTable(block_mode=blocks.LanguageTableBlockVariants.BLOCK_8,
                                       reward_factory=block2block.BlockToBlockReward, seed=seed)

    class _Adapter:
        def __init__(self, inner):
            self.inner = inner

        def _obs(self, o):
            text = bytes(o["instruction"][o["instruction"] != 0].tolist()).decode("utf-8")
            return {"rgb": o["rgb"], "instruction_embedding": instruction_encoder(text)}

        def reset(self):
            return self._obs(self.inner.reset())

        def step(self, a):
            o, r, d, info = self.inner.step(a)
            return self._obs(o), r, d, info

        def render(self):
            return self.inner.render()

        @property
        def succeeded(self):
            return self.inner.succeeded
    return _Adapter(env)


class SimEnvAdapter:
    """``sim.LanguageTable`` -> {rgb, instruction_embedding} observations for the RT-1 rollout loop."""

    def __init__(self, env, encoder: Callable[[str], np.ndarray], reject_unsolvable: bool = True,
                 max_resets: int = 20, oracle_steps: int = 80):
        self.inner, self.encoder = env, encoder
        self.reject_unsolvable, self.max_resets, self.oracle_steps = reject_unsolvable, max_resets, oracle_steps

    def _obs(self, o):
        return {"rgb": o["rgb"], "instruction_embedding": self.encoder(self.inner.instruction_str or "")}

    def reset(self):
        from ..sim import RRTPushOracle, plan_succeeds
        o = self.inner.reset()
        if self.reject_unsolvable:
            # the reference rejects boards its RRT* push oracle cannot plan; we also require the rollout to succeed
            for _ in range(self.max_resets):
                if plan_succeeds(self.inner, self.oracle_steps, oracle_cls=RRTPushOracle):
                    break
                o = self.inner.reset()
        return self._obs(o)

    def step(self, a):
        o, r, d, info = self.inner.step(a)
        return self._obs(o), r, d, info

    def render(self):
        return self.inner.render()

    @property
    def succeeded(self):
        return self.inner.succeeded

    @property
    def instruction(self) -> str:
        return self.inner.instruction_str or ""


def make_sim_env(reward: str = "block2block", block_mode: str = "BLOCK_8", seed: int = 0,
                 encoder: Optional[Callable[[str], np.ndarray]] = None, reject_unsolvable: bool = True,
                 delay_reward_steps: int = 0) -> SimEnvAdapter:
    """The eval protocol of ``main_rt1.py:130-142`` on the in-tree board: BLOCK_8 + BlockToBlock by default."""
    from ..sim import REWARDS, BlockMode, HashedTextEncoder, LanguageTable
    if reward not in REWARDS:
        raise ValueError(f"unknown reward {reward!r}; choose from {sorted(REWARDS)}")
    env = LanguageTable(BlockMode[block_mode], reward_factory=REWARDS[reward], seed=seed,
                        delay_reward_steps=delay_reward_steps)
    return SimEnvAdapter(env, encoder or HashedTextEncoder(), reject_unsolvable=reject_unsolvable)
