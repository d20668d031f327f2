"""Language-Table gym-style environment on the planar world.

API of the reference env (``language_table/environments/language_table.py:45-231``): construct with a
block mode, a reward factory, a seed and ``delay_reward_steps``; ``reset() -> obs``,
``step(action) -> (obs, reward, done, info)`` with ``action`` = effector delta xy in [-0.1, 0.1]^2,
``render()``, ``succeeded``, ``compute_state()``, ``encode_instruction`` / ``decode_instruction`` (512 utf-8
bytes as int32), state save / restore, ``seed()``, ``get_control_frequency()``.  Observations are the
reference's: ``effector_translation``, ``effector_target_translation``, ``instruction`` (int32[512]) and
``rgb`` (180 x 320 x 3 uint8).  Reset follows ``_reset_poses_randomly`` (``:822-931``): a block subset for
the mode, a random effector start, rejection-sampled block poses (>= 1.75 cm apart, >= 6 cm from the
effector), settle, then ask the reward for a task and re-sample the board on ``FAILURE``.
"""
from __future__ import annotations

import collections
from typing import Callable, Dict, Optional

import numpy as np

from .. import spaces
from . import board, kinematics
from .tasks import (FAILURE, Block2BlockRelativeLocationTaskInfo, Block2BlockTaskInfo, Block2LocationTaskInfo,
                    Block2RelativeLocationTaskInfo, Point2BlockTaskInfo, SeparateBlocksTaskInfo)
from .world import OFF_TABLE, PlanarWorld


class LanguageTable:
    def __init__(self, block_mode=board.BlockMode.BLOCK_8, training: bool = True,
                 reward_factory: Optional[Callable] = None, control_frequency: float = 10.0,
                 seed: Optional[int] = None, delay_reward_steps: int = 0, render_text_in_image: bool = True,
                 use_arm: bool = True, asset_root: Optional[str] = None):
        self._block_mode = block_mode
        # xArm6 joint state driven by IK each step (sim/kinematics.py; the reference's XArmSimRobot)
        self.robot = kinematics.XArmSimRobot() if use_arm else None
        self._training = training
        self._rng = np.random.RandomState(seed=seed)
        self._control_frequency = control_frequency
        self._render_text_in_image = render_text_in_image
        self._world = PlanarWorld()
        if asset_root is not None:
            # the reference loads one URDF per block from its asset tree (language_table.py:738-760); here the
            # tree is generated on first use and the world takes its radii / colours from it
            from . import assets
            self._world.load_assets(assets.write_assets(asset_root))
        self._reward_calculator = None
        self._instruction_str: Optional[str] = None
        self._instruction = self.encode_instruction("")
        self._start_block = board.ALL_BLOCKS[0]
        self._oracle_target_block = None
        self._oracle_target_translation = None
        self._blocks_on_table = ()
        self._task_info = None
        if reward_factory is not None:
            self._reward_calculator = reward_factory(goal_reward=100.0, rng=self._rng,
                                                     delay_reward_steps=delay_reward_steps, block_mode=block_mode)
        self.action_space = spaces.Box(-0.1, 0.1, (2,), np.float32)
        lo, hi = board.WORKSPACE_BOUNDS[0] - 0.1, board.WORKSPACE_BOUNDS[1] + 0.1
        self.observation_space = spaces.Dict(collections.OrderedDict(
            effector_translation=spaces.Box(lo, hi, (2,), np.float32),
            effector_target_translation=spaces.Box(lo, hi, (2,), np.float32),
            instruction=spaces.Box(0, 2147483647, (board.INSTRUCTION_LENGTH,), np.int32),
            rgb=spaces.Box(0, 255, (board.IMAGE_HEIGHT, board.IMAGE_WIDTH, 3), np.uint8)))
        self.reset()

    # ------------------------------------------------------------------ gym API
    def seed(self, seed=None):
        self._rng = np.random.RandomState(seed=seed)
        if self._reward_calculator is not None:
            self._reward_calculator.seed(self._rng)

    def get_control_frequency(self) -> float:
        return self._control_frequency

    def reset(self):
        subsets = board.block_subsets(self._block_mode, self._training)
        blocks_on_table = tuple(subsets[self._rng.choice(len(subsets))])
        self._blocks_on_table = blocks_on_table
        self._reset_poses_randomly(blocks_on_table)
        return self._observation(self.compute_state())

    def step(self, action):
        a = np.asarray(action, np.float64).reshape(2)
        w = self._world
        w.set_effector_target(w.effector_target + a)
        self._drive_arm()
        w.step()
        state = self.compute_state()
        if self._reward_calculator is None:
            reward, done = 0.0, False
        else:
            reward, done = self._reward_calculator.reward(state)
        return self._observation(state), reward, done, {}

    def render(self, mode: str = "rgb_array") -> np.ndarray:
        img = self._world.render()
        if self._render_text_in_image and self._instruction_str:
            img = _draw_text(img, self._instruction_str)
        return img

    @property
    def succeeded(self) -> bool:
        if self._reward_calculator is None:
            return False
        return self._reward_calculator.reward(self.compute_state())[0] > 0.0

    @property
    def instruction_str(self) -> Optional[str]:
        return self._instruction_str

    @property
    def blocks_on_table(self):
        return self._blocks_on_table

    @property
    def world(self) -> PlanarWorld:
        return self._world

    # ------------------------------------------------------------------ instruction bytes
    @staticmethod
    def encode_instruction(instruction: str) -> np.ndarray:
        out = np.zeros(board.INSTRUCTION_LENGTH, np.int32)
        if not instruction:
            return out
        b = list(instruction.encode("utf-8"))
        if len(b) > board.INSTRUCTION_LENGTH:
            raise ValueError(f"instruction too long ({len(b)} > {board.INSTRUCTION_LENGTH}): {instruction}")
        out[:len(b)] = b
        return out

    @staticmethod
    def decode_instruction(codes) -> str:
        nz = np.asarray(codes)[np.asarray(codes) != 0]
        return bytes(nz.astype(np.uint8).tolist()).decode("utf-8") if nz.size else ""

    # ------------------------------------------------------------------ state
    def compute_state(self, request_task_update: bool = True) -> Dict[str, np.ndarray]:
        w = self._world
        obs: Dict[str, np.ndarray] = collections.OrderedDict()
        for name in w.names:
            i = w.index[name]
            obs[f"block_{name}_translation"] = w.pos[i].astype(np.float32)
            obs[f"block_{name}_orientation"] = np.array([w.yaw[i]], np.float32)
            obs[f"block_{name}_mask"] = np.array([1.0 if name in self._blocks_on_table else 0.0], np.float32)
        eff_t = w.effector_target.astype(np.float32)
        if request_task_update and hasattr(self._reward_calculator, "get_current_task_info") and \
                self._task_info is not None:
            self._set_task_info(self._reward_calculator.get_current_task_info(obs))
        start = w.pos[w.index[self._start_block]]
        obs["effector_target_to_start_block_translation"] = (start - w.effector_target).astype(np.float32)
        obs["start_block_orientation"] = np.array([w.yaw[w.index[self._start_block]]], np.float32)
        if self._oracle_target_translation is not None:
            tgt = np.asarray(self._oracle_target_translation, np.float64)
            obs["task_target_orientation"] = np.array([0.0], np.float32)
        elif self._oracle_target_block is not None:
            tgt = w.pos[w.index[self._oracle_target_block]]
            obs["task_target_orientation"] = np.array([w.yaw[w.index[self._oracle_target_block]]], np.float32)
        else:
            tgt = w.effector_target
            obs["task_target_orientation"] = np.array([0.0], np.float32)
        obs["effector_target_to_task_target_translation"] = (tgt - w.effector_target).astype(np.float32)
        obs["effector_translation"] = w.effector.astype(np.float32)
        obs["effector_target_translation"] = eff_t
        obs["instruction"] = self._instruction
        obs["rgb"] = w.render()
        return obs

    def _drive_arm(self):
        if self.robot is not None:
            self.robot.set_target_effector_pose(kinematics.effector_pose(self._world.effector_target))
            self.robot.step()

    def get_state(self) -> Dict:
        """Snapshot for save / restore (the reference's ``get_pybullet_state``)."""
        s = self._world.get_state()
        if self.robot is not None:
            s["robot"] = self.robot.get_state()
        s.update(blocks_on_table=tuple(self._blocks_on_table), instruction=self._instruction_str,
                 task_info=self._task_info, start_block=self._start_block,
                 oracle_target_block=self._oracle_target_block,
                 oracle_target_translation=None if self._oracle_target_translation is None
                 else np.array(self._oracle_target_translation),
                 rng=self._rng.get_state())
        if self._reward_calculator is not None:
            # the reward's task (blocks / targets / phrase) and its delayed-reward counter
            s["reward"] = {k: v for k, v in vars(self._reward_calculator).items()
                           if k != "_rng" and _plain(v)}
        return s

    def set_state(self, s: Dict):
        self._world.set_state(s)
        if self.robot is not None and "robot" in s:
            self.robot.set_state(s["robot"])
        self._blocks_on_table = tuple(s["blocks_on_table"])
        self._task_info = s["task_info"]
        self._start_block = s["start_block"]
        self._oracle_target_block = s["oracle_target_block"]
        self._oracle_target_translation = s["oracle_target_translation"]
        self._instruction_str = s["instruction"]
        self._instruction = self.encode_instruction(self._instruction_str or "")
        if "rng" in s:
            self._rng.set_state(tuple(s["rng"]))
        if self._reward_calculator is not None and "reward" in s:
            for k, v in s["reward"].items():
                setattr(self._reward_calculator, k, v)

    def _observation(self, state) -> Dict[str, np.ndarray]:
        return collections.OrderedDict(effector_translation=state["effector_translation"],
                                       effector_target_translation=state["effector_target_translation"],
                                       instruction=state["instruction"], rgb=state["rgb"])

    # ------------------------------------------------------------------ reset
    def _reset_poses_randomly(self, blocks_on_table):
        w = self._world
        lo = board.WORKSPACE_BOUNDS[0] + board.WORKSPACE_BOUNDS_BUFFER
        hi = board.WORKSPACE_BOUNDS[1] - board.WORKSPACE_BOUNDS_BUFFER
        attempts_with_reward = 0
        while True:
            w.remove_all()
            eff = self._rng.uniform(lo, hi)
            w.effector = eff.copy()
            w.effector_target = eff.copy()
            placed = []
            for name in blocks_on_table:
                for _ in range(21):
                    xy = self._rng.uniform(lo, hi)
                    yaw = self._rng.uniform(0.0, 2 * np.pi)
                    if (not placed or min(np.linalg.norm(xy - p) for p in placed) > board.BLOCK_DISTANCE_THRESHOLD) \
                            and np.linalg.norm(xy - eff) > board.ARM_DISTANCE_THRESHOLD:
                        placed.append(xy)
                        w.place(name, xy, yaw)
                        break
                else:
                    raise ValueError("exceeded max attempts for generating a block pose")
            w.settle()
            if self.robot is not None:
                self.robot.reset_joints(self.robot.initial_joint_positions)
                self._drive_arm()
            if self._reward_calculator is None:
                self._task_info = None
                return
            info = self._reward_calculator.reset(self.compute_state(request_task_update=False), blocks_on_table)
            if info == FAILURE:
                attempts_with_reward += 1
                if attempts_with_reward > 200:
                    raise ValueError("cannot find a block configuration with a valid task")
                continue
            self._set_task_info(info)
            return

    def _set_task_info(self, info):
        self._task_info = info
        self._oracle_target_block = None
        self._oracle_target_translation = None
        if isinstance(info, Block2BlockTaskInfo):
            self._start_block, self._oracle_target_block = info.block1, info.block2
        elif isinstance(info, (Block2LocationTaskInfo, Block2RelativeLocationTaskInfo, SeparateBlocksTaskInfo)):
            self._start_block, self._oracle_target_translation = info.block, info.target_translation
        elif isinstance(info, Block2BlockRelativeLocationTaskInfo):
            self._start_block = info.block
            self._oracle_target_block = info.target_block
            self._oracle_target_translation = info.target_translation
        elif isinstance(info, Point2BlockTaskInfo):
            self._start_block = self._oracle_target_block = info.block_target
        else:
            raise ValueError(f"unknown task info {info!r}")
        self._instruction_str = info.instruction
        self._instruction = self.encode_instruction(info.instruction)

    @property
    def is_point_task(self) -> bool:
        return isinstance(self._task_info, Point2BlockTaskInfo)

    @property
    def oracle_target(self):
        """(block to push, xy to push it to) for the scripted oracle."""
        w = self._world
        if self._oracle_target_translation is not None:
            tgt = np.asarray(self._oracle_target_translation, np.float64)
        elif self._oracle_target_block is not None:
            tgt = w.pos[w.index[self._oracle_target_block]].copy()
        else:
            tgt = None
        return self._start_block, tgt


def _plain(v) -> bool:
    """Values a state snapshot can carry (and sim/state_io.py can serialise)."""
    if v is None or isinstance(v, (bool, int, float, str, np.ndarray, np.integer, np.floating)):
        return True
    if isinstance(v, (list, tuple)):
        return all(_plain(x) for x in v)
    return type(v).__name__.endswith("TaskInfo")


def _draw_text(img: np.ndarray, text: str) -> np.ndarray:
    try:
        from PIL import Image, ImageDraw
    except ImportError:  # pragma: no cover
        return img
    im = Image.fromarray(img)
    ImageDraw.Draw(im).text((4, 2), text[:80], fill=(255, 255, 255))
    return np.asarray(im).copy()


OFF_TABLE_XY = OFF_TABLE
