"""Language-Table task rewards: reset (pick blocks / targets, sample an instruction) and sparse success.

Behavioural spec: ``language_table/environments/rewards/*.py``.  Every reward takes the env
state dict (``block_<name>_translation`` / ``_orientation``, ``effector_target_translation``), returns a
task-info record from ``reset`` (or ``FAILURE`` when the board admits no valid task, so the env re-samples
the board), and a sparse ``(reward, done)`` from ``reward``: ``goal_reward`` once the goal condition has
held for ``delay_reward_steps`` consecutive calls.  Thresholds, magnitudes and phrase tables come from
``sim.phrases``.  Family list: block2block, point2block, block2relativelocation, block2absolutelocation,
block2block_relative_location, separate_blocks, block1_to_corner, play (no success signal).
"""
from __future__ import annotations

import dataclasses
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import board, phrases as P

FAILURE = "failure"


# ------------------------------------------------------------------ task records (task_info.py)
@dataclasses.dataclass
class Block2BlockTaskInfo:
    instruction: str
    block1: str
    block2: str


@dataclasses.dataclass
class Block2LocationTaskInfo:
    instruction: str
    block: str
    target_translation: np.ndarray
    location: str


@dataclasses.dataclass
class Block2RelativeLocationTaskInfo:
    instruction: str
    block: str
    target_translation: np.ndarray
    location: str


@dataclasses.dataclass
class Block2BlockRelativeLocationTaskInfo:
    instruction: str
    block: str
    target_block: str
    direction: str
    target_translation: np.ndarray


@dataclasses.dataclass
class SeparateBlocksTaskInfo:
    instruction: str
    block: str
    avoid_blocks: List[str]
    target_translation: np.ndarray


@dataclasses.dataclass
class Point2BlockTaskInfo:
    instruction: str
    block_target: str


def target_inside_bounds(xy, buffer: float = board.WORKSPACE_BOUNDS_BUFFER) -> bool:
    return (board.X_MIN + buffer < xy[0] < board.X_MAX - buffer) and (board.Y_MIN + buffer < xy[1] < board.Y_MAX - buffer)


class TaskReward:
    """Shared machinery: rng, delayed sparse reward, block pose lookup."""

    def __init__(self, goal_reward: float = 100.0, rng=None, delay_reward_steps: int = 0,
                 block_mode=board.BlockMode.BLOCK_8):
        self._goal_reward = goal_reward
        self._rng = rng if rng is not None else np.random.RandomState(0)
        self._delay_reward_steps = delay_reward_steps
        self._block_mode = block_mode
        self._in_reward_zone_steps = 0
        self._target_translation = None

    def seed(self, rng):
        self._rng = rng

    def get_goal_region(self):
        return None, None

    @staticmethod
    def xy(state, block) -> np.ndarray:
        return np.asarray(state[f"block_{block}_translation"], np.float64)[:2]

    def _pick(self, blocks_on_table):
        return blocks_on_table[self._rng.choice(len(blocks_on_table))]

    def _pick_two(self, blocks_on_table):
        i, j = self._rng.choice(len(blocks_on_table), 2, replace=False)
        return blocks_on_table[i], blocks_on_table[j]

    def _name(self, block, blocks_on_table) -> str:
        syn = P.block_synonyms(block, blocks_on_table)
        return syn[self._rng.choice(len(syn))]

    def _choice(self, seq):
        return seq[self._rng.choice(len(seq))]

    def _sparse(self, in_goal: bool, delay: Optional[int] = None) -> Tuple[float, bool]:
        delay = self._delay_reward_steps if delay is None else delay
        if not in_goal:
            return 0.0, False
        if self._in_reward_zone_steps >= delay:
            return self._goal_reward, True
        self._in_reward_zone_steps += 1
        return 0.0, False


class BlockToBlockReward(TaskReward):
    """'push the red moon next to the blue cube': success when the two blocks are < 5 cm apart."""

    def reset(self, state, blocks_on_table):
        for _ in range(11):
            a, b = self._pick_two(blocks_on_table)
            if np.linalg.norm(self.xy(state, a) - self.xy(state, b)) >= board.TARGET_BLOCK_DISTANCE + 0.01:
                break
        else:
            return FAILURE
        self._start_block, self._target_block = a, b
        self._instruction = (f"{self._choice(P.PUSH_VERBS)} {self._name(a, blocks_on_table)} "
                             f"{self._choice(P.PREPOSITIONS)} {self._name(b, blocks_on_table)}")
        self._in_reward_zone_steps = 0
        return Block2BlockTaskInfo(self._instruction, a, b)

    def get_goal_region(self):
        return self._target_translation, board.TARGET_BLOCK_DISTANCE

    def reward(self, state):
        a, b = self.xy(state, self._start_block), self.xy(state, self._target_block)
        self._target_translation = b
        return self._sparse(np.linalg.norm(a - b) < board.TARGET_BLOCK_DISTANCE)


class PointToBlockReward(TaskReward):
    """'point at the green star': success when the effector target is < 5 cm from the block."""

    def reset(self, state, blocks_on_table):
        eff = np.asarray(state["effector_target_translation"], np.float64)
        for _ in range(11):
            blk = self._pick(blocks_on_table)
            if np.linalg.norm(self.xy(state, blk) - eff) >= board.TARGET_BLOCK_DISTANCE + 0.01:
                break
        else:
            return FAILURE
        self._block = blk
        self._instruction = f"{self._choice(P.POINT_PREPOSITIONS)} {self._name(blk, blocks_on_table)}"
        self._in_reward_zone_steps = 0
        return Point2BlockTaskInfo(self._instruction, blk)

    def reward(self, state):
        eff = np.asarray(state["effector_target_translation"], np.float64)
        return self._sparse(np.linalg.norm(self.xy(state, self._block) - eff) < board.TARGET_BLOCK_DISTANCE)


class BlockToRelativeLocationReward(TaskReward):
    """'slide the blue cube slightly up': a target offset 15 cm (near) or 25 cm (far) along one of 8 directions."""

    def reset(self, state, blocks_on_table):
        for _ in range(101):
            blk = self._pick(blocks_on_table)
            direction = self._choice(sorted(P.REL_DIRECTIONS))
            mode = self._choice(sorted(P.REL_MAGNITUDES))
            target = self.xy(state, blk) + P.REL_DIRECTIONS[direction] * P.REL_MAGNITUDES[mode]
            if target_inside_bounds(target):
                break
        else:
            return FAILURE
        self._block = blk
        verb = self._choice(P.REL_VERBS)
        name = self._name(blk, blocks_on_table)
        phrase = (P.sample_diagonal(self._rng, direction) if direction.startswith("diagonal")
                  else self._choice(P.REL_DIRECTION_WORDS[direction]))
        self._instruction = (P.sample_slightly(self._rng, verb, name, phrase) if mode == "near"
                             else f"{verb} {name} {phrase}")
        self._target_translation = target.copy()
        self._in_reward_zone_steps = 0
        return Block2RelativeLocationTaskInfo(self._instruction, blk, self._target_translation, direction)

    def get_goal_region(self):
        return self._target_translation, P.REL_TARGET_DISTANCE

    def reward(self, state):
        d = np.linalg.norm(self.xy(state, self._block) - self._target_translation)
        return self._sparse(d < P.REL_TARGET_DISTANCE)


class BlockToAbsoluteLocationReward(TaskReward):
    """'push the red moon to the top left corner': one of 9 board locations (10 / 11.5 cm radius)."""

    locations = P.ABS_LOCATIONS
    words = P.ABS_LOCATION_WORDS

    def _radius(self):
        return P.ABS_CENTER_TARGET_DISTANCE if self._location == "center" else P.ABS_TARGET_DISTANCE

    def reset(self, state, blocks_on_table):
        blk = self._pick(blocks_on_table)
        loc = self._choice(sorted(self.locations))
        info = self.reset_to(state, blk, loc, blocks_on_table)
        if self._in_goal(state, blk, self._target_translation):
            return FAILURE
        return info

    def reset_to(self, state, block, location, blocks_on_table):
        self._block, self._location = block, location
        self._instruction = (f"{self._choice(P.PUSH_VERBS)} {self._name(block, blocks_on_table)} to the "
                             f"{self._choice(self.words[location])}")
        self._target_translation = np.array(self.locations[location], np.float64)
        self._in_reward_zone_steps = 0
        return Block2LocationTaskInfo(self._instruction, block, self._target_translation, location)

    def _in_goal(self, state, block, target) -> bool:
        return np.linalg.norm(self.xy(state, block) - target) < self._radius()

    def get_goal_region(self):
        return self._target_translation, self._radius()

    def reward(self, state):
        return self._sparse(self._in_goal(state, self._block, self._target_translation))


class Block1ToCornerLocationReward(BlockToAbsoluteLocationReward):
    """'move the yellow pentagon to the bottom left corner' (8 cm radius)."""

    locations = P.CORNER_LOCATIONS
    words = P.CORNER_WORDS

    def _radius(self):
        return P.CORNER_TARGET_DISTANCE


class BlockToBlockRelativeLocationReward(TaskReward):
    """'put the red moon to the left of the blue cube': the pushed block must end on the segment from 0.5x to
    1.1x of an 8 cm (4 cm diagonal) offset from the target block, without dragging the target > 5 cm."""

    def target_translation_for(self, state, target_block, direction, scale: float = 1.0):
        mag = P.B2B_REL_MAG_DIAG if direction.startswith("diagonal") else P.B2B_REL_MAG
        return self.xy(state, target_block) + np.array(P.B2B_REL_DIRECTIONS[direction]) * mag * scale

    def reset(self, state, blocks_on_table):
        for _ in range(101):
            blk, tgt = self._pick_two(blocks_on_table)
            direction = self._choice(list(P.B2B_REL_DIRECTIONS))
            if target_inside_bounds(self.target_translation_for(state, tgt, direction)):
                break
        else:
            return FAILURE
        info = self.reset_to(state, blk, tgt, direction, blocks_on_table)
        self._in_reward_zone_steps = 0
        if self.reward_for(state, blk, tgt, direction, 0)[1]:
            return FAILURE
        return info

    def reset_to(self, state, block, target_block, direction, blocks_on_table):
        self._block, self._target_block, self._direction = block, target_block, direction
        self._target_reset_xy = self.xy(state, target_block).copy()
        self._target_translation = self.target_translation_for(state, target_block, direction)
        self._instruction = (f"{self._choice(P.PUSH_VERBS)} {self._name(block, blocks_on_table)} "
                             f"{self._choice(P.B2B_REL_WORDS[direction])} {self._name(target_block, blocks_on_table)}")
        return self.get_current_task_info(state)

    def get_current_task_info(self, state):
        self._target_translation = self.target_translation_for(state, self._target_block, self._direction)
        return Block2BlockRelativeLocationTaskInfo(self._instruction, self._block, self._target_block, self._direction,
                                                   self._target_translation)

    def reward_for(self, state, block, target_block, direction, delay):
        pb, tb = self.xy(state, block), self.xy(state, target_block)
        offset = self.target_translation_for(state, target_block, direction) - tb
        on_line = any(np.linalg.norm(tb + f * offset - pb) < P.B2B_REL_TARGET_DISTANCE
                      for f in np.linspace(0.5, 1.1, 10))
        dragged = np.linalg.norm(self._target_reset_xy - tb) > P.B2B_REL_DRAGGED_THRESHOLD
        return self._sparse(on_line and not dragged, delay)

    def get_goal_region(self):
        return self._target_translation, P.B2B_REL_TARGET_DISTANCE

    def reward(self, state):
        return self.reward_for(state, self._block, self._target_block, self._direction, self._delay_reward_steps)


class SeparateBlocksReward(TaskReward):
    """'pull the red moon apart from the blue cube and green star': the block touching most others is pushed
    10 cm beyond their centroid, away from it."""

    def _closest(self, block, xy, others):
        d = sorted(((n, np.linalg.norm(xy - p)) for n, p in others if n != block), key=lambda t: t[1])
        close = [t for t in d if t[1] < P.SEPARATE_JOINED_THRESHOLD]
        if not close:
            return [], np.inf
        return [t[0] for t in close], float(np.mean([t[1] for t in close]))

    def _choose(self, state, blocks_on_table):
        pts = [(b, self.xy(state, b)) for b in blocks_on_table]
        ranked = sorted(((b, self._closest(b, p, pts)) for b, p in pts), key=lambda t: t[1][1])
        push, (avoid, _) = ranked[0]
        return push, avoid

    def target_translation_for(self, state, block, avoid):
        centroid = np.mean([self.xy(state, b) for b in avoid], axis=0)
        self._avoid_centroid = centroid
        away = self.xy(state, block) - centroid
        away = away / (np.linalg.norm(away) + np.finfo(np.float32).eps)
        return centroid + away * P.SEPARATE_MAGNITUDE

    def reset(self, state, blocks_on_table):
        push, avoid = self._choose(state, blocks_on_table)
        if not avoid:
            return FAILURE
        target = self.target_translation_for(state, push, avoid)
        if not target_inside_bounds(target):
            return FAILURE
        self._block, self._avoid = push, avoid
        self._target_translation = target
        names = [self._name(b, blocks_on_table) for b in avoid]
        group = self._choice(P.GROUP_WORDS)
        phrase = P.separate_avoid_phrase(names, len(blocks_on_table), group,
                                         three_choice=lambda listed, g: self._choice([listed, g]))
        self._instruction = self._choice(P.SEPARATE_FORMS) % (self._name(push, blocks_on_table), phrase)
        self._in_reward_zone_steps = 0
        return self.get_current_task_info(state)

    def get_current_task_info(self, state):
        self._target_translation = self.target_translation_for(state, self._block, self._avoid)
        return SeparateBlocksTaskInfo(self._instruction, self._block, list(self._avoid), self._target_translation)

    def get_goal_region(self):
        return self._target_translation, P.SEPARATE_TARGET_DISTANCE

    def reward(self, state):
        d = np.linalg.norm(self.xy(state, self._block) - self._target_translation)
        return self._sparse(d < P.SEPARATE_TARGET_DISTANCE)


class PlayReward(TaskReward):
    """Long-horizon free-form instruction (play data collection): never terminates by itself."""

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self._play4 = P.play4_instructions() if self._block_mode == board.BlockMode.BLOCK_4 else None

    def reset(self, state, blocks_on_table):
        for _ in range(11):
            a, b = self._pick_two(blocks_on_table)
            if np.linalg.norm(self.xy(state, a) - self.xy(state, b)) >= board.TARGET_BLOCK_DISTANCE + 0.01:
                break
        else:
            return FAILURE
        if self._block_mode == board.BlockMode.BLOCK_4:
            inst = self._choice(self._play4)
        elif self._block_mode == board.BlockMode.BLOCK_8:
            inst = P.sample_play8_instruction(self._rng)
        else:
            raise ValueError(f"play reward supports BLOCK_4 / BLOCK_8, not {self._block_mode}")
        self._instruction = inst
        return Block2BlockTaskInfo(inst, a, b)

    def reward(self, state):
        return 0.0, False


REWARDS = {
    "block2block": BlockToBlockReward,
    "point2block": PointToBlockReward,
    "block2relativelocation": BlockToRelativeLocationReward,
    "block2absolutelocation": BlockToAbsoluteLocationReward,
    "block2block_relative_location": BlockToBlockRelativeLocationReward,
    "separate_blocks": SeparateBlocksReward,
    "block1_to_corner": Block1ToCornerLocationReward,
    "play": PlayReward,
}
