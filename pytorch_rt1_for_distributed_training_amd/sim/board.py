"""Language-Table board: workspace geometry, camera, and the block catalogue.

Behavioural spec: ``language_table/environments/constants.py:22-65`` (workspace bounds,
camera pose/intrinsics, spawn thresholds, 512-byte instruction field, 180x320 images) and
``language_table/environments/blocks.py:24-160`` (block variants, the fixed 4/8-block sets, and the
N-choose-K subsets of the 16 colour x shape blocks split 90/10 into train/test after a seeded shuffle).
The numbers are the reference's; the code is a plain-Python catalogue (the planar simulator in ``sim.world``
models each block as a rigid footprint; ``sim.assets`` writes matching OBJ / URDF files for tools that want them).
"""
from __future__ import annotations

import enum
import itertools
import math
from typing import List, Sequence, Tuple

import numpy as np

# ---------------------------------------------------------------- workspace (metres, robot base frame)
X_MIN, X_MAX = 0.15, 0.6
Y_MIN, Y_MAX = -0.3048, 0.3048
CENTER_X = (X_MAX - X_MIN) / 2.0 + X_MIN
CENTER_Y = (Y_MAX - Y_MIN) / 2.0 + Y_MIN
WORKSPACE_BOUNDS = np.array(((X_MIN, Y_MIN), (X_MAX, Y_MAX)))
WORKSPACE_BOUNDS_BUFFER = 0.08          # spawn / target margin
BLOCK_DISTANCE_THRESHOLD = 0.0175       # min centre distance between spawned blocks
ARM_DISTANCE_THRESHOLD = 0.06           # min spawn distance from the effector
EFFECTOR_HEIGHT = 0.145
INSTRUCTION_LENGTH = 512                # bytes of the encoded instruction observation
TARGET_BLOCK_DISTANCE = 0.05            # block-to-block success radius (rewards/constants.py)

# ---------------------------------------------------------------- camera (RealSense-like, tiny renderer)
IMAGE_HEIGHT, IMAGE_WIDTH = 180, 320
CAMERA_POSE = (0.75, 0.0, 0.5)
CAMERA_ORIENTATION = (math.pi / 5, math.pi, -math.pi / 2)   # roll, pitch, yaw
FOCAL_PX = 0.803 * IMAGE_WIDTH

# ---------------------------------------------------------------- blocks
COLORS = ["red", "blue", "green", "yellow"]
SHAPES = ["moon", "cube", "star", "pentagon"]
ALL_BLOCKS = ["_".join(cs) for cs in itertools.product(COLORS, SHAPES)]
RGB = {"red": (214, 54, 54), "blue": (52, 96, 210), "green": (56, 168, 76), "yellow": (232, 200, 48),
       "purple": (140, 70, 170)}


class BlockMode(enum.Enum):
    BLOCK_1 = "BLOCK_1"
    BLOCK_4 = "BLOCK_4"
    BLOCK_8 = "BLOCK_8"
    BLOCK_4_WPOLE = "BLOCK_4_WPOLE"
    BLOCK_8_WPOLE = "BLOCK_8_WPOLE"
    N_CHOOSE_K = "N_CHOOSE_K"


FIXED_1 = ("green_star",)
FIXED_4 = ("red_moon", "blue_cube", "green_star", "yellow_pentagon")
FIXED_8 = ("red_moon", "red_pentagon", "blue_moon", "blue_cube", "green_cube", "green_star", "yellow_star",
           "yellow_pentagon")
FIXED_4_WPOLE = FIXED_4 + ("purple_pole",)
FIXED_8_WPOLE = FIXED_8 + ("purple_pole",)
MIN_K, MAX_K = 4, 10


def _n_choose_k_split() -> Tuple[List[tuple], List[tuple]]:
    combos: List[tuple] = []
    for k in range(MIN_K, MAX_K + 1):
        combos.extend(itertools.combinations(ALL_BLOCKS, k))
    np.random.RandomState(seed=0).shuffle(combos)      # same seeded shuffle -> same train/test split
    cut = int(len(combos) * 0.9)
    return combos[:cut], combos[cut:]


_SPLIT = None


def n_choose_k_split():
    global _SPLIT
    if _SPLIT is None:
        _SPLIT = _n_choose_k_split()
    return _SPLIT


def block_subsets(mode: BlockMode, training: bool = True) -> Sequence[tuple]:
    """Every block set the env may put on the table for ``mode`` (``get_all_block_subsets``)."""
    fixed = {BlockMode.BLOCK_1: FIXED_1, BlockMode.BLOCK_4: FIXED_4, BlockMode.BLOCK_8: FIXED_8,
             BlockMode.BLOCK_4_WPOLE: FIXED_4_WPOLE, BlockMode.BLOCK_8_WPOLE: FIXED_8_WPOLE}
    if mode in fixed:
        return [fixed[mode]]
    if mode == BlockMode.N_CHOOSE_K:
        train, test = n_choose_k_split()
        return train if training else test
    raise ValueError(f"unsupported block mode {mode}")


def block_set(mode: BlockMode) -> Sequence[str]:
    """The distinct blocks of a mode (used to enumerate instructions)."""
    table = {BlockMode.BLOCK_1: FIXED_1, BlockMode.BLOCK_4: FIXED_4, BlockMode.BLOCK_8: FIXED_8,
             BlockMode.N_CHOOSE_K: tuple(ALL_BLOCKS)}
    if mode not in table:
        raise ValueError(f"unsupported block mode {mode}")
    return table[mode]


def block_text(block: str) -> str:
    return block.replace("_", " ")


def blocks_text(mode: BlockMode) -> List[str]:
    return [block_text(b) for b in block_set(mode)]


def color_shape(block: str) -> Tuple[str, str]:
    c, s = block.split("_")
    return c, s


def all_block_names() -> List[str]:
    """Every block the simulator knows (the 16 colour x shape blocks + the goal pole)."""
    return list(ALL_BLOCKS) + ["purple_pole"]
