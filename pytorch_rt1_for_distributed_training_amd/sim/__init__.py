"""Language-Table simulator without pybullet: board, instruction language, task rewards,
planar pushing world with the reference camera, gym-style env, scripted push oracle, text encoder."""
from . import assets, board, phrases, rrt_star, state_io, tasks
from .board import BlockMode
from .env import LanguageTable
from .oracle import PushOracle, RRTPushOracle, plan_succeeds
from .tasks import FAILURE, REWARDS
from .text import HashedTextEncoder

__all__ = ["assets", "board", "phrases", "state_io", "tasks", "BlockMode", "LanguageTable", "PushOracle", "RRTPushOracle", "rrt_star", "plan_succeeds", "FAILURE",
           "REWARDS", "HashedTextEncoder"]
