#!/usr/bin/env python3
"""Step the in-tree Language-Table board and save the rollout as a GIF (the role of the reference's
``language_table/examples/environment_example.py``).

  python examples/environment_example.py --reward block2block --oracle rrt --steps 60 --out /tmp/lt.gif
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_rt1_for_distributed_training_amd.eval import save_gif  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.sim import REWARDS, BlockMode, LanguageTable  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.sim.oracle import PushOracle, RRTPushOracle  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--reward", default="block2block", choices=sorted(REWARDS))
    ap.add_argument("--block_mode", default="BLOCK_8", choices=[m.name for m in BlockMode])
    ap.add_argument("--oracle", default="rrt", choices=["rrt", "push", "random"])
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    env = LanguageTable(BlockMode[a.block_mode], reward_factory=REWARDS[a.reward], seed=a.seed)
    obs = env.reset()
    print("instruction:", env.instruction_str)
    print("observation:", {k: (v.shape, v.dtype) for k, v in obs.items()})
    policy = {"rrt": RRTPushOracle, "push": PushOracle}.get(a.oracle)
    oracle = policy(env) if policy else None
    rng = np.random.default_rng(a.seed)
    frames, total = [env.render()], 0.0
    for t in range(a.steps):
        act = oracle.action() if oracle else rng.uniform(-0.03, 0.03, 2).astype(np.float32)
        obs, reward, done, _ = env.step(act)
        total += reward
        frames.append(env.render())
        if done:
            print(f"solved at step {t + 1}")
            break
    print(f"return {total:.1f}  effector {obs['effector_translation']}  arm joints "
          f"{np.round(env.robot.get_joint_positions(), 3) if env.robot is not None else None}")
    if a.out:
        save_gif(frames, a.out)
        print("wrote", a.out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
