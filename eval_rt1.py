"""Closed-loop evaluation of an RT-1 checkpoint (reference: ``language_table/eval/main_rt1.py``).

  python eval_rt1.py --ckpt exp/ckpt/exp_rt1/last.ckpt --env toy --episodes 10
  python eval_rt1.py --ckpt ... --env sim --reward block2block   # in-tree Language-Table board (sim/)
  python eval_rt1.py --ckpt ... --env language_table     # needs pybullet + language_table + a USE encoder

Protocol kept from the reference: BlockToBlock reward, 10 episodes, at most 80
(+1) policy steps, 456x256 central crop with factor 0.95, 6-frame history, the
policy state zeroed per episode, actions clipped to +-0.03.
"""
from __future__ import annotations

import argparse
import json
import sys


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--ckpt", required=True)
    ap.add_argument("--env", choices=["sim", "toy", "language_table"], default="sim")
    ap.add_argument("--reward", default="block2block", help="sim task family (sim.REWARDS)")
    ap.add_argument("--block_mode", default="BLOCK_8")
    ap.add_argument("--no_reject", action="store_true", help="sim: keep boards the scripted oracle cannot solve")
    ap.add_argument("--episodes", type=int, default=10)
    ap.add_argument("--max_episode_steps", type=int, default=80)
    ap.add_argument("--workdir", default="./exp/eval")
    ap.add_argument("--height", type=int, default=256)
    ap.add_argument("--width", type=int, default=456)
    ap.add_argument("--seq_len", type=int, default=6)
    ap.add_argument("--num_layers", type=int, default=8)
    ap.add_argument("--random_crop_factor", type=float, default=0.95)
    ap.add_argument("--device", default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no_video", action="store_true")
    a = ap.parse_args(argv)

    import torch
    from pytorch_rt1_for_distributed_training_amd.config import RT1Config
    from pytorch_rt1_for_distributed_training_amd.eval import (CentralCropResize, RT1Policy, ToyPushEnv, evaluate,
                                                               make_language_table_env, make_sim_env)
    torch.manual_seed(a.seed)
    device = a.device or ("cuda" if torch.cuda.is_available() else "cpu")
    cfg = RT1Config(height=a.height, width=a.width, seq_len=a.seq_len, num_layers=a.num_layers)
    policy = RT1Policy.from_checkpoint(a.ckpt, cfg, device=device)
    if a.env == "sim":
        env = make_sim_env(a.reward, a.block_mode, seed=a.seed, reject_unsolvable=not a.no_reject)
    elif a.env == "toy":
        env = ToyPushEnv(seed=a.seed)
    else:
        env = make_language_table_env(seed=a.seed)
    res = evaluate(policy, env, episodes=a.episodes, max_episode_steps=a.max_episode_steps, name=a.reward,
                   crop=CentralCropResize(a.width, a.height, a.random_crop_factor), history_length=a.seq_len,
                   video_dir=None if a.no_video else f"{a.workdir}/videos")
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
