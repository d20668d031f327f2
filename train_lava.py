"""Train the LAVA behaviour-cloning policy on one or more GPUs.

Reference: ``language_table/train/main.py`` + ``train.py`` + ``bc.py`` + ``configs/language_table_sim_local.py``
(JAX pmap data parallelism).  Same recipe on the RT-1 runtime: one process per GPU (torchrun), bucketed RCCL
gradient all-reduce, fused Adam (lr 1e-3, eps 1e-7), MSE on normalised actions, periodic logging and
checkpoints, restore-or-init.  Data: scripted demonstrations collected on the in-tree Language-Table board
(``--collect``), or synthetic windows (``--synthetic``); the RLDS datasets are not reachable offline.

  python train_lava.py --collect 40 --steps 200 --batch_size 32
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 train_lava.py --collect 400 --steps 2000
  python train_lava.py --collect 40 --steps 200 --eval_episodes 10     # + closed-loop eval in the sim
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--collect", type=int, default=0, help="oracle episodes to collect in the sim")
    ap.add_argument("--synthetic", type=int, default=0, help="synthetic episodes instead of sim demos")
    ap.add_argument("--rlds", default="", help="RLDS builder directory (TFRecord shards, read without TensorFlow)")
    ap.add_argument("--rlds_limit", type=int, default=0, help="use only the first N RLDS episodes")
    ap.add_argument("--reward", default="block2block")
    ap.add_argument("--oracle", default="push", choices=["push", "rrt"], help="demonstration oracle")
    ap.add_argument("--augment", action="store_true",
                    help="on-device random crop (0.95) + resize + photometric distortions (the reference pipeline)")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--batch_size", type=int, default=32, help="per process")
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--sequence_length", type=int, default=4)
    ap.add_argument("--d_model", type=int, default=128)
    ap.add_argument("--log_every", type=int, default=20)
    ap.add_argument("--ckpt", default="./exp/lava/last.pt")
    ap.add_argument("--ckpt_every", type=int, default=100)
    ap.add_argument("--eval_episodes", type=int, default=0)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--network", choices=["lava", "pixel"], default="lava",
                    help="SequenceLAVMSE (reference default) or PixelLangMSE (networks/pixel.py)")
    ap.add_argument("--freeze_keys", nargs="*", default=[], help="parameter-name substrings to keep frozen")
    ap.add_argument("--pretrained", nargs="*", default=[],
                    help="PATH:CKPT_PREFIX=MODEL_PREFIX[,CKPT_PREFIX=MODEL_PREFIX] pretrained checkpoints")
    a = ap.parse_args(argv)

    import numpy as np
    import torch
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from pytorch_rt1_for_distributed_training_amd.data import normalization, sim_demos
    from pytorch_rt1_for_distributed_training_amd.engine.bc import BCTrainer
    from pytorch_rt1_for_distributed_training_amd.models.lava import LavaConfig, SequenceLAVMSE
    from pytorch_rt1_for_distributed_training_amd.parallel import dist as pdist

    ctx = pdist.init_distributed(a.device)
    torch.manual_seed(a.seed)
    if a.rlds:
        episodes = sim_demos.rlds_episodes(a.rlds, rank=ctx.rank, world_size=ctx.world_size, limit=a.rlds_limit)
    elif a.synthetic or not a.collect:
        episodes = sim_demos.synthetic_episodes(max(a.synthetic, 8), seed=a.seed + ctx.rank)
    else:
        per_rank = max(1, a.collect // ctx.world_size)
        episodes = sim_demos.collect_episodes(per_rank, a.reward, seed=a.seed + 1000 * ctx.rank, oracle=a.oracle)
    ds = sim_demos.WindowDataset(episodes, a.sequence_length)
    stats = None
    if ctx.is_main:
        stats = normalization.compute_dataset_statistics(sim_demos.action_batches(ds), num_samples=len(ds))
    stats = normalization.broadcast_stats(stats)
    cfg = LavaConfig(sequence_length=a.sequence_length, d_model=a.d_model)
    augment = None
    if a.augment:
        from pytorch_rt1_for_distributed_training_amd.data.augment import BCAugment
        augment = BCAugment(seed=a.seed + ctx.rank)
    if a.network == "pixel":
        from pytorch_rt1_for_distributed_training_amd.models.lava import PixelLangMSE
        net = PixelLangMSE(sequence_length=a.sequence_length)
    else:
        net = SequenceLAVMSE(cfg)
    pre = []
    for spec in a.pretrained:
        path, _, reps = spec.partition(":")
        pre.append((path, [tuple(r.split("=", 1)) for r in reps.split(",") if r]))
    trainer = BCTrainer(net, stats, lr=a.lr, device=ctx.device, augment=augment, freeze_keys=a.freeze_keys,
                        pretrained_checkpoints=pre)
    resumed = trainer.restore_or_init(a.ckpt)
    loader = torch.utils.data.DataLoader(ds, batch_size=a.batch_size, shuffle=True, drop_last=len(ds) >= a.batch_size,
                                         collate_fn=sim_demos.collate)
    it = iter(loader)
    t0 = time.perf_counter()
    log = []
    while trainer.step < a.steps:
        try:
            batch = next(it)
        except StopIteration:
            it = iter(loader)
            batch = next(it)
        loss = trainer.train_step(sim_demos.to_device(batch, ctx.device))
        if trainer.step % a.log_every == 0 or trainer.step == a.steps:
            l = float(loss)
            log.append(l)
            if ctx.is_main:
                dt = time.perf_counter() - t0
                print(json.dumps({"step": trainer.step, "loss": round(l, 6),
                                  "samples_per_s": round(a.batch_size * ctx.world_size * a.log_every / dt, 1)}),
                      flush=True)
            t0 = time.perf_counter()
        if trainer.step % a.ckpt_every == 0:
            trainer.save(a.ckpt)
    trainer.save(a.ckpt)
    res = {"final_loss": log[-1] if log else None, "resumed": resumed, "windows": len(ds)}
    if a.eval_episodes and ctx.is_main:
        from pytorch_rt1_for_distributed_training_amd.eval import evaluate, make_sim_env
        from pytorch_rt1_for_distributed_training_amd.eval.policy import LavaPolicy
        pol = LavaPolicy(trainer.model, stats, device=ctx.device)
        env = make_sim_env(a.reward, seed=a.seed + 7)
        res["eval"] = evaluate(pol, env, episodes=a.eval_episodes, max_episode_steps=80,
                               crop=lambda x: x, history_length=1, video_dir=None, name=a.reward)
    if ctx.is_main:
        print(json.dumps(res), flush=True)
    pdist.shutdown()
    return res


if __name__ == "__main__":
    main()
