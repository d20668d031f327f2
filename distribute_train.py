"""RT-1 training entrypoint (MI355X / ROCm).

Same flags as the reference ``distribute_train.py:270-293`` (``--device --gpus
--max_epochs --batch_size --num_workers --milestones --lr --exp_name --log_dir
--ckpt_dir --log_every_n_steps --ckpt_every_n_epochs --dataset_dir
--train_episode --test_episode --eval_episode --random_crop_factor --height
--width --seq_len``) plus framework flags (``--mode``, ``--synthetic``,
``--resume``, ``--dtype``, ``--backend``, ...).

Launch:
  single GPU / CPU:   python distribute_train.py --gpus 0 ...
  one node, N GPUs:   python distribute_train.py --gpus 0,1,2,3 ...   (spawns one process per GPU)
                  or  torchrun --nproc-per-node N --master-addr 127.0.0.1 distribute_train.py ...
``--mode debug`` reproduces the reference's default smoke test (``debug()``,
``:250-266``): one train-mode forward at B=2 and one inference step at B=1.
"""
from __future__ import annotations

import argparse
import os

import numpy as np
import subprocess
import sys


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    # ---- reference flags
    p.add_argument("--device", type=str, default="gpu")
    p.add_argument("--gpus", type=str, default="0")
    p.add_argument("--max_epochs", type=int, default=100)
    p.add_argument("--batch_size", type=int, default=8)
    p.add_argument("--num_workers", type=int, default=15)
    p.add_argument("--milestones", type=int, nargs="+", default=[50, 75, 90])
    p.add_argument("--lr", type=float, default=5e-4)
    p.add_argument("--exp_name", type=str, default="exp_rt1")
    p.add_argument("--log_dir", type=str, default="./exp/logs")
    p.add_argument("--ckpt_dir", type=str, default="./exp/ckpt")
    p.add_argument("--log_every_n_steps", type=int, default=500)
    p.add_argument("--ckpt_every_n_epochs", type=int, default=1)
    p.add_argument("--dataset_dir", type=str, default="./data/language_table_b2b_npz")
    p.add_argument("--train_episode", type=int, default=7800)
    p.add_argument("--test_episode", type=int, default=50)
    p.add_argument("--eval_episode", type=int, default=50)
    p.add_argument("--random_crop_factor", type=float, default=0.95)
    p.add_argument("--height", type=int, default=256)
    p.add_argument("--width", type=int, default=456)
    p.add_argument("--seq_len", type=int, default=6)
    # ---- framework flags
    p.add_argument("--mode", choices=["train", "debug"], default="train")
    p.add_argument("--synthetic", action="store_true", help="synthetic windows of the real shapes (no dataset)")
    p.add_argument("--synthetic_samples", type=int, default=4096)
    p.add_argument("--resume", type=str, default=None, help="checkpoint to resume from (e.g. .../last.ckpt)")
    p.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16")
    p.add_argument("--backend", choices=["auto", "hip", "torch"], default="auto")
    p.add_argument("--num_layers", type=int, default=8)
    p.add_argument("--weight_decay", type=float, default=0.0, help="AdamW decoupled decay (0 = Adam, reference)")
    p.add_argument("--bucket_cap_mb", type=float, default=32.0)
    p.add_argument("--no_broadcast_buffers", action="store_true")
    p.add_argument("--comm", choices=["torch", "native"], default="torch",
                    help="gradient collectives: torch ProcessGroup (RCCL) or the native C++ RCCL communicator")
    p.add_argument("--limit_train_batches", type=int, default=None)
    p.add_argument("--limit_val_batches", type=int, default=None)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--graph", choices=["auto", "on", "off"], default="auto",
                   help="hipGraph training step (auto = on for the hip backend on GPU; the step bench.py measures)")
    p.add_argument("--pretrained", type=str, default=None,
                   help="torchvision efficientnet_b3 state dict for the backbone (reference weights='imagenet')")
    p.add_argument("--data_format", choices=["auto", "npz", "shard"], default="auto",
                   help="episode storage: per-episode .npz (CPU PIL crop) or a packed shard (GPU crop+resize)")
    p.add_argument("--data_residency", choices=["auto", "host", "hbm"], default="auto",
                   help="packed shards: 'hbm' keeps each rank's episodes resident on its GPU (one copy at start, no "
                        "per-step frame H2D; data/resident.py), 'host' gathers raw frames into pinned batches every "
                        "step; 'auto' = hbm on GPU when the rank's frames fit --hbm_data_gb")
    p.add_argument("--hbm_data_gb", type=float, default=96.0,
                   help="HBM budget per rank for resident training frames (of 288 GB per MI355X)")
    return p


def _spawn_local(args) -> int:
    """One process per listed GPU (what Lightning's DDP launcher does for the reference), via the shared
    launcher (``parallel/launch.py``): children are fresh processes, the parent never touches the GPU."""
    from pytorch_rt1_for_distributed_training_amd.parallel.launch import spawn_local
    gpus = [g for g in args.gpus.split(",") if g.strip() != ""]
    return spawn_local(len(gpus), sys.argv, {"CUDA_VISIBLE_DEVICES": ",".join(gpus)})


def make_config(args):
    from pytorch_rt1_for_distributed_training_amd.config import RT1Config
    return RT1Config(height=args.height, width=args.width, seq_len=args.seq_len, num_layers=args.num_layers,
                     dtype=args.dtype, backend=args.backend, pretrained=getattr(args, "pretrained", None))


def make_loaders(args, cfg, ctx):
    import torch
    from torch.utils.data import DataLoader
    from torch.utils.data.distributed import DistributedSampler
    from pytorch_rt1_for_distributed_training_amd import data as D

    def loader(ds, shuffle):
        sampler = DistributedSampler(ds, ctx.world_size, ctx.rank, shuffle=shuffle) if ctx.distributed else None
        return DataLoader(ds, batch_size=args.batch_size, shuffle=(shuffle and sampler is None), sampler=sampler,
                          collate_fn=D.collate_fn, num_workers=args.num_workers,
                          pin_memory=ctx.device.type == "cuda", drop_last=shuffle,
                          persistent_workers=args.num_workers > 0)

    if args.synthetic:
        mk = lambda n, seed: D.SyntheticDataset(n, cfg.seq_len, cfg.height, cfg.width, seed=seed, uint8=True)
        return (loader(mk(args.synthetic_samples, 0), True), loader(mk(max(args.batch_size * 2, 16), 1), False),
                loader(mk(max(args.batch_size * 2, 16), 2), False))
    root = args.dataset_dir
    fmt = getattr(args, "data_format", "auto")
    if fmt == "shard" or (fmt == "auto" and D.is_shard(os.path.join(root, "train"))):
        # packed shards: raw frames gathered into pinned batches by threads; crop+resize on the GPU
        def shard(split, shuffle, bs):
            return D.ShardBatchLoader(os.path.join(root, split), bs, cfg.seq_len, args.random_crop_factor,
                                      shuffle=shuffle, rank=ctx.rank, world=ctx.world_size, seed=args.seed,
                                      drop_last=shuffle, threads=max(2, min(args.num_workers, 16)),
                                      pin=ctx.device.type == "cuda")
        train = _resident_train_loader(args, cfg, ctx, os.path.join(root, "train"))
        if train is None:
            train = shard("train", True, args.batch_size)
        return train, shard("test", False, args.batch_size), shard("val", False, args.batch_size)
    tf = D.DecodeAndRandomResizedCrop(args.random_crop_factor, (args.width, args.height), as_uint8=True)
    for split in ("train", "test", "val"):
        if not os.path.isdir(os.path.join(root, split)):
            raise SystemExit(f"dataset split {os.path.join(root, split)} not found (use --synthetic, or convert the "
                             f"Language-Table episodes with data.convert_reference_episodes)")
    train = D.EpisodeWindowDataset(os.path.join(root, "train"), range(args.train_episode), cfg.seq_len, tf)
    test = D.EpisodeWindowDataset(os.path.join(root, "test"), range(args.test_episode), cfg.seq_len, tf)
    val = D.EpisodeWindowDataset(os.path.join(root, "val"), range(args.eval_episode), cfg.seq_len, tf)
    return loader(train, True), loader(test, False), loader(val, False)


def _resident_train_loader(args, cfg, ctx, path):
    """The HBM-resident training loader (data/resident.py) when --data_residency asks for it (or 'auto' finds the
    rank's frames within --hbm_data_gb on a GPU); None selects the host-gather loader."""
    from pytorch_rt1_for_distributed_training_amd.data import resident as R
    from pytorch_rt1_for_distributed_training_amd.data.shards import Shard
    mode = getattr(args, "data_residency", "auto")
    if mode == "host" or (mode == "auto" and ctx.device.type != "cuda"):
        return None
    sh = Shard(path)
    try:
        eps = R.assign_episodes(sh.lengths, ctx.world_size, args.seed)[ctx.rank]
    except ValueError as e:          # fewer episodes than ranks
        if mode == "hbm":
            raise
        if ctx.is_main:
            print(f"[data] {e}: host-gather path", flush=True)
        return None
    need_gb = float(sh.lengths[eps].sum()) * float(np.prod(sh.frame_shape)) / 2 ** 30
    if mode == "auto" and need_gb > args.hbm_data_gb:
        if ctx.is_main:
            print(f"[data] {need_gb:.1f} GB of frames per rank > --hbm_data_gb {args.hbm_data_gb}: host-gather path",
                  flush=True)
        return None
    res = R.ResidentShard(path, ctx.device, rank=ctx.rank, world=ctx.world_size, max_gb=args.hbm_data_gb,
                          seed=args.seed)
    if ctx.is_main:
        print(f"[data] resident training frames: {res.frames.shape[0]} frames, {res.nbytes / 2 ** 30:.2f} GB per rank, "
              f"loaded in {res.load_s:.1f} s", flush=True)
    return R.ResidentBatchLoader(res, args.batch_size, cfg.seq_len, args.random_crop_factor, shuffle=True,
                                 seed=args.seed, drop_last=True)


def _batch_transform(train_loader, cfg):
    from pytorch_rt1_for_distributed_training_amd.data.resident import ResidentBatchLoader, decode_resident
    from pytorch_rt1_for_distributed_training_amd.data.shards import decode_on_device
    res = train_loader.res if isinstance(train_loader, ResidentBatchLoader) else None

    def transform(b):
        if res is not None and "plan_rows" in b:
            return decode_resident(res, b, cfg.height, cfg.width)
        return decode_on_device(b, cfg.height, cfg.width)
    return transform


def train(args):
    import torch
    from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine
    from pytorch_rt1_for_distributed_training_amd.engine.trainer import Trainer
    from pytorch_rt1_for_distributed_training_amd.models import build_rt1
    from pytorch_rt1_for_distributed_training_amd.parallel import dist as pdist
    from pytorch_rt1_for_distributed_training_amd.utils.checkpoint import ModelCheckpoint
    from pytorch_rt1_for_distributed_training_amd.utils.logging import CSVLogger, MultiLogger, TensorBoardLogger

    ctx = pdist.init_distributed("cpu" if args.device == "cpu" else "auto")
    torch.manual_seed(args.seed + ctx.rank)
    cfg = make_config(args)
    train_loader, test_loader, eval_loader = make_loaders(args, cfg, ctx)
    if ctx.is_main:
        print(f"Building RT-1 (world={ctx.world_size}, device={ctx.device}, dtype={cfg.dtype})", flush=True)
    torch.manual_seed(args.seed)  # identical init on every rank (rank 0 broadcasts anyway)
    model = build_rt1(cfg)
    # --graph auto: the hipGraph step (segmented graph-DP with several ranks), the step bench.py measures.  The trainer
    # checks it once against the eager bucketed DP step on the first batch (bitwise, every rank) and falls back to the
    # eager step if they differ (Trainer._check_graph)
    use_graph = args.graph in ("on", "auto")
    engine = TrainEngine(model, cfg, lr=args.lr, milestones=args.milestones, weight_decay=args.weight_decay,
                         bucket_cap_mb=args.bucket_cap_mb, broadcast_buffers=not args.no_broadcast_buffers,
                         comm=args.comm, graph=use_graph)
    ckpt = ModelCheckpoint(os.path.join(args.ckpt_dir, args.exp_name), every_n_epochs=args.ckpt_every_n_epochs)
    loggers = []
    if ctx.is_main:
        loggers = [CSVLogger(os.path.join(args.log_dir, "csv"), args.exp_name),
                   TensorBoardLogger(os.path.join(args.log_dir, "tb"), args.exp_name)]
    trainer = Trainer(engine, args.max_epochs, args.log_every_n_steps, ckpt, MultiLogger(loggers),
                      args.limit_train_batches, args.limit_val_batches,
                      batch_transform=_batch_transform(train_loader, cfg))
    if args.resume:
        trainer.resume(args.resume)
    if ctx.is_main:
        print("Start Training ...", flush=True)
    trainer.fit(train_loader, eval_loader)
    if ctx.is_main:
        print("Start Final Testing ...", flush=True)
    trainer.test(test_loader, args.limit_val_batches)
    pdist.shutdown()


def debug(args):
    """Reference ``debug()``: train-mode forward (B=2) then one inference step (B=1)."""
    import torch
    from pytorch_rt1_for_distributed_training_amd.models import build_rt1
    from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine
    from pytorch_rt1_for_distributed_training_amd.parallel import dist as pdist

    ctx = pdist.init_distributed("cpu" if args.device == "cpu" else "auto")
    cfg = make_config(args)
    model = build_rt1(cfg)
    eng = TrainEngine(model, cfg, order_probe=False)
    dev, T, H, W = ctx.device, cfg.seq_len, cfg.height, cfg.width
    batch = {"train_observation": {"image": torch.full((2, T, 3, H, W), 0.5, device=dev),
                                   "natural_language_embedding": torch.full((2, T, 512), 1.0, device=dev)},
             "action_label": {"terminate_episode": torch.full((2, T), 1, device=dev),
                              "action": torch.zeros(2, T, 2, device=dev)}}
    print("=========Training Debug=========")
    eng.model.train()
    with eng.autocast():
        eng.model.set_actions(batch["action_label"])
        loss_bt, aux = eng.model.train_forward(batch["train_observation"]["image"],
                                               batch["train_observation"]["natural_language_embedding"],
                                               batch["action_label"])
    pred = eng.model._action_tokenizer.detokenize(aux["predicted_tokens_for_output"])
    print(f"pred_action:{tuple(pred['action'].shape)}")
    print(f"is_terminate:{tuple(pred['terminate_episode'].shape)}")
    print(f"action_loss:{tuple(loss_bt.shape)}, mean_loss:{float(loss_bt.mean()):.6f}")
    print("=========Inference Debug=========")
    eng.model.eval()
    state = eng.model.initial_state(1, dev)
    with eng.autocast():
        pred, state = eng.model({"image": torch.full((1, 3, H, W), 0.5, device=dev),
                                 "natural_language_embedding": torch.full((1, 512), 1.0, device=dev)}, state)
    print(f"pred_action:{tuple(pred['action'].shape)}")
    print(f"is_terminate:{tuple(pred['terminate_episode'].shape)}")
    print(f"seq_idx:{state['seq_idx'].tolist()}")


def main(argv=None):
    args = build_parser().parse_args(argv)
    gpus = [g for g in args.gpus.split(",") if g.strip() != ""]
    if args.mode == "train" and args.device != "cpu" and len(gpus) > 1 and "RANK" not in os.environ:
        return _spawn_local(args)
    if "RANK" not in os.environ and args.device != "cpu" and len(gpus) == 1:
        os.environ.setdefault("CUDA_VISIBLE_DEVICES", gpus[0])
    if args.device != "cpu":
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from pytorch_rt1_for_distributed_training_amd.utils.tuned_gemms import enable_tuned_gemms
        enable_tuned_gemms()          # recorded hipBLASLt solutions (before the first GEMM)
    if args.mode == "debug":
        debug(args)
    else:
        train(args)
    return 0


if __name__ == "__main__":
    sys.exit(main())
