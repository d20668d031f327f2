#!/usr/bin/env python3
"""Input-path throughput of N concurrent rank loaders on the host (no GPU): what an 8-GPU node's ranks ask of the
CPU side at the bench config (b128, T=6, 360x640 Language-Table frames).

  python tools/loader_bench.py --ranks 8 --batches 200 [--mode host|plan] [--shard /tmp/lt_bench_shard]

``host``: ``ShardBatchLoader`` -- the raw frames of every batch gathered from the memory-mapped shard into (pageable
here, pinned on a GPU box) host buffers by a thread pool, the path whose batches then cross PCIe.  ``plan``: the
HBM-resident path's host side (``ResidentBatchLoader``): frame rows + crop boxes only; the gather and crop run on the
GPU from resident frames (timed separately on the box: tools/gpu/resident_decode.py).

Each rank is a separate process (like the training ranks); every rank iterates ``--batches`` batches after one
warm-up batch.  The aggregate is the sum of batches over all ranks divided by the slowest rank's wall time.  The node
needs ``N * samples_per_sec_per_gpu / batch`` batches/s (8 x 1283 / 128 ~= 80 at the round-3 bench rate).
"""
from __future__ import annotations

import argparse
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def make_shard(path: str, episodes: int, steps: int, hw):
    from pytorch_rt1_for_distributed_training_amd.data import shards as S
    from pytorch_rt1_for_distributed_training_amd.data.episodes import make_fake_episodes
    if S.is_shard(path):
        return
    src = path + "_npz"
    ids = make_fake_episodes(src, episodes, steps=steps, height=hw[0], width=hw[1], seed=0)
    S.pack_shard(src, ids, path)
    import shutil
    shutil.rmtree(src, ignore_errors=True)


def rank_main(rank, args, q, start):
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    import torch
    torch.set_num_threads(1)
    from pytorch_rt1_for_distributed_training_amd.data import shards as S
    from pytorch_rt1_for_distributed_training_amd.data import resident as R
    if args.mode == "host":
        ld = S.ShardBatchLoader(args.shard, args.batch, args.seq, 0.95, shuffle=True, rank=rank, world=args.ranks,
                                seed=0, threads=args.threads, pin=False, reuse_buffers=4)
    else:
        res = R.ResidentShard(args.shard, "meta", rank=rank, world=args.ranks)
        ld = R.ResidentBatchLoader(res, args.batch, args.seq, 0.95, shuffle=True, seed=0, pin=False)

    def batches():
        ep = 0
        while True:
            ld.set_epoch(ep)
            for b in ld:
                yield b
            ep += 1
    it = batches()
    next(it)
    start.wait()
    t0 = time.perf_counter()
    nbytes = 0
    for _ in range(args.batches):
        b = next(it)
        if args.mode == "host":
            nbytes += b["train_observation"]["raw_frames"].numel()
    dt = time.perf_counter() - t0
    q.put((rank, args.batches, dt, nbytes))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--batches", type=int, default=200)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--seq", type=int, default=6)
    ap.add_argument("--threads", type=int, default=2, help="gather threads per rank (host mode)")
    ap.add_argument("--mode", choices=["host", "plan"], default="host")
    ap.add_argument("--shard", default="/tmp/lt_bench_shard")
    ap.add_argument("--episodes", type=int, default=200)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--hw", type=int, nargs=2, default=[360, 640])
    ap.add_argument("--need", type=float, default=80.0, help="batches/s the node needs (8 x 1283 / 128)")
    args = ap.parse_args()
    t = time.perf_counter()
    make_shard(args.shard, args.episodes, args.steps, args.hw)
    print(f"shard {args.shard} ready ({time.perf_counter() - t:.1f} s); cpus {os.cpu_count()}", flush=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    start = ctx.Barrier(args.ranks + 1)
    procs = [ctx.Process(target=rank_main, args=(r, args, q, start)) for r in range(args.ranks)]
    for p in procs:
        p.start()
    start.wait()
    res = [q.get() for _ in procs]
    for p in procs:
        p.join()
    res.sort()
    wall = max(r[2] for r in res)
    total = sum(r[1] for r in res)
    gbs = sum(r[3] for r in res) / wall / 1e9
    for r, n, dt, nb in res:
        print(f"rank {r}: {n} batches in {dt:.2f} s = {n / dt:.2f} batches/s", flush=True)
    agg = total / wall
    print(f"mode {args.mode}: {args.ranks} ranks x {args.batches} batches (b{args.batch}, T={args.seq}, "
          f"{args.hw[0]}x{args.hw[1]} frames, {args.threads} gather threads/rank): aggregate {agg:.1f} batches/s "
          f"({agg * args.batch:.0f} windows/s; {gbs:.1f} GB/s of frames gathered); node needs {args.need:.0f} "
          f"batches/s -> {'OK' if agg >= 1.1 * args.need else 'SHORT'} (10 % headroom: {1.1 * args.need:.0f})",
          flush=True)


if __name__ == "__main__":
    main()
