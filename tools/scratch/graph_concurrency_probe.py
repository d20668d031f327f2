#!/usr/bin/env python3
"""Debug: is a 1-GPU whole-step graph replay deterministic while ANOTHER process keeps the same GPU busy?

  torchrun --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29536 tools/scratch/graph_concurrency_probe.py
Rank 0 (no DP: each rank is its own world-of-1 engine) captures the forward+backward+gather of a graph step and
replays it N times on one batch with lr=0, comparing gradients bitwise.  Phase A: rank 1 idles.  Phase B: rank 1
runs eager steps of its own engine concurrently.
"""
from __future__ import annotations

import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import pytorch_rt1_for_distributed_training_amd as rt1  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.data.synthetic import make_batch  # noqa: E402


def main():
    rank = int(os.environ["RANK"])
    os.environ["WORLD_SIZE"] = "1"          # engines below are single-rank; ranks coordinate through files
    flag = "/tmp/rt1_gconc_"
    from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine
    from pytorch_rt1_for_distributed_training_amd.models import build_rt1
    from pytorch_rt1_for_distributed_training_amd.parallel import dist as pdist
    torch.cuda.set_device(0)
    cfg = rt1.RT1Config(height=128, width=128, seq_len=6, backend="hip", dropout_rate=0.0, drop_connect_rate=0.0,
                        crop_ratio=0.0)
    torch.manual_seed(0)
    eng = TrainEngine(build_rt1(cfg), cfg, order_probe=False, graph=(rank == 0), device=torch.device("cuda", 0))
    eng.optimizer.param_groups[0]["lr"] = 0.0
    g = torch.Generator().manual_seed(5)
    batch = make_batch(4, cfg.seq_len, 128, 128, device="cuda:0", generator=g)
    eng.train_step(batch)                     # rank 0: eager + capture
    torch.cuda.synchronize()
    open(flag + f"ready{rank}", "w").close()
    while not all(os.path.exists(flag + f"ready{r}") for r in (0, 1)):
        time.sleep(0.1)
    if rank == 0:
        for phase in ("idle", "busy"):
            if phase == "busy":
                open(flag + "busy", "w").close()
                time.sleep(2.0)
            ref, bad = None, 0
            for i in range(12):
                eng.train_step(batch)
                torch.cuda.synchronize()
                gr = eng.flat.grad.clone()
                if ref is None:
                    ref = gr
                elif not torch.equal(gr, ref):
                    bad += 1
            print(f"[{phase}] rank-0 graph replays differing from the first: {bad}/11", flush=True)
        open(flag + "done", "w").close()
    else:
        while not os.path.exists(flag + "busy"):
            time.sleep(0.05)
        n = 0
        while not os.path.exists(flag + "done"):
            eng.train_step(batch)
            torch.cuda.synchronize()
            n += 1
        print(f"rank 1 ran {n} eager steps", flush=True)


if __name__ == "__main__":
    main()
