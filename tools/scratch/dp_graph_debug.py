#!/usr/bin/env python3
"""Debug: where does the graph-DP step's gradient differ from the eager-DP step's?  2 ranks on one GPU (gloo).

  torchrun --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 tools/scratch/dp_graph_debug.py
Runs three variants for 2 steps: 4 MB buckets with all-reduce, 4 MB buckets without any all-reduce (local grads),
one bucket with all-reduce; after step 2 prints every parameter whose gradient differs.
"""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import pytorch_rt1_for_distributed_training_amd as rt1  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.data.synthetic import make_batch  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.models import build_rt1  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.parallel import dist as pdist  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.parallel.ddp import DataParallel  # noqa: E402


def diffs(eng, a, b):
    names = {id(p): n for n, p in eng.model.named_parameters()}
    out = []
    for i, p in enumerate(eng.flat.params):
        off, n = eng.flat.segment(i)
        d = float((a[off:off + n] - b[off:off + n]).abs().max())
        if d != 0:
            out.append((names[id(p)], d, float(b[off:off + n].abs().max()), eng.ddp._param_bucket[i]))
    return out


def run(ctx, cfg, cap_mb, comm, order_probe, steps=2):
    orig = DataParallel._all_reduce
    if not comm:
        DataParallel._all_reduce = lambda self, t: None
    try:
        torch.manual_seed(0)
        eg = TrainEngine(build_rt1(cfg), cfg, order_probe=order_probe, bucket_cap_mb=cap_mb, graph=True)
        torch.manual_seed(0)
        ee = TrainEngine(build_rt1(cfg), cfg, order_probe=order_probe, bucket_cap_mb=cap_mb, graph=False)
        g = torch.Generator().manual_seed(100 + ctx.rank)
        batches = [make_batch(4, cfg.seq_len, 128, 128, device=ctx.device, generator=g) for _ in range(steps)]
        for s, batch in enumerate(batches):
            eg.train_step(batch)
            ee.train_step(batch)
            torch.cuda.synchronize()
            d = diffs(eg, eg.flat.grad, ee.flat.grad)
            if ctx.rank == 0:
                print(f"[cap {cap_mb} comm {comm} probe {order_probe}] step {s + 1}: {len(d)} params differ "
                      f"(buckets {len(eg.ddp.buckets)})", flush=True)
                for name, dd, mx, bk in d[:40]:
                    print(f"     {name}: max|diff| {dd:.3e} (max|g| {mx:.3e}) bucket {bk}", flush=True)
        # replay the graph twice on the same batch: is the graph itself deterministic?
        gl = []
        for _ in range(2):
            eg._copy_done = None
            eg.optimizer.zero_grad(set_to_none=False)
            eg._static_batch_ref = None
            eg._segments.replay_with(lambda b: None)
            torch.cuda.synchronize()
            gl.append(eg.flat.grad.clone())
        if ctx.rank == 0:
            print(f"   graph replay twice on one batch: equal {torch.equal(gl[0], gl[1])}", flush=True)
    finally:
        DataParallel._all_reduce = orig


def main():
    ctx = pdist.init_distributed("cuda", backend="gloo")
    cfg = rt1.RT1Config(height=128, width=128, seq_len=6, backend="hip", dropout_rate=0.0, drop_connect_rate=0.0,
                        crop_ratio=0.0)
    run(ctx, cfg, 4.0, True, True)
    run(ctx, cfg, 4.0, False, True)
    run(ctx, cfg, 4.0, True, False)
    run(ctx, cfg, 1e4, True, True)
    pdist.shutdown()


if __name__ == "__main__":
    main()
