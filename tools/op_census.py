#!/usr/bin/env python3
"""Which torch-level ops launch GPU kernels inside one hip-backend training step (everything that is not one of the
framework's own HIP kernels): aten op name x calls, with the innermost package source line of each call site.

  python tools/op_census.py [--batch 128] [--res 300]
"""
from __future__ import annotations

import argparse
import collections
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--res", type=int, default=300)
    a = ap.parse_args()
    from pytorch_rt1_for_distributed_training_amd.config import RT1Config
    from pytorch_rt1_for_distributed_training_amd.data.synthetic import make_batch
    from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine, to_device
    from pytorch_rt1_for_distributed_training_amd.models import build_rt1

    dev = torch.device("cuda", 0)
    cfg = RT1Config(height=a.res, width=a.res, seq_len=6, backend="hip")
    eng = TrainEngine(build_rt1(cfg), cfg, order_probe=False, device=dev)
    batch = to_device(make_batch(a.batch, cfg.seq_len, cfg.height, cfg.width), dev)
    eng.train_step(batch)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        eng.train_step(batch)
        torch.cuda.synchronize()
    cnt = collections.Counter()
    for ev in prof.events():
        if ev.device_type.name != "CPU" or not ev.name.startswith("aten::"):
            continue
        if ev.name in ("aten::empty", "aten::empty_strided", "aten::view", "aten::as_strided", "aten::reshape",
                       "aten::t", "aten::transpose", "aten::slice", "aten::select", "aten::split",
                       "aten::narrow", "aten::unsqueeze", "aten::squeeze", "aten::permute", "aten::expand",
                       "aten::detach", "aten::alias", "aten::_reshape_alias", "aten::resize_", "aten::lift_fresh",
                       "aten::split_with_sizes", "aten::unbind", "aten::chunk"):
            continue
        if not ev.kernels:
            # only ops that launched device work directly
            continue
        site = "?"
        for fr in (ev.stack or []):
            if "pytorch_rt1_for_distributed_training_amd" in fr and "op_census" not in fr:
                site = fr.split("pytorch_rt1_for_distributed_training_amd/")[-1]
                break
        cnt[(ev.name, site)] += 1
    tot = sum(cnt.values())
    print(f"{tot} torch ops with device kernels in one step")
    for (n, site), c in cnt.most_common(60):
        print(f"{c:5d}  {n:28s} {site}")


if __name__ == "__main__":
    main()
