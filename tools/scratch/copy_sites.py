#!/usr/bin/env python3
"""Debug: where do the per-step D2D copies (__amd_rocclr_copyBuffer) of the hip backend come from?  Counts
aten::copy_ / clone calls during one eager train step by Python call site."""
import collections
import os
import sys
import traceback

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pytorch_rt1_for_distributed_training_amd.config import RT1Config  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.data.synthetic import make_batch  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.models import build_rt1  # noqa: E402

cfg = RT1Config(height=128, width=128, seq_len=6, backend="hip")
eng = TrainEngine(build_rt1(cfg), cfg, order_probe=False, device=torch.device("cuda", 0))
batch = make_batch(8, 6, 128, 128, device="cuda:0")
eng.train_step(batch)
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    eng.train_step(batch)
    torch.cuda.synchronize()
sites = collections.Counter()
for ev in prof.events():
    if ev.name in ("aten::copy_", "aten::clone", "aten::contiguous", "aten::_to_copy", "Memcpy DtoD (Device -> Device)"):
        st = [f for f in (ev.stack or []) if "pytorch_rt1" in f or "torch/autograd" in f]
        sites[(ev.name, st[0] if st else (ev.stack[0] if ev.stack else "?"))] += 1
for (name, site), n in sites.most_common(40):
    print(f"{n:5d}  {name:28s} {site}")
