#!/usr/bin/env python3
"""Debug: which CPU-side ops of one eager hip-backend train step issue device memcpys (the per-step
__amd_rocclr_copyBuffer dispatches of the rocprof table)?  torch.profiler kernel lists per op + innermost package frame."""
import collections
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pytorch_rt1_for_distributed_training_amd.config import RT1Config  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.data.synthetic import make_batch  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine, to_device  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.models import build_rt1  # noqa: E402

res = int(os.environ.get("CS_RES", "128"))
cfg = RT1Config(height=res, width=res, seq_len=6, backend="hip")
dev = torch.device("cuda", 0)
eng = TrainEngine(build_rt1(cfg), cfg, order_probe=False, device=dev, graph=False)
batch = to_device(make_batch(8, 6, res, res), dev)
eng.train_step(batch)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    eng.train_step(batch)
    torch.cuda.synchronize()
cnt = collections.Counter()
kinds = collections.Counter()
for ev in prof.events():
    if ev.device_type.name != "CPU":
        continue
    ks = [k for k in (ev.kernels or []) if "emcpy" in k.name or "opyBuffer" in k.name or "emset" in k.name]
    if not ks:
        continue
    site = "?"
    for fr in (ev.stack or []):
        if "pytorch_rt1_for_distributed_training_amd" in fr:
            site = fr.split("pytorch_rt1_for_distributed_training_amd/")[-1]
            break
    for k in ks:
        cnt[(ev.name, k.name[:40], site)] += 1
        kinds[k.name[:40]] += 1
print("memcpy-like device ops by issuing CPU op:")
for (n, k, site), c in cnt.most_common(80):
    print(f"{c:5d}  {n[:40]:40s} {k:40s} {site}")
print(kinds)
