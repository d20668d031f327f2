#!/usr/bin/env python3
"""Debug: where do the per-step D2D copies (__amd_rocclr_copyBuffer) of the hip backend come from?  Counts the
aten copy-like ops dispatched during one eager train step (a TorchDispatchMode, so copies issued from inside the
C++ bindings are caught too) by the innermost Python frame of this package."""
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pytorch_rt1_for_distributed_training_amd.config import RT1Config  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.data.synthetic import make_batch  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.models import build_rt1  # noqa: E402

WATCH = ("copy_", "clone", "_to_copy", "contiguous", "cat", "stack", "index_put", "copy", "zero_", "fill_",
         "_foreach_copy_", "new_zeros", "zeros_like")


class Sites(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.sites = collections.Counter()
        self.ops = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.overloadpacket.__name__
        self.ops[name] += 1
        if any(name == w or name.startswith(w) for w in WATCH):
            st = [f for f in traceback.extract_stack() if "pytorch_rt1" in f.filename or "torch/autograd" in f.filename]
            site = f"{os.path.basename(st[-1].filename)}:{st[-1].lineno} {st[-1].name}" if st else "?"
            self.sites[(name, site)] += 1
        return func(*args, **(kwargs or {}))


res = int(os.environ.get("CS_RES", "128"))
cfg = RT1Config(height=res, width=res, seq_len=6, backend="hip")
eng = TrainEngine(build_rt1(cfg), cfg, order_probe=False, device=torch.device("cuda", 0), graph=False)
batch = make_batch(8, 6, res, res, device="cuda:0")
eng.train_step(batch)
torch.cuda.synchronize()
mode = Sites()
with mode:
    eng.train_step(batch)
    torch.cuda.synchronize()
print("per-step copy-like ops by site:")
for (name, site), n in mode.sites.most_common(60):
    print(f"{n:5d}  {name:20s} {site}")
print("\nall aten ops:", sum(mode.ops.values()))
for name, n in mode.ops.most_common(40):
    print(f"{n:5d}  {name}")
