#!/usr/bin/env python3
"""Which framework bindings (csrc/bindings*.cpp entry points) one eager hip-backend training step calls, and from
where: binding name x calls, with the innermost package source line of each call site; then the same for the aten
ops that launch device work (a TorchDispatchMode, views and allocations left out).  Most bindings launch one kernel,
the multi-pass ones (colsum with row chunks, finalize pairs) two.

  python tools/ext_census.py [--batch 128] [--res 300] [--top 80]
"""
from __future__ import annotations

import argparse
import collections
import os
import sys
import traceback

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PKG = "pytorch_rt1_for_distributed_training_amd"


def _site() -> str:
    for fr in reversed(traceback.extract_stack()[:-2]):
        if PKG in fr.filename and "ext_census" not in fr.filename:
            return f"{fr.filename.split(PKG + '/')[-1]}:{fr.lineno}"
    return "?"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--res", type=int, default=300)
    ap.add_argument("--top", type=int, default=80)
    a = ap.parse_args()
    from pytorch_rt1_for_distributed_training_amd.config import RT1Config
    from pytorch_rt1_for_distributed_training_amd.data.synthetic import make_batch
    from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine, to_device
    from pytorch_rt1_for_distributed_training_amd.models import build_rt1
    from pytorch_rt1_for_distributed_training_amd.ops._ext import load

    ext = load()
    counts = collections.Counter()
    active = [False]

    def wrap(name, fn):
        def w(*args, **kw):
            if active[0]:
                counts[(name, _site())] += 1
            return fn(*args, **kw)
        return w

    for name in dir(ext):
        fn = getattr(ext, name)
        if callable(fn) and not name.startswith("_") and not name.endswith("_supported"):
            setattr(ext, name, wrap(name, fn))

    dev = torch.device("cuda", 0)
    cfg = RT1Config(height=a.res, width=a.res, seq_len=6, backend="hip")
    eng = TrainEngine(build_rt1(cfg), cfg, order_probe=False, device=dev)
    eng.graph = False
    batch = to_device(make_batch(a.batch, cfg.seq_len, cfg.height, cfg.width), dev)
    eng.train_step(batch)
    torch.cuda.synchronize()
    from torch.utils._python_dispatch import TorchDispatchMode

    aten = collections.Counter()
    quiet = ("empty", "view", "as_strided", "_reshape_alias", "t.", "transpose", "slice", "select", "unsqueeze",
             "squeeze", "permute", "expand", "detach", "alias", "split", "unbind", "lift_fresh",
             "is_same_size", "_unsafe_view", "new_empty", "resize_", "set_", "record_stream", "chunk", "narrow")

    class Census(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            name = str(func.name()).replace("aten::", "")
            if not any(name.startswith(q) or name == q.rstrip(".") for q in quiet):
                site = _site()
                if site == "?":      # from the autograd engine itself: name the shape instead
                    site = "engine " + ",".join(str(list(x.shape)) for x in args if isinstance(x, torch.Tensor))
                    if name.startswith("zeros") or name.startswith("new_zeros"):
                        site += " " + str(args[0] if args and not isinstance(args[0], torch.Tensor) else "")
                aten[(name, site)] += 1
            return func(*args, **(kwargs or {}))

    active[0] = True
    with Census():
        eng.train_step(batch)
    torch.cuda.synchronize()
    active[0] = False
    per_name = collections.Counter()
    for (n, _), c in counts.items():
        per_name[n] += c
    print(f"{sum(counts.values())} binding calls in one step, {len(per_name)} distinct bindings")
    for n, c in per_name.most_common():
        print(f"{c:5d}  {n}")
    print("-- by call site")
    for (n, site), c in counts.most_common(a.top):
        print(f"{c:5d}  {n:28s} {site}")
    print(f"-- aten ops: {sum(aten.values())} calls")
    for (n, site), c in aten.most_common(a.top):
        print(f"{c:5d}  {n:28s} {site}")


if __name__ == "__main__":
    main()
