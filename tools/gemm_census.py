#!/usr/bin/env python3
"""Census of the library GEMMs (torch.mm / bmm / addmm / linear -> hipBLASLt) one RT-1 training step still issues on
the hip backend, with each distinct shape re-timed in isolation against its HBM / MFMA roofline.

  python tools/gemm_census.py [--batch 128] [--res 300] [--seq_len 6]

Prints one row per (op, shapes, dtypes): calls per step, median us per call, roofline us, and where in the model it
was called from (the innermost frame inside the package).
"""
from __future__ import annotations

import argparse
import collections
import os
import sys
import traceback

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HBM = 5.5e12
MFMA = 2.3e15

CALLS = collections.OrderedDict()


def _site():
    for fr in reversed(traceback.extract_stack()[:-2]):
        if "pytorch_rt1_for_distributed_training_amd" in fr.filename and "gemm_census" not in fr.filename:
            return f"{os.path.basename(fr.filename)}:{fr.lineno}"
    return "?"


def _wrap(name, fn):
    def inner(*args, **kw):
        ts = tuple((tuple(a.shape), str(a.dtype).replace("torch.", ""), a.is_contiguous())
                   for a in args if isinstance(a, torch.Tensor))
        key = (name, ts, tuple(sorted((k, str(v)) for k, v in kw.items() if not isinstance(v, torch.Tensor))))
        ent = CALLS.setdefault(key, {"n": 0, "site": _site(), "args": None})
        ent["n"] += 1
        if ent["args"] is None:
            ent["args"] = ([a.detach().clone() if isinstance(a, torch.Tensor) else a for a in args], dict(kw))
        return fn(*args, **kw)
    return inner


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--res", type=int, default=300)
    ap.add_argument("--seq_len", type=int, default=6)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from pytorch_rt1_for_distributed_training_amd.config import RT1Config
    from pytorch_rt1_for_distributed_training_amd.data.synthetic import make_batch
    from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine, to_device
    from pytorch_rt1_for_distributed_training_amd.models import build_rt1

    dev = torch.device("cuda", 0)
    cfg = RT1Config(height=a.res, width=a.res, seq_len=a.seq_len, backend="hip")
    model = build_rt1(cfg)
    eng = TrainEngine(model, cfg, order_probe=False, device=dev)
    batch = to_device(make_batch(a.batch, cfg.seq_len, cfg.height, cfg.width), dev)
    eng.train_step(batch)                                     # warm-up (lazy init) outside the census
    torch.cuda.synchronize()
    orig = {"mm": torch.mm, "bmm": torch.bmm, "addmm": torch.addmm, "linear": F.linear, "matmul": torch.matmul}
    torch.mm = _wrap("mm", orig["mm"])
    torch.bmm = _wrap("bmm", orig["bmm"])
    torch.addmm = _wrap("addmm", orig["addmm"])
    F.linear = _wrap("linear", orig["linear"])
    torch.matmul = _wrap("matmul", orig["matmul"])
    eng.train_step(batch)
    torch.cuda.synchronize()
    torch.mm, torch.bmm, torch.addmm, F.linear, torch.matmul = (orig["mm"], orig["bmm"], orig["addmm"],
                                                                 orig["linear"], orig["matmul"])
    # Tensor.__matmul__ (the @ operator) bypasses the wrappers: count it through the dispatcher-level profiler
    print(f"{'op':7s} {'shapes':58s} {'calls':>5s} {'us':>8s} {'roof us':>8s} {'%':>4s}  site")
    tot = tot_roof = 0.0
    for (name, ts, kw), ent in CALLS.items():
        args, kwargs = ent["args"]
        fn = orig[name]
        for _ in range(3):
            fn(*args, **kwargs)
        times = []
        for _ in range(a.iters):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            out = fn(*args, **kwargs)
            e1.record()
            e1.synchronize()
            times.append(e0.elapsed_time(e1) * 1e3)
        times.sort()
        us = times[len(times) // 2]
        tens = [x for x in args if isinstance(x, torch.Tensor)]
        byts = sum(x.numel() * x.element_size() for x in tens) + out.numel() * out.element_size()
        if name in ("mm", "addmm", "linear", "matmul"):
            A, B = tens[-2], tens[-1]
            m = A.numel() // A.shape[-1]
            kk = A.shape[-1]
            n = out.shape[-1]
            fl = 2.0 * m * kk * n
        else:
            A, B = tens[0], tens[1]
            fl = 2.0 * A.shape[0] * A.shape[1] * A.shape[2] * B.shape[2]
        roof = max(byts / HBM, fl / MFMA) * 1e6
        tot += us * ent["n"]
        tot_roof += roof * ent["n"]
        shp = " x ".join(f"{list(s)}{'' if c else 'T'}:{d[:4]}" for s, d, c in ts)
        print(f"{name:7s} {shp[:58]:58s} {ent['n']:5d} {us:8.1f} {roof:8.1f} {100 * roof / us:4.0f}  {ent['site']}")
    print(f"total: {tot / 1e3:.2f} ms/step of wrapped library GEMMs, roofline {tot_roof / 1e3:.2f} ms")


if __name__ == "__main__":
    main()
