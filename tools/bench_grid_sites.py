#!/usr/bin/env python3
"""Grid-cap sweep per call site: every call of the bindings below in one eager hip-backend training step (the
depthwise forward / backward kernels, the stem, the skinny pointwise GEMM) re-timed in isolation with its
``max_blocks`` argument at each value of --caps, next to the value the step used (median us).  One site at a time:
a step runs with a spy that clones that site's arguments only, so memory stays at one step plus one call.

  python tools/bench_grid_sites.py [--batch 128] [--only dw_fwd,pw_bwd_z] [--caps 512,1024,2048,3072,4096]
"""
from __future__ import annotations

import argparse
import os
import sys
import traceback

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_dw_phases import timeit  # noqa: E402

PKG = "pytorch_rt1_for_distributed_training_amd"
# binding -> positional index of its max_blocks argument
GRID_ARG = {"dw_fwd": 7, "dw_fwd_x": 7, "dw_bwd_fused": 19, "dw_bwd_fused_x": 19, "pw_gemm": 2, "pw_gemm_bnbwd": 11,
            "stem_fwd": 3, "stem_bwd_weight": 3, "pw_bwd_z": 7}
# binding -> (keyword, values) of a tile-config argument swept the same way (--only gemm,gemm_tail,gemm256)
KW_ARG = {"gemm": ("cfg", [0, 1, 2]), "gemm_tail": ("cfg", [0, 1, 2]), "gemm256": ("bn", [128, 256])}


def _site() -> str:
    for fr in reversed(traceback.extract_stack()[:-2]):
        if PKG in fr.filename and "bench_grid_sites" not in fr.filename:
            return f"{fr.filename.split(PKG + '/')[-1]}:{fr.lineno}"
    return "?"


def _clone(v):
    return v.clone() if isinstance(v, torch.Tensor) else v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="")
    ap.add_argument("--caps", default="256,512,1024,1536,2048,3072,4096")
    a = ap.parse_args()
    caps = [int(c) for c in a.caps.split(",")]
    from pytorch_rt1_for_distributed_training_amd.config import RT1Config
    from pytorch_rt1_for_distributed_training_amd.data.synthetic import make_batch
    from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine, to_device
    from pytorch_rt1_for_distributed_training_amd.models import build_rt1
    from pytorch_rt1_for_distributed_training_amd.ops._ext import load

    ext = load()
    only = [o for o in a.only.split(",") if o]
    real = {n: getattr(ext, n) for n in list(GRID_ARG) + list(KW_ARG) if (not only and n in GRID_ARG) or n in only}
    state = {"mode": "off", "order": [], "want": None, "got": None}

    def make_spy(name):
        fn = real[name]

        def spy(*args, **kw):
            if state["mode"] != "off":
                key = (name, _site(), tuple(tuple(x.shape) for x in args if isinstance(x, torch.Tensor)))
                if state["mode"] == "list" and key not in state["order"]:
                    state["order"].append(key)
                elif state["mode"] == "grab" and key == state["want"] and state["got"] is None:
                    state["got"] = ([_clone(x) for x in args], {k: _clone(v) for k, v in kw.items()})
            return fn(*args, **kw)
        return spy

    for n in real:
        setattr(ext, n, make_spy(n))
    dev = torch.device("cuda", 0)
    cfg = RT1Config(height=300, width=300, seq_len=6, backend="hip")
    eng = TrainEngine(build_rt1(cfg), cfg, order_probe=False, device=dev)
    eng.graph = False
    batch = to_device(make_batch(a.batch, cfg.seq_len, cfg.height, cfg.width), dev)
    eng.train_step(batch)
    state["mode"] = "list"
    eng.train_step(batch)
    print(f"{len(state['order'])} call sites", flush=True)
    for key in state["order"]:
        name, site, shapes = key
        state.update(mode="grab", want=key, got=None)
        eng.train_step(batch)
        state["mode"] = "off"
        torch.cuda.synchronize()
        args, kw = state["got"]
        fn = real[name]
        t_used = timeit(lambda: fn(*args, **kw), a.iters)
        res = []
        if name in KW_ARG:
            kwn, values = KW_ARG[name]
            used = kw.get(kwn, "default")
            for c in values:
                kw2 = dict(kw)
                kw2[kwn] = c
                res.append((timeit(lambda: fn(*args, **kw2), a.iters), c))
        else:
            gi = GRID_ARG[name]
            used = args[gi]
            for c in caps:
                args2 = list(args)
                args2[gi] = c
                res.append((timeit(lambda: fn(*args2, **kw), a.iters), c))
        best_t, best_c = min(res)
        row = " ".join(f"{c}:{t:.1f}" for t, c in res)
        print(f"{name:16s} {str(shapes[0]):24s} used {used}:{t_used:8.1f} best {best_c}:{best_t:8.1f} "
              f"({100 * (t_used - best_t) / t_used:4.1f} %) | {row} | {site}", flush=True)
        del args, kw
        state["got"] = None
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
