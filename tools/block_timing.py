#!/usr/bin/env python3
"""Per-MBConv-block forward / backward time of one eager hip-backend training step, with the bytes each block
must move and the achieved rate -- the table that says which blocks are far from the HBM roofline.

  RT1_BLOCK_TIMING=1 python tools/block_timing.py --batch 128 [--res 300]

Bytes per block ("compulsory", bf16 activations): forward reads x and writes y1, y2, y3/out and re-reads y2 for
the SE pool and the gate apply; backward reads/writes the same set roughly twice.  They are lower bounds for the
current dataflow, not for a fused one.
"""
from __future__ import annotations

import argparse
import os
import sys

os.environ.setdefault("RT1_BLOCK_TIMING", "1")
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_rt1_for_distributed_training_amd.config import RT1Config  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.data.synthetic import make_batch  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.models import build_rt1  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.models.efficientnet import block_specs, conv_out_size  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.ops import backbone  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--res", type=int, default=300)
    ap.add_argument("--seq", type=int, default=6)
    a = ap.parse_args()
    cfg = RT1Config(height=a.res, width=a.res, seq_len=a.seq, backend="hip")
    torch.manual_seed(0)
    eng = TrainEngine(build_rt1(cfg), cfg, order_probe=False, graph=False)
    batch = make_batch(a.batch, cfg.seq_len, cfg.height, cfg.width, device="cuda")
    for _ in range(2):
        eng.train_step(batch)
    torch.cuda.synchronize()
    backbone.TIMING_EVENTS.clear()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    eng.train_step(batch)
    e.record()
    torch.cuda.synchronize()
    step_ms = s.elapsed_time(e)
    ev = {n: x for n, x in backbone.TIMING_EVENTS}
    N = a.batch * a.seq
    H = W = conv_out_size(a.res, 3, 2)
    print(f"step {step_ms:.2f} ms (eager)  frames {N}")
    print(f"{'blk':>3} {'Cin':>5} {'Ce':>5} {'Cout':>5} {'k':>2} {'s':>2} {'HxW':>9} | {'fwd ms':>7} {'bwd ms':>7} |"
          f" {'act GB':>7} {'fwd TB/s':>8} {'bwd TB/s':>8}")
    tf = tb = 0.0
    for sp in block_specs():
        Ho, Wo = conv_out_size(H, sp.kernel, sp.stride), conv_out_size(W, sp.kernel, sp.stride)
        f = ev[f"fwd{sp.index}"].elapsed_time(ev[f"fwd{sp.index}_end"])
        b = ev[f"bwd{sp.index}"].elapsed_time(ev[f"bwd{sp.index}_end"])
        tf += f
        tb += b
        x = N * H * W * sp.in_ch * 2
        y1 = N * H * W * sp.expand_ch * 2 if sp.expand_ch != sp.in_ch else 0
        y2 = N * Ho * Wo * sp.expand_ch * 2
        y3 = N * Ho * Wo * sp.out_ch * 2
        fwd_bytes = x + 2 * y1 + 4 * y2 + y2 + 3 * y3 + (y3 if sp.has_skip else 0)
        bwd_bytes = 2 * (fwd_bytes + y2)
        print(f"{sp.index:>3} {sp.in_ch:>5} {sp.expand_ch:>5} {sp.out_ch:>5} {sp.kernel:>2} {sp.stride:>2} "
              f"{H:>4}x{W:<4} | {f:7.3f} {b:7.3f} | {fwd_bytes / 1e9:7.2f} {fwd_bytes / f / 1e9:8.2f} "
              f"{bwd_bytes / b / 1e9:8.2f}")
        H, W = Ho, Wo
    print(f"blocks total: fwd {tf:.2f} ms, bwd {tb:.2f} ms, rest of step {step_ms - tf - tb:.2f} ms")


if __name__ == "__main__":
    main()
