#!/usr/bin/env python3
"""Time the phases of one RT-1 training step on the fused HIP backend (HIP events, median).

  encoder   : image tokenizer fwd + bwd (stem, 26 MBConv, top, conv1x1, FiLM, TokenLearner)
  tf+head   : token assembly, 8 transformer layers, logits head, CE loss, fwd + bwd
  optimizer : fused Adam over the flat buffer
  step      : the whole engine.train_step

  python tools/bench_phases.py --batch 128
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pytorch_rt1_for_distributed_training_amd as rt1  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.data.synthetic import make_batch  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.models import build_rt1  # noqa: E402


def timed(fn, iters):
    ts = []
    for _ in range(iters + 2):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts = sorted(ts[2:])
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--res", type=int, default=300)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--only", default="", help="run just one phase (e.g. tf+head) for profiling")
    a = ap.parse_args()
    cfg = rt1.RT1Config(height=a.res, width=a.res, backend="hip")
    model = build_rt1(cfg)
    eng = TrainEngine(model, cfg, order_probe=False)
    m = eng.model
    batch = make_batch(a.batch, cfg.seq_len, a.res, a.res, device="cuda")
    obs, acts = batch["train_observation"], batch["action_label"]
    imgs, ctx = obs["image"], obs["natural_language_embedding"]
    b, t = imgs.shape[:2]

    def step():
        eng.train_step(batch)

    def encoder():
        tok = m.tokenize_images(imgs, ctx, None)
        tok.float().sum().backward()

    m.train()
    tok = m.tokenize_images(imgs, ctx, None).detach()

    def tf_head():
        x = tok.clone().requires_grad_(True)
        targets = m._action_tokenizer.tokenize(acts)
        hidden = m.transformer_hidden(m.assemble_tokens(x))
        logits = m.action_logits(hidden, m._predicted_positions)
        loss = m.action_loss(logits, targets, b, t)
        loss.mean().backward()

    def optim():
        eng.optimizer.step()

    phases = {"step": step, "encoder": encoder, "tf+head": tf_head, "optimizer": optim}
    if a.only:
        phases = {a.only: phases[a.only]}
    res = {k: timed(f, a.iters) for k, f in phases.items()}
    print({k: round(v, 2) for k, v in res.items()}, "ms")


if __name__ == "__main__":
    main()
