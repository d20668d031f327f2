#!/usr/bin/env python3
"""Bisect hipGraph capture of the RT-1 train step: capture growing prefixes of the step, print tracebacks."""
import os
import sys
import traceback

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pytorch_rt1_for_distributed_training_amd.config import RT1Config  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.data.synthetic import make_batch  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine, split_batch  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.models import build_rt1  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "global"
cfg = RT1Config(height=96, width=96, seq_len=2, num_layers=2, backend="hip", crop_ratio=0.0)
torch.manual_seed(0)
eng = TrainEngine(build_rt1(cfg), cfg, order_probe=False)
batch = make_batch(4, cfg.seq_len, cfg.height, cfg.width, device="cuda")
eng.train_step(batch)
torch.cuda.synchronize()
m = eng.model
images, ctx, actions = split_batch(batch)


def enc():
    m.train()
    return m.tokenize_images(images, ctx, None)


def tf():
    tok = torch.randn(4, 2, 8, 512, device="cuda", dtype=torch.bfloat16)
    m.train()
    return m.transformer_hidden(m.assemble_tokens(tok))


def fwd():
    return eng.forward_loss(batch)[0]


def fwd_bwd():
    eng.optimizer.zero_grad()
    loss = eng.forward_loss(batch)[0]
    loss.backward()
    return loss


def enc_bwd():
    t = enc()
    t.float().sum().backward()


def tf_bwd():
    tok = torch.randn(4, 2, 8, 512, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    m.train()
    h = m.transformer_hidden(m.assemble_tokens(tok))
    h.float().sum().backward()


eng.optimizer.sync_device_state()


def opt():
    eng.flat.gather_grads()
    eng.optimizer.step()


for name, fn in [("encoder fwd", enc), ("transformer fwd", tf), ("full fwd", fwd), ("encoder fwd+bwd", enc_bwd),
                 ("transformer fwd+bwd", tf_bwd), ("fwd+bwd", fwd_bwd), ("optimizer", opt)]:
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g, capture_error_mode=mode):
            fn()
        g.replay()
        torch.cuda.synchronize()
        print(f"[probe] {name}: capture+replay OK", flush=True)
    except Exception:
        print(f"[probe] {name}: FAILED", flush=True)
        traceback.print_exc()
        torch.cuda.synchronize()
