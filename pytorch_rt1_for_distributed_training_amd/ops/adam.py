"""Fused flat Adam/AdamW (``csrc/kernels/adam.hip``)."""
from __future__ import annotations

import math

import torch

from ._ext import load


def flat_adam_step(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, *, lr: float, beta1: float,
                   beta2: float, eps: float, weight_decay: float, step: int, grad_scale: float = 1.0):
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    load().flat_adam(p, g, m, v, lr, beta1, beta2, eps, weight_decay, lr / bc1, 1.0 / math.sqrt(bc2), grad_scale)


def flat_adam_dev_step(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, state: torch.Tensor, *,
                       beta1: float, beta2: float, eps: float, weight_decay: float, grad_scale: float = 1.0):
    """Same update with {step, lr} read from the device tensor ``state`` (hipGraph-replayable)."""
    load().flat_adam_dev(p, g, m, v, state, beta1, beta2, eps, weight_decay, grad_scale)


def reference_adam_step(p, g, m, v, *, lr, beta1, beta2, eps, weight_decay, step, grad_scale=1.0):
    """Plain PyTorch fp32 oracle (same math as torch.optim.Adam / AdamW)."""
    g = g * grad_scale
    if weight_decay:
        p.mul_(1 - lr * weight_decay)
    m.mul_(beta1).add_(g, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    denom = (v.sqrt() / math.sqrt(1 - beta2 ** step)).add_(eps)
    p.addcdiv_(m, denom, value=-lr / (1 - beta1 ** step))
