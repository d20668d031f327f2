"""Fused action head: gather -> logits -> CE -> argmax in ONE HIP kernel (``csrc/kernels/head.hip``).

Reference: the logits head runs over all ``T*L`` positions (``transformer.py:197``), the ``T*A`` rows that
predict action tokens are gathered, scored with ``cross_entropy(reduction='none')`` and argmax-decoded
(``transformer_network.py:304-322,310-312``).  Forward here is one kernel per 16 scored rows (MFMA GEMM,
log-softmax, CE, argmax, and the softmax-minus-onehot gradient all on chip); the backward scales that
gradient by ``dce`` (one small kernel), runs dh on hipBLASLt and dW on the MFMA wgrad kernel.
"""
from __future__ import annotations

import torch

from ._ext import load
from .attention import _wgrad

BF = torch.bfloat16


class HeadCEFn(torch.autograd.Function):
    """(hidden [B,S,E] fp32, W [V,E], bias [V], positions int32 [P], targets int32 [B*P]) -> (ce [B*P], pred)."""

    @staticmethod
    def forward(ctx, hidden, W, bias, positions, targets):
        from .backbone import _bf
        ext = load()
        h = hidden.float().contiguous()
        Wb = _bf(W).contiguous()
        ce, pred, G, hb = ext.head_ce_fwd(h, positions, Wb, bias.float().contiguous(), targets)
        ctx.save_for_backward(G, hb, Wb, positions)
        ctx.shape = h.shape
        ctx.mark_non_differentiable(pred)
        ctx.set_materialize_grads(False)        # no zero-filled gradient for pred
        return ce, pred

    @staticmethod
    def backward(ctx, dce, _dpred):
        G, hb, Wb, positions = ctx.saved_tensors
        B, S, E = ctx.shape
        dz = load().head_ce_scale(G, dce.float().contiguous())             # [R, V] bf16
        dh = torch.mm(dz, Wb)                                               # [R, E]
        dW = _wgrad(dz, hb, True, ctx.needs_input_grad[1])                                                 # [V, E] fp32, MFMA wgrad kernel
        db = load().colsum(dz)
        dhidden = torch.zeros(B, S, E, device=G.device, dtype=torch.float32)
        dhidden[:, positions.long()] = dh.view(B, -1, E).float()           # positions are unique
        return dhidden, dW, db, None, None


def head_supported(linear: torch.nn.Linear) -> bool:
    return load().head_ce_supported(linear.out_features, linear.in_features)


def head_ce(linear: torch.nn.Linear, hidden: torch.Tensor, positions: torch.Tensor, targets: torch.Tensor,
            targets32: torch.Tensor = None):
    """Per-row CE and argmax of ``linear(hidden[:, positions])`` against ``targets`` (b, T*A); ``targets32`` is the
    int32 copy the fused tokenizer already wrote (no conversion launch)."""
    pos = positions if positions.dtype == torch.int32 else positions.to(torch.int32)
    tgt = (targets32 if targets32 is not None else targets).reshape(-1).to(torch.int32).contiguous()
    return HeadCEFn.apply(hidden, linear.weight, linear.bias, pos.contiguous(), tgt)
