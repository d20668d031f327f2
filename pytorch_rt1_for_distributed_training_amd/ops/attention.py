"""RT-1 masked attention on MFMA (``csrc/kernels/attention.hip``) and the fused transformer layer.

Forward is the HIP kernel (Q/K/V from ONE fused projection GEMM, mask computed
in-kernel, softmax + dropout + P@V on-chip, per-row log-sum-exp saved).  The
backward recomputes P from Q, K and the saved LSE (no S x S tensor is kept
from the forward) and regenerates the identical dropout mask from the same
counter-based hash; its small batched GEMMs (S = 66) run on hipBLASLt.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from ._ext import load
from ..models.transformer import rt1_attention_mask

BF = torch.bfloat16
_MASKS = {}


def _allowed(S, L, Kimg, device):
    key = (S, L, Kimg, str(device))
    m = _MASKS.get(key)
    if m is None:
        steps = (S + L - 1) // L
        m = rt1_attention_mask(steps, Kimg, L - Kimg)[:S, :S].to(device=device, dtype=torch.bool)
        _MASKS[key] = m
    return m


class RT1AttentionFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, L: int, Kimg: int, drop_p: float, seed: int):
        qkv = qkv.contiguous()
        D = qkv.shape[-1]
        scale = 1.0 / math.sqrt(D)
        out, lse = load().attn_fwd(qkv, L, Kimg, scale, drop_p, seed)
        ctx.save_for_backward(qkv, out, lse)
        ctx.args = (L, Kimg, drop_p, seed, scale)
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        L, Kimg, drop_p, seed, scale = ctx.args
        B, S, _, H, D = qkv.shape
        q, k, v = qkv.float().permute(2, 0, 3, 1, 4).unbind(0)               # [B, H, S, D]
        allowed = _allowed(S, L, Kimg, qkv.device)
        s = torch.matmul(q, k.transpose(-1, -2)) * scale
        p = torch.exp(s.masked_fill(~allowed, float("-inf")) - lse[..., None])
        do = dout.float().permute(0, 2, 1, 3)                                  # [B, H, S, D]
        if drop_p > 0:
            keep = load().attn_keepmask(B * H, S, drop_p, seed, qkv).view(B, H, S, S).float() / (1.0 - drop_p)
            pd = p * keep
        else:
            keep = None
            pd = p
        dv = torch.matmul(pd.transpose(-1, -2), do)
        dpd = torch.matmul(do, v.transpose(-1, -2))
        dp = dpd * keep if keep is not None else dpd
        delta = (do * out.float().permute(0, 2, 1, 3)).sum(-1, keepdim=True)
        ds = p * (dp - delta)
        dq = torch.matmul(ds, k) * scale
        dk = torch.matmul(ds.transpose(-1, -2), q) * scale
        dqkv = torch.stack([dq, dk, dv], dim=0).permute(1, 3, 0, 2, 4).to(qkv.dtype).contiguous()
        return dqkv, None, None, None, None


def fused_qkv_weights(attn):
    w = torch.cat([attn.q_linear.weight, attn.k_linear.weight, attn.v_linear.weight], 0)
    b = torch.cat([attn.q_linear.bias, attn.k_linear.bias, attn.v_linear.bias], 0)
    return w, b


def transformer_layer(layer, x: torch.Tensor, L: int, Kimg: int, training: bool) -> torch.Tensor:
    """One RT-1 layer (``_TransformerLayer``) with the fused QKV GEMM and the HIP attention."""
    B, S, E = x.shape
    att = layer.attn
    x1 = layer.norm_1(x)
    w, b = fused_qkv_weights(att)
    qkv = F.linear(x1, w, b).view(B, S, 3, att.h, att.key_dim)
    p = att.dropout.p if training else 0.0
    seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) if p > 0 else 0
    o = RT1AttentionFn.apply(qkv, L, Kimg, p, seed)
    x = x + att.out(o.reshape(B, S, att.h * att.value_dim))
    return x + layer.dropout_1(layer.ff(layer.norm_2(x)))
