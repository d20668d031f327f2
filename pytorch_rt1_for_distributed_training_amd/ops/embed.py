"""Transformer token embedding on the ``hip`` backend (reference transformer.py:181-189).

``x = tokens @ W^T + b + pos[:S]`` as ONE MFMA kernel with a bias + position-row epilogue that writes the fp32
residual stream directly (``csrc/kernels/pwtall.hip``, ``rt1_embed_fwd``), replacing a bf16 GEMM, a position add
and an fp32 up-cast.  Backward: dX through the transformer's data-gradient route (attention._proj), dW on the MFMA
wgrad kernel (bf16 operands, fp32 dW), db / dpos as row reductions.
"""
from __future__ import annotations

import torch

from ._ext import load as _ext
from .attention import _proj, _wgrad

BF = torch.bfloat16


class EmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tokens, w, b, pos):
        from .backbone import _bf
        B, S, K = tokens.shape
        x = tokens.to(BF).contiguous()
        wb = _bf(w).contiguous()
        out = _ext().embed_fwd(x, wb, b.float().contiguous(), pos.float().contiguous())
        ctx.save_for_backward(x, wb)
        ctx.meta = (B, S, K, pos.shape[0], tokens.dtype)
        return out

    @staticmethod
    def backward(ctx, g):
        x, wb = ctx.saved_tensors
        B, S, K, P, tdt = ctx.meta
        N = wb.shape[0]
        g2 = g.reshape(B * S, N)
        gb = g2.to(BF)
        dx = _proj(gb, wb, True).view(B, S, K).to(tdt) if ctx.needs_input_grad[0] else None
        # dW on the streaming MFMA wgrad kernel with the transformer's short-reduction split (hipBLASLt ran this
        # [512, 8448] x [8448, 512] TN product at 64 us, ~5 % of its roofline: tools/gemm_census.py)
        dw = _wgrad(gb, x.view(B * S, K), True) if ctx.needs_input_grad[1] else None
        db = _ext().colsum(g2) if ctx.needs_input_grad[2] else None
        dpos = None
        if ctx.needs_input_grad[3]:
            dpos = torch.zeros(P, N, device=g.device, dtype=torch.float32)
            dpos[:S] = _ext().colsum(g.contiguous())
        return dx, dw, db, dpos


def supported(tf, tokens: torch.Tensor) -> bool:
    K = tokens.shape[-1]
    N = tf._token_emb.weight.shape[0]
    return tokens.is_cuda and K % 8 == 0 and N % 16 == 0 and tokens.shape[1] <= tf.max_seq_len


def embed(tf, tokens: torch.Tensor) -> torch.Tensor:
    """fp32 [B, S, N] residual stream input."""
    return EmbedFn.apply(tokens, tf._token_emb.weight, tf._token_emb.bias, tf._position_emb.weight)
