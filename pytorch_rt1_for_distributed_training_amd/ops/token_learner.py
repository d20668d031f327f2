"""TokenLearner on two HIP kernels (``csrc/kernels/tokenlearner.hip``), one workgroup per frame.

Reference: ``tokenizers/token_learner.py:64-95`` (LayerNorm -> 1x1 conv 512->64 -> GELU(tanh) -> 1x1 conv
64->8 -> softmax over positions -> weighted sum of the un-normalised features).  The forward kernel keeps
everything of a frame on chip; the backward kernel produces dx, the LayerNorm / conv2 parameter gradients
as per-frame partials (summed here in a fixed order) and dz1 / xn for the one large weight gradient,
dW1 = dz1^T xn, which runs as a split-K hipBLASLt GEMM.
"""
from __future__ import annotations

import torch

from ._ext import load

BF = torch.bfloat16


class TokenLearnerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, feats, ln_w, ln_b, w1, b1, w2, b2, eps: float):
        from .backbone import _bf
        ext = load()
        x = feats.to(BF).contiguous()
        W1 = _bf(w1).reshape(64, 512).contiguous()
        W2 = w2.float().reshape(8, 64).contiguous()
        out, mu, rs, z1, s = ext.tl_fwd(x, ln_w.float().contiguous(), ln_b.float().contiguous(), eps, W1,
                                        b1.float().contiguous(), W2, b2.float().contiguous())
        ctx.save_for_backward(x, mu, rs, z1, s, ln_w, ln_b, W1, W2)
        ctx.shapes = (w1.shape, w2.shape)
        return out

    @staticmethod
    def backward(ctx, dout):
        from .backbone import wgrad
        x, mu, rs, z1, s, ln_w, ln_b, W1, W2 = ctx.saved_tensors
        w1_shape, w2_shape = ctx.shapes
        dx, dz1, xn, pw2, pg = load().tl_bwd(x, dout.to(BF).contiguous(), s, z1, mu, rs, ln_w.float().contiguous(),
                                             ln_b.float().contiguous(), W1.t().contiguous(), W2)
        dW1 = wgrad(dz1, xn, final=True, ok=ctx.needs_input_grad[3]).view(w1_shape)
        db1 = load().colsum(dz1)
        w2p = load().colsum(pw2)                                                   # [8, 65]
        dW2 = w2p[:, :64].contiguous().view(w2_shape)
        db2 = w2p[:, 64].contiguous()
        g = load().colsum(pg)                                                      # [2, 512]
        return dx, g[0], g[1], dW1, db1, dW2, db2, None


def supported(tl, positions: int) -> bool:
    return (tl.dropout_rate == 0 and tl.num_tokens == 8 and tl.conv1.out_channels == 64
            and tl.conv1.in_channels == 512 and load().tl_supported(positions, 512, 64, 8))


def token_learner(tl, feats: torch.Tensor) -> torch.Tensor:
    """feats [N, P, 512] (bf16) -> tokens [N, 8, 512] bf16."""
    return TokenLearnerFn.apply(feats, tl.layerNorm.weight, tl.layerNorm.bias, tl.conv1.weight, tl.conv1.bias,
                                tl.conv2.weight, tl.conv2.bias, tl.layerNorm.eps)
