"""RT-1 masked attention on MFMA (``csrc/kernels/attention.hip``) and the fused transformer layer.

Forward is the HIP kernel (Q/K/V from ONE fused projection GEMM, mask computed
in-kernel, softmax + dropout + P@V on-chip, per-row log-sum-exp saved).  The
backward is a HIP kernel too (one workgroup per (batch, head)): it recomputes P
from Q, K and the saved LSE (no S x S tensor is kept from the forward),
regenerates the identical dropout mask from the same counter-based hash and
produces dQ, dK, dV with MFMAs (transposed operands via ds_read_b64_tr_b16).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import rng, switches
from ._ext import load
from ..models.transformer import rt1_attention_mask
from ..parallel.flat import defer_partials

BF = torch.bfloat16
BWD_MAX_S = 96     # single-kernel attn_bwd covers S <= 96 (T <= 8); longer histories (<= 256) use attn_bwd_long
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
        out, lse = load().attn_fwd(qkv, L, Kimg, scale, drop_p, seed, _ctr(qkv))
        ctx.save_for_backward(qkv, out, lse)
        ctx.args = (L, Kimg, drop_p, seed, scale)
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        L, Kimg, drop_p, seed, scale = ctx.args
        B, S, _, H, D = qkv.shape
        return attn_backward(qkv, out, dout.to(qkv.dtype).contiguous(), lse, L, Kimg, scale, drop_p, seed), \
            None, None, None, None

    @staticmethod
    def _backward_torch(qkv, out, lse, dout, L, Kimg, drop_p, seed, scale):
        """fp32 batched-GEMM backward with the kernels' keep-mask: the numerical oracle of the HIP backward."""
        B, S, _, H, D = qkv.shape
        q, k, v = qkv.float().permute(2, 0, 3, 1, 4).unbind(0)               # [B, H, S, D]
        allowed = _allowed(S, L, Kimg, qkv.device)
        s = torch.matmul(q, k.transpose(-1, -2)) * scale
        p = torch.exp(s.masked_fill(~allowed, float("-inf")) - lse[..., None])
        do = dout.float().permute(0, 2, 1, 3)                                  # [B, H, S, D]
        if drop_p > 0:
            keep = load().attn_keepmask(B * H, S, drop_p, seed, qkv, _ctr(qkv)).view(B, H, S, S).float() / (1.0 - drop_p)
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


def attn_backward(qkv, out, dout, lse, L, Kimg, scale, drop_p, seed):
    """dQKV on the HIP kernels: one workgroup per (b, h) with the S x S tiles in LDS for S <= 96 (T <= 8),
    the streamed dK/dV + dQ kernel pair (O(chunk) LDS) for longer histories up to the 256-position table."""
    S = qkv.shape[1]
    ext = load()
    if S <= BWD_MAX_S:
        return ext.attn_bwd(qkv, out, dout, lse, L, Kimg, scale, drop_p, seed, _ctr(qkv))
    return ext.attn_bwd_long(qkv, out, dout, lse, L, Kimg, scale, drop_p, seed, _ctr(qkv))


# The projections stay on the recorded hipBLASLt solutions (tuning/): gemm.hip beat UNtuned hipBLASLt on the fused
# Q/K/V forward, the FF forward and the out / FF data gradients in isolation (profiles/r4_gemm_bench_lds_store.log) but
# not the tuned library in the step (-0.3 %, profiles/r4_tf_gemm_lds_ab.log), and the full-row gemm path with the
# LayerNorm in the epilogue (tfrow.hip) was 2 ms/step slower (profiles/r5_tfrow_ab.log); both were removed.


# (N, K, nn) -> gemm.hip tile config for the projections where its small tiles beat the tuned library in the step
# (tools/bench_tf_gemms.py); the rest stay on hipBLASLt
# (in the step: FF / out data gradients 14.2 / 20.6 us vs the library's 16.2 / 21.2; the forward products stayed on the
# library, 19 vs 17 us on 64 x 64 tiles -- gpurun_out/trN vs trN_film kernel traces)
_TF_GEMM_CFG = {(512, 512, True): 3, (1024, 512, True): 4}
TF_GEMM = _TF_GEMM_CFG if switches.on("tf_gemm") else {}


def _proj(a, w, nn: bool = False):
    """a @ w^T (w [N, K], a Linear weight) or, nn, a @ w (w [K, N]: the data gradient through that weight)."""
    cfg = TF_GEMM.get((w.shape[1], w.shape[0], True) if nn else (w.shape[0], w.shape[1], False))
    if cfg is not None and a.shape[0] >= 1024:
        return load().gemm(a, w, nn, cfg=cfg)[0]
    return torch.mm(a, w) if nn else torch.mm(a, w.t())


_QKV = {}     # data_ptr(q weight) -> (Wqkv [3HD, E], bqkv [3HD]) bf16, packed per step by FusedRT1._refresh_shadow


def set_qkv_packs(packs):
    global _QKV
    _QKV = packs


def _bfw(w):
    from .backbone import _bf
    return _bf(w)


def _mm32(a, b):
    try:
        return torch.mm(a, b, out_dtype=torch.float32)
    except (TypeError, RuntimeError):
        return torch.mm(a, b).float()


# projection weight gradients on the streaming MFMA kernel (csrc/kernels/wgrad.hip, split over the T = B*S token rows,
# fixed-order reduce): hipBLASLt runs dW = dY^T X with K = 8448 and a 512x512 output on 16 macro tiles, ~5 % of its
# roofline (tools/gemm_census.py)
TF_WGRAD = switches.on("tf_wgrad")


def _tf_wgrad_cfg(M: int, Co: int):
    """(tile variant, row splits) of wgrad.hip for the transformer's short reductions (T = B x S tokens, 8448 at
    b128): the automatic choice aims at ~512 workgroups of the widest tile, right for the encoder's millions of rows
    but here every split writes a whole fp32 [Co, Ci] partial.  Swept per shape (tools/bench_wgrad_short.py,
    profiles/r5_wgrad_short.log): 128 x 128 tiles with ~1056-row splits for the 3072-wide QKV gradient (105.6 -> 56.2
    us), 64 x 128 tiles with ~704-row splits for the 512-wide ones (58.4 -> 31.2, 44.0 -> 23.8 us)."""
    if M > 65536:
        return -1, -1
    if Co >= 2048:
        return 2, max(1, min(16, M // 1056))
    return 1, max(1, min(16, M // 704))


def _wgrad_bias(dy, x, ok: bool = True):
    """(dW = dy^T x, db = sum_rows dy) of a parameter pair: the column sums of dy come from the wgrad kernel's staged
    rows and share its split partials' fixed-order sum (one launch instead of a colsum re-reading dy)."""
    Co, Ci = dy.shape[1], x.shape[1]
    if TF_WGRAD and dy.dtype == BF and x.dtype == BF and Co % 8 == 0 and Ci % 8 == 0:
        v, s = _tf_wgrad_cfg(dy.shape[0], Co)
        flat = defer_partials(load().wgrad(dy.contiguous(), x.contiguous(), variant=v, splits=s, partials=True,
                                           sums=True), ok)
        return flat[:Co * Ci].view(Co, Ci), flat[Co * Ci:]
    return _wgrad(dy, x, True, ok), load().colsum(dy)


def _wgrad(dy, x, final: bool = False, ok: bool = True):
    """dW = dy^T x: dy [T, Co], x [T, Ci] bf16 -> fp32 [Co, Ci].  ``final``: a parameter gradient as is (``ok``: every
    row slice of it reaches a parameter that requires one), its split-K sum left to the flat gather."""
    if TF_WGRAD and dy.dtype == BF and x.dtype == BF and dy.shape[1] % 8 == 0 and x.shape[1] % 8 == 0:
        v, s = _tf_wgrad_cfg(dy.shape[0], dy.shape[1])
        out = load().wgrad(dy.contiguous(), x.contiguous(), variant=v, splits=s, partials=final)
        return defer_partials(out, ok) if final else out
    return _mm32(dy.t(), x)


def _seed(p: float) -> int:
    """Per-call-site dropout salt; the per-step randomness is the device counter of ``ops.rng``."""
    return rng.next_salt() if p > 0 else 0


def _ctr(t: torch.Tensor) -> torch.Tensor:
    return rng.counter(t.device)


# the LayerNorm after each residual formed by the residual kernel itself, and the LN2 backward emitting the
# out-projection's bf16 gradient operand (+0.3 % step, 24 launches fewer: profiles/r5_tf_fuse_ln_ab.log; off: the
# standalone ln_fwd / drop_bwd launches)
TF_FUSE_LN = switches.on("tf_fuse_ln")
_EMPTY = {}


def _empty(dev):
    t = _EMPTY.get(dev)
    if t is None:
        t = torch.empty(0, device=dev)
        _EMPTY[dev] = t
    return t


class RT1LayerFn(torch.autograd.Function):
    """One pre-LN RT-1 decoder layer (reference ``transformer.py:112-144``) with an fp32 residual stream:

        x2 = x + Wo . attn(Wqkv . LN1(x)) + bo
        x3 = x2 + dropout(Wff . LN2(x2) + bff)

    The attention, LayerNorms, residual adds and dropout are HIP kernels (``attention.hip``, ``transformer.hip``); the
    projections are bf16 hipBLASLt GEMMs (fp32 accumulate) on the bf16 weight shadow.  Each residual kernel also forms
    the LayerNorm that follows it on the same rows (LN2 after the out-projection; the NEXT layer's LN1 after the FF),
    so no LayerNorm re-reads the residual stream: ``aux`` = (LN1(x), mean, rstd) when the previous layer formed them,
    ``next_ln`` = the next layer's (gamma, beta, eps), returned as three non-differentiable extra outputs (their
    gradient is the next layer's LayerNorm backward, which it runs itself from x3 and the saved statistics).  The LN2
    backward also emits the out-projection's bf16 gradient operand and its bias gradient.  The backward recomputes
    nothing but P inside the attention kernel."""

    @staticmethod
    def forward(ctx, x, g1, b1, wq, bq, wk, bk, wv, bv, wo, bo, g2, b2, wf, bff, aux_xn, aux_mu, aux_rs, meta):
        ext = load()
        L, Kimg, H, D, p_attn, p_ff, eps1, eps2, next_ln = meta
        B, S, E = x.shape
        T = B * S
        x2d = x.reshape(T, E).float().contiguous()
        if aux_xn.numel():
            xn1, mu1, rs1 = aux_xn, aux_mu, aux_rs
        else:
            xn1, mu1, rs1 = ext.tf_ln_fwd(x2d, g1.float(), b1.float(), eps1)
        pk = _QKV.get(wq.data_ptr())
        if pk is not None:
            Wqkv, bqkv = pk                                                     # packed with the weight shadow
        else:
            Wqkv = torch.cat([_bfw(wq), _bfw(wk), _bfw(wv)], 0)                # [3*H*D, E]
            bqkv = torch.cat([bq, bk, bv]).to(BF)
        qkv = torch.addmm(bqkv, xn1, Wqkv.t()).view(B, S, 3, H, D)
        scale = 1.0 / math.sqrt(D)
        seed_a, seed_f = _seed(p_attn), _seed(p_ff)
        ctr = _ctr(x)
        o, lse = ext.attn_fwd(qkv, L, Kimg, scale, p_attn, seed_a, ctr)
        o2d = o.view(T, H * D)
        wo_b, wf_b = _bfw(wo), _bfw(wf)
        empty = _empty(x.device)
        nxt = (empty, empty, empty)
        if TF_FUSE_LN:
            x2, xn2, mu2, rs2 = ext.tf_resid(x2d, _proj(o2d, wo_b), bo.float().contiguous(), 0.0, 0, None,
                                             g2.float(), b2.float(), eps2)
        else:
            (x2,) = ext.tf_resid(x2d, _proj(o2d, wo_b), bo.float().contiguous(), 0.0, 0)
            xn2, mu2, rs2 = ext.tf_ln_fwd(x2, g2.float(), b2.float(), eps2)
        ff = _proj(xn2, wf_b)
        if next_ln is not None and TF_FUSE_LN:
            gn, bn, epsn = next_ln
            x3, *nxt = ext.tf_resid(x2, ff, bff.float().contiguous(), p_ff, seed_f, ctr, gn.float(), bn.float(), epsn)
        else:
            (x3,) = ext.tf_resid(x2, ff, bff.float().contiguous(), p_ff, seed_f, ctr)
            if next_ln is not None:
                gn, bn, epsn = next_ln
                nxt = ext.tf_ln_fwd(x3, gn.float(), bn.float(), epsn)
        ctx.save_for_backward(x2d, xn1, mu1, rs1, qkv, o, lse, x2, xn2, mu2, rs2, Wqkv, wo_b, wf_b, g1, g2)
        ctx.meta = (L, Kimg, H, D, p_attn, p_ff, seed_a, seed_f, scale, B, S, E)
        ctx.mark_non_differentiable(*nxt)
        ctx.set_materialize_grads(False)        # no zero-filled gradients for the three LN outputs
        return (x3.view(B, S, E), *nxt)

    @staticmethod
    def backward(ctx, dx3, *_):
        ext = load()
        (x2d, xn1, mu1, rs1, qkv, o, lse, x2, xn2, mu2, rs2, Wqkv, wo_b, wf_b, g1, g2) = ctx.saved_tensors
        if dx3 is None:
            dx3 = torch.zeros_like(x2)
        L, Kimg, H, D, p_attn, p_ff, seed_a, seed_f, scale, B, S, E = ctx.meta
        T = B * S
        dx3 = dx3.reshape(T, E).float().contiguous()
        # FF branch: dropout, GEMM grads, LN2 (+ the residual grad)
        ctr = _ctr(dx3)
        dh, dbff = ext.tf_drop_bwd(dx3, p_ff, seed_f, ctr)
        nig = ctx.needs_input_grad
        dwf = _wgrad(dh, xn2, True, nig[13])
        o2d = o.view(T, H * D)
        # LN2 backward (+ the residual grad dx3); its bf16 copy of dx2 is the out-projection's gradient operand
        if TF_FUSE_LN:
            dx2, dg2, db2, da, dbo = ext.tf_ln_bwd(_proj(dh, wf_b, True), x2, mu2, rs2, g2.float(), dx3, True)
        else:
            dx2, dg2, db2 = ext.tf_ln_bwd(_proj(dh, wf_b, True), x2, mu2, rs2, g2.float(), dx3)
            da, dbo = ext.tf_drop_bwd(dx2, 0.0, 0)
        # attention branch: out-projection, attention, QKV projection, LN1 (+ residual)
        dwo = _wgrad(da, o2d, True, nig[9])
        do = _proj(da, wo_b, True).view(B, S, H, D)
        dqkv = attn_backward(qkv, o, do, lse, L, Kimg, scale, p_attn, seed_a)
        dq2d = dqkv.view(T, 3 * H * D)
        dWqkv, dbqkv = _wgrad_bias(dq2d, xn1, all(nig[3:9]))
        dx, dg1, db1 = ext.tf_ln_bwd(_proj(dq2d, Wqkv, True), x2d, mu1, rs1, g1.float(), dx2)
        n = H * D
        return (dx.view(B, S, E), dg1, db1, dWqkv[:n], dbqkv[:n], dWqkv[n:2 * n], dbqkv[n:2 * n],
                dWqkv[2 * n:], dbqkv[2 * n:], dwo, dbo, dg2, db2, dwf, dbff, None, None, None, None)


def fused_layer(layer, x: torch.Tensor, L: int, Kimg: int, training: bool, aux=None, next_norm=None):
    """One fused layer: returns (x3, aux for the next layer or None).  ``aux`` = (LN1(x), mean, rstd) from the previous
    layer's epilogue; ``next_norm`` = the next layer's norm_1 (its LayerNorm is formed in this layer's epilogue)."""
    att = layer.attn
    p_attn = att.dropout.p if training else 0.0
    p_ff = layer.dropout_1.p if training else 0.0
    nl = (next_norm.weight, next_norm.bias, next_norm.eps) if next_norm is not None else None
    meta = (L, Kimg, att.h, att.key_dim, p_attn, p_ff, layer.norm_1.eps, layer.norm_2.eps, nl)
    e = _empty(x.device)
    ax = aux if aux is not None else (e, e, e)
    out = RT1LayerFn.apply(x, layer.norm_1.weight, layer.norm_1.bias, att.q_linear.weight, att.q_linear.bias,
                           att.k_linear.weight, att.k_linear.bias, att.v_linear.weight, att.v_linear.bias,
                           att.out.weight, att.out.bias, layer.norm_2.weight, layer.norm_2.bias, layer.ff.weight,
                           layer.ff.bias, ax[0], ax[1], ax[2], meta)
    return out[0], (tuple(out[1:]) if nl is not None else None)


def fused_layer_supported(layer) -> bool:
    att = layer.attn
    return (layer.ff.in_features == 512 and layer.ff.out_features == 512 and att.key_dim == 128
            and att.value_dim == 128 and att.h * att.key_dim == att.q_linear.out_features)


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
    o = RT1AttentionFn.apply(qkv, L, Kimg, p, _seed(p))
    x = x + att.out(o.reshape(B, S, att.h * att.value_dim))
    return x + layer.dropout_1(layer.ff(layer.norm_2(x)))
