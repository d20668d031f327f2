"""Fused HIP implementation of the FiLM-EfficientNet-B3 image encoder (reference:
``film_efficientnet/film_efficientnet_encoder.py:142-224``; ``models.efficientnet.MBConvBlock`` is the eager oracle).

Activations are channels-last bf16 ``[N, H, W, C]`` (N = b*t frames) end to end; BatchNorm statistics, running stats
and every reduction are fp32/fp64 with a fixed summation order.  Per MBConv block, as it runs today:

forward   y1 = x @ We^T + BN1 partials   expand 1x1: pwgemm.hip MFMA kernels with a BN-stat epilogue where they cover
                                         the shape, else hipBLASLt + bn_stats (deep blocks); x-mode (block 2): y1 is
                                         never formed -- BN1 stats come from x's Gram moments (xexpand.hip)
          y2 = dwconv(silu(bn1(y1)))    dw_fwd_kernel (dwconv.hip): BN1+SiLU prologue while staging the tile (x-mode:
                                         y1 recomputed per tile on MFMA from x), BN2 partials epilogue
          s  = SE(mean_hw silu(bn2(y2))) frame_pool + fp32 fc1 / SiLU / fc2 / sigmoid
          y3 = (silu(bn2(y2)) * s) @ Wp^T project 1x1 with the operand built in the GEMM's registers and a BN3-stat
                                         epilogue: pwgemm.hip pw_gemm / pw_tall (blocks 0-17), gemm.hip (blocks 18-23); the two widest
                                         project convs materialise A (bn_apply) for hipBLASLt
          out = (bn3(y3)*keep + x) * (1+gamma_film) + beta_film      block_tail
backward  tail_bwd_reduce (FiLM grads + BN3 partials) -> bn_bwd_apply -> dA = dy3 @ Wp
          proj_bwd (projbwd.hip): SE / BN2 backward sums and dWp from (dy3, y2) without A (fused-project blocks);
          otherwise bn_apply(A) + wgrad + se_bn_bwd_reduce
          SE backward (se_bwd_dz / se_bwd_dh / se_bwd_bnsum around the small fp32 GEMMs)
          dw_bwd_uni / dw_bwd_uni_s2 (dwconv.hip): ONE pass per tile -- dy2 rebuilt from (dA, y2, gate, rb) while
          staging (BN2-backward apply), depthwise data AND weight gradients, BN1-backward partials; expand blocks store
          dz = dx * silu'(z) directly
          pw_bwd_z (pwbwd.hip): dx = dz' @ We and dWe with the BN1 backward folded in through G = x^T x (y1-free)

Saved per block: x, y2, y3 (bf16), y1 only outside x-mode, A only for the hipBLASLt project convs, the SE vectors
(pool, h, gate) and per-channel constants.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.nn.functional as F

from . import switches
from ._ext import load
from ..parallel.flat import defer_partials

ACT_NONE, ACT_SILU = 0, 1
MAX_BLOCKS = 2048   # ~8 workgroups per CU on 256 CUs: upper bound for persistent tile loops / partial rows
BF = torch.bfloat16


def _ext():
    return load()


def _mm(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """bf16 x bf16 -> bf16 GEMM on hipBLASLt (fp32 accumulate)."""
    return torch.mm(a, b)


PW_BLOCKS = 2048


def _pw_blocks(M: int) -> int:
    """Grid cap of the skinny pointwise GEMM (pwgemm.hip): 512 on the 38x38 maps (M ~ 1.1 M rows: 135-143 vs 145-157
    us for the expand / project convs, 270 vs 286 us for the BN3-backward dgrad, per-site sweep
    tools/bench_grid_sites.py, profiles/r5_grid_sites.log), PW_BLOCKS elsewhere (flat or worse below 2048)."""
    return 512 if 500_000 <= M <= 2_000_000 else PW_BLOCKS


# per-(map side, channels) grid cap of the fused depthwise backward where the per-site sweep beat MAX_BLOCKS by more
# than its ~2 % noise (profiles/r5_grid_sites.log: 38x38x288 1328 -> 1277 us, 38x38x192 1484 -> 1423, 19x19x288
# 574 -> 537, 19x19x576 686 -> 661)
_DW_BWD_BLOCKS = {(38, 288): 1024, (38, 192): 512, (19, 288): 512, (19, 576): 256}
# ... and of the stem forward / weight gradient and block 2's y1-free depthwise pair (same sweep: stem 527 -> 509 and
# 782 -> 760 us, dw_fwd_x 1900 -> 1832 us, dw_bwd_fused_x 3773 -> 3734 us)
STEM_FWD_BLOCKS, STEM_BWD_BLOCKS, XMODE_BLOCKS = 3072, 1536, 4096
# RT1_BLOCK_TIMING=1: HIP events around every block's forward / backward (tools/block_timing.py)
_TIMING = os.environ.get("RT1_BLOCK_TIMING", "0") == "1"
TIMING_EVENTS: List = []


def _mark(name: str):
    if _TIMING:
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        TIMING_EVENTS.append((name, ev))
# tall-skinny MFMA kernel for wide-K / narrow-N 1x1 convs (switch pw_tall=0 routes them to hipBLASLt)
PW_TALL = switches.on("pw_tall")
_SHADOW = None   # data_ptr(fp32 master weight) -> bf16 view of the per-step shadow (FusedRT1.attach_flat)


def set_weight_shadow(views):
    global _SHADOW
    _SHADOW = views


def _bf(w: torch.Tensor) -> torch.Tensor:
    """bf16 copy of a weight: the per-step shadow when one is attached, else a cast."""
    if _SHADOW is not None:
        s = _SHADOW.get(w.data_ptr())
        if s is not None and s.shape == w.shape:
            return s
    return w.to(BF)


def _lin(a: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """1x1 conv as a @ w^T for a [M, K] bf16, w [N, K] bf16.

    The skinny high-resolution shapes (K, N <= 288; HBM-bound) run on the MFMA streaming kernel of
    ``csrc/kernels/pwgemm.hip`` (86-100 % of the HBM roofline vs 15-70 % for hipBLASLt's macro tiles), the
    wide-K narrow-N ones on ``pwtall.hip``; the rest stay on hipBLASLt."""
    ext = _ext()
    if ext.pw_gemm_supported(a.shape[1], w.shape[0]):
        return ext.pw_gemm(a, w.contiguous(), _pw_blocks(a.shape[0]))[0]
    if PW_TALL and a.shape[0] >= 4096 and ext.pw_tall_preferred(a.shape[1], w.shape[0]):
        # wide reduction, narrow output (project convs, expand data-gradients; N <= 144): csrc/kernels/pwtall.hip
        return ext.pw_tall(a.contiguous(), w.contiguous())[0]
    return torch.mm(a, w.t())


# the wide-N top / block-25 expand 1x1 convs (K = 384 -> N = 1536 / 2304, M = 76,800) on gemm256.hip's 256 x 256 LDS-DMA
# tiles with the BN-statistics epilogue: 126 / 184 us against 138-164 / 196-249 us for the library, gemm.hip and pw_wide
# (tools/bench_gemm256.py, profiles/r5_gemm256_bench.log), and the bn_stats pass over the 1536 / 2304-wide output (61 / 94
# us per step) disappears.  g256=0: the pw_wide + bn_stats path.
G256_STATS = {(384, 1536), (384, 2304)} if switches.on("g256") else set()


def _lin_bn(a: torch.Tensor, w: torch.Tensor, bnc: "BNCtx", training: bool, pro=None):
    """1x1 conv + the consumer BatchNorm's constants; in training the batch statistics come from the
    GEMM epilogue (one pass over the output) when the MFMA kernel covers the shape.  ``pro = (scale, shift, gate,
    hw)`` makes the operand silu(a*scale + shift) * gate inside the GEMM (project convs, see project_fused)."""
    ext = _ext()
    if pro is not None:
        sc, sh, gate, hw, store = pro         # project_fused: pw_gemm-supported shapes only
        res = ext.pw_gemm(a, w.contiguous(), _pw_blocks(a.shape[0]), training, sc, sh, gate, hw, store)
        consts = bnc.train_consts(res[1], res[2], a.shape[0]) if training else bnc.eval_consts()
        return res[0], consts, (res[-1] if store else None)
    if training and ext.pw_stats_supported(a.shape[1], w.shape[0]):
        y, ps, pq = ext.pw_gemm(a, w.contiguous(), _pw_blocks(a.shape[0]), True)
        return y, bnc.train_consts(ps, pq, a.shape[0])
    if training and (a.shape[1], w.shape[0]) in G256_STATS:
        y, ps, pq = ext.gemm256(a, w.contiguous(), False, stats=True, bn=256)
        return y, bnc.train_consts(ps, pq, a.shape[0])
    y = _lin(a, w)
    return y, _bn_train_or_eval(bnc, training, y)


def _pw_bwd_blocks(M: int, z: bool = False) -> int:
    """Grid cap of the fused expand backward (pwbwd.hip), from sweeps at 768 frames
    (tools/scratch/pwbwd_grid_sweep.py, profiles/r2_pwbwd_grid_sweep.log): the 150x150 block wants 4096
    workgroups (-14 % vs 512), the 75x75 ones 2048 (-6 %), the 38x38 ones 512.  The y-free kernel (pw_bwd_z,
    tools/scratch/pwbwd_z_grid_sweep.py, profiles/r2_pwbwd_z_grid_sweep.log): flat from 1024 up at 150x150, 3072 at
    75x75 (-4..-5 % vs 2048), 512 at 38x38."""
    if M >= 10_000_000:
        return 4096
    if M >= 3_000_000:
        return 3072 if z else 2048
    return 512


def _dw_wgrad_blocks(C: int) -> int:
    """Grid cap of the depthwise weight-gradient kernel (``tools/gpu_wgb.sh`` sweep, partial-row sum
    included): the <= 144-channel high-resolution layers keep improving up to 4096 workgroups (-12 % vs 1024),
    the wider ones are flat from 1024 to 2048."""
    return 4096 if C <= 144 else 2048


def _mm_f32(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """bf16 x bf16 with fp32 output (weight gradients, reduction over millions of rows)."""
    try:
        return torch.mm(a, b, out_dtype=torch.float32)
    except (TypeError, RuntimeError):
        return torch.mm(a, b).float()


def _wgrad_splits(M: int, out_elems: int) -> int:
    """Split-K factor of the weight-gradient batched GEMM, fitted to MI355X sweeps of the encoder's shapes
    (``tools/debug/wgrad_sweep.py``; 1.2-1.8x faster than a rows-per-split rule): the best split keeps
    ~4-70 k rows per batch entry, enough batch entries to fill the chip, and few fp32 partials to sum."""
    if M >= 8_000_000:
        S = 256
    elif M >= 2_000_000:
        S = 128
    elif M >= 600_000:
        S = 256
    elif M >= 150_000:
        S = 64 if out_elems < 40_000 else 32
    elif M >= 16_384:
        S = 16
    else:
        S = max(1, M // 2048)
    return max(1, min(S, M // 256))


WGRAD_MFMA = switches.on("wgrad_mfma")
DW_FUSED = switches.on("dw_fused")      # fused stride-1 depthwise backward


PW_PRO = switches.on("pw_pro")          # project-conv operand prologue
# (not in the tall-skinny kernel of blocks 8-17: the 2 transcendentals per element make that HBM-bound GEMM
# VALU-bound, 0.1-0.4 ms/step slower than bn_apply + the plain kernel -- profiles/r2_pw_tall_pro_ab.log,
# profiles/r3_pw_tall_pro_ab.log; the kernel keeps the prologue, tests/test_pwgemm_gpu.py)


def project_fused(Ce: int, Cout: int, HW2: int) -> bool:
    """Build the project conv's operand A = silu(bn2(y2)) * gate in the skinny GEMM's registers instead of a
    bn_apply pass (read y2 + write A, then the GEMM reads A).  In training the GEMM also stores A for the weight
    gradient (store_operand): rebuilding A a second time inside the wgrad kernel measured 1.8x slower there than the
    saved pass (profiles/r2_project_prologue_ab.log), so the win is the bn_apply read of y2 and the GEMM's read of A."""
    if not PW_PRO:
        return False
    ext = _ext()
    return HW2 >= 128 and ext.pw_gemm_supported(Ce, Cout)


# project-conv backward of the skinny blocks from (dy3, y2) per frame (csrc/kernels/projbwd.hip): the SE / BN2
# backward sums and dWp come out of one pass, so the forward no longer stores the operand A and the backward no longer
# reads A (dWp) nor dA (se_bn_bwd_reduce)
PROJ_BWD = switches.on("proj_bwd")


def proj_bwd_fused(Ce: int, Cout: int, HW2: int) -> bool:
    return PROJ_BWD and project_fused(Ce, Cout, HW2) and _ext().proj_bwd_supported(Cout, Ce)


# squeeze-excitation MLP forward / backward as the fused se.hip kernels (se_fwd / se_bwd) instead of hipBLASLt
# addmm/mm + elementwise launches.  The round-2 pair was 2.5-5x slower (profiles/r2_se_fused_ab.log: per-frame dot
# products as long dependent FMA chains on 96 workgroups); the round-3 kernels (tiled split-K row products, sliced
# frame reductions) beat the library path: 1278-1282 -> 1293-1295 samples/s same-box A/B (profiles/r3_se_fused_ab.log).
SE_FUSED = switches.on("se_fused")
# Rounds 3-4 ran it on one rank only: the two-rank rehearsal (two processes on one GPU) saw SE fc1 weight gradients
# differ run to run.  Root cause (profiles/r4_se_dp_rootcause.md): a v_pk_fma_f32 with a high-element op_sel in
# se_wsum_part occasionally lost its low-lane product for 16 lanes -- dw1 came out as the exact sum minus one frame's
# term.  The SE kernels are now built without packed fp32 (NO_PACKED_FP32, tests/test_isa_audit.py) and the fused
# path is on for any world size.


def se_fused_active() -> bool:
    return SE_FUSED


# RT1_SE_DEBUG=1 (tools/dp_gpu_check.py): the fused SE forward keeps copies of (pool, h, gate); the backward flags any
# of them changed since the forward and re-runs se_bwd on the same inputs to flag a non-reproducible output.  Flags
# are device booleans collected in SE_DEBUG_LOG (eager steps only, never inside a capture).
_SE_DEBUG = os.environ.get("RT1_SE_DEBUG", "0") == "1"
SE_DEBUG_LOG: List = []
_SE_NAMES = ("dw2", "db2", "dw1", "db1", "rb", "db2bn", "dg2", "mdz2", "mdzx2")


def _se_debug_check(ext, index: int, saved, args, outs):
    """RT1_SE_DEBUG: inputs changed since the forward?  Re-run se_bwd on the same inputs: which outputs differ?  On a
    dw1 difference (host-synchronous): how many distinct (row, column) positions, and how many distinct results over
    8 more re-runs; RT1_SE_DUMP=<dir> also saves the inputs and both outputs for an offline replay."""
    red, gate, h, pool = args[:4]
    for nm, a, b in (("pool", pool, saved[0]), ("h", h, saved[1]), ("gate", gate, saved[2])):
        SE_DEBUG_LOG.append((f"blk{index}.{nm}", (a != b).sum()))
    rerun = ext.se_bwd(*args)
    for nm, a, b in zip(_SE_NAMES, outs, rerun):
        SE_DEBUG_LOG.append((f"blk{index}.{nm}_rerun", (a != b).sum()))
    bad = outs[2] != rerun[2]
    if not bool(bad.any()):
        return
    where = bad.nonzero()
    SE_DEBUG_LOG.append((f"blk{index}.dw1_bad_rows", int(where[:, 0].unique().numel())))
    SE_DEBUG_LOG.append((f"blk{index}.dw1_bad_cols", int(where[:, 1].unique().numel())))
    results = [outs[2], rerun[2]] + [ext.se_bwd(*args)[2] for _ in range(8)]
    distinct = []
    for r in results:
        if not any(torch.equal(r, d) for d in distinct):
            distinct.append(r)
    SE_DEBUG_LOG.append((f"blk{index}.dw1_distinct_of_10", len(distinct)))
    SE_DEBUG_LOG.append((f"blk{index}.dw1_first_eq_later", sum(torch.equal(outs[2], r) for r in results[2:])))
    dump = os.environ.get("RT1_SE_DUMP")
    if dump:
        os.makedirs(dump, exist_ok=True)
        rank = int(os.environ.get("RANK", "0"))
        torch.save({"args": [a.detach().cpu() if torch.is_tensor(a) else a for a in args],
                    "first": outs[2].cpu(), "rerun": rerun[2].cpu()},
                   os.path.join(dump, f"se_r{rank}_b{index}_{len(os.listdir(dump))}.pt"))
# the stem's BatchNorm + SiLU applied inside block 0 (StemPreFn): no separate activated stem tensor
STEM_IN_BLOCK0 = switches.on("stem_in_block0")
# ... and the stem BN's backward-apply folded into the stem weight-gradient kernel's staging: block 0
# hands the stem the gradient of silu(bn(x)) plus the BN backward constants through a StemLink instead of writing
# the [N, 150, 150, 40] dy (one write + one read of 1.4 GB per step at b128)
STEM_BN_BWD_FUSED = switches.on("stem_bn_bwd")


class StemLink:
    """Side channel from block 0's backward to StemPreFn's backward (both run in the same autograd pass; x's only
    consumer is block 0, so the tensor block 0 returns for x reaches the stem unchanged)."""

    def __init__(self):
        self.bn = None
# stride-2 blocks through the unified stride-2 kernel (dw_bwd_uni_s2_kernel) instead of bn_bwd_apply + data + weight
DW_S2_FUSED = switches.on("dw_s2_fused")
# dw_bwd_fused kernel variant: 1 = unified single-pass kernel (dw_bwd_uni_kernel), 0 = the two-pass kernel
DW_VARIANT = int(switches.get("dw_variant"))
# y-free expand backward (pwbwd.hip pw_bwd_z): the unified depthwise backward stores dz = dA1 * silu'(bn1(y1)) and
# the expand dgrad / wgrad are rewritten over the block input x (dy1 = k1*dz + k2*(x @ We^T) + k0), so the Ce-wide
# y1 is not read a second time in the backward
PW_BWD_Z = switches.on("pw_bwd_z")


# ... also for the wide expand convs whose dgrad runs on the tall-skinny kernel (blocks 9-17: Cin 96 / 136).  The first
# version (library GEMMs for x @ Mk and G, a VALU Mk kernel) measured net slower (profiles/r2_pw_z_wide_ab.log); this
# one folds x @ Mk + r0 into the dgrad's K loop (pw_tall_tail) and runs G on the MFMA weight-gradient kernel.
PW_Z_WIDE = switches.on("pw_z_wide")


def pw_bwd_z_preferred(Ce: int, Cin: int, k: int, H2: int, W2: int, s: int) -> bool:
    """dz-mode expand backward: needs the unified depthwise kernel (its BN1 epilogue stores dz); the fused pwbwd.hip
    kernel for the high-resolution shapes, library / MFMA GEMMs around pw_z_prep / pw_z_finish for the wide ones."""
    ext = _ext()
    if not (PW_BWD_Z and dw_fused_preferred(k, H2, W2, s) and (s == 2 or DW_VARIANT == 1)):
        return False
    if ext.pw_bwd_supported(Ce, Cin):
        return True
    if PW_Z_WIDE and z_gemm_preferred(Ce, Cin):
        return True
    return (PW_Z_WIDE and PW_TALL and ext.pw_tall_preferred(Ce, Cin) and wgrad_mfma_preferred(1 << 20, Cin, Cin)
            and (Ce, Cin) not in _Z_WIDE_OFF)


# ... and for the deep blocks 19-24 (expand 232 -> 1392), whose data gradient runs on gemm.hip's two-segment kernel
# (gemm_tail: dz . (diag(k1) We) + x . Mk + r0 + dout * fmul in one pass).  Replaces the bn_bwd_apply pass over the
# Ce-wide (dA1, y1) -> dy1, the hipBLASLt dgrad of dy1 and the add_scaled_ residual pass.  (Ce, Cin) -> gemm.hip tile
# config (-1: automatic).  Blocks 13-18 keep the tall-skinny pw_tall_tail (faster at N = 96 / 136).  Measured
# step-neutral (profiles/r3_z_gemm_ab.log: 1297-1301 samples/s either way; the removed passes are paid for by the
# slower-than-library gemm.hip tiles at N = 232 / 384), on by default for 12 fewer launches and 7 fewer hipBLASLt
# GEMMs per step.  z_gemm=1 (default since the round-5 re-check, profiles/r5_switch_recheck_ab.log: +0.15 %): blocks
# 19-24 only; 2: also block 25's 2304 -> 384; 0: the bn_bwd_apply + library path.
_ZG = switches.get("z_gemm")
Z_GEMM = {} if _ZG == "0" else ({(1392, 232): -1, (2304, 384): -1} if _ZG == "2" else {(1392, 232): -1})


def z_gemm_preferred(Ce: int, Cin: int) -> bool:
    return (Ce, Cin) in Z_GEMM


# y1-free expand blocks ("x-mode", csrc/kernels/dwconv.hip stage_xmfma + xexpand.hip): the expand output y1 is never
# written.  BN1's batch statistics come from the block input's Gram matrix (sum y1 = We sum x, sum y1^2 = w^T G w),
# the depthwise forward and its unified backward recompute y1 = x @ We^T per staged tile on MFMA, and the expand
# backward is the dz-mode pw_bwd_z (it reads dz and x only).  Removes the expand GEMM's write of y1 and both depthwise
# reads of it.  The kernels cover blocks 2-8 (Cin <= 48), but the depthwise backward is VALU-issue bound and holds
# its K x K weight-gradient accumulators in registers: recomputing y1 there (MFMA staging, LDS for the centres) made
# the backward of blocks 3-8 slower than the y1 bytes it saves, so by default only block 2 (150x150 -> 75x75, 5 GB of
# y1 per step) runs y1-free (profiles/r3_xmode_ab.md).  xmode=all: every supported block; 0: none.
_XMODE_ENV = switches.get("xmode")
XMODE = _XMODE_ENV != "0"
XMODE_SHAPES = None if _XMODE_ENV == "all" else {(24, 144, 3, 2)}   # (Cin, Ce, k, s)


def x_mode_preferred(Cin: int, Ce: int, k: int, s: int, H2: int, W2: int) -> bool:
    ext = _ext()
    if not XMODE or (XMODE_SHAPES is not None and (Cin, Ce, k, s) not in XMODE_SHAPES):
        return False
    return (ext.dw_x_supported(Cin, Ce, k, s) and ext.pw_bwd_supported(Ce, Cin)
            and pw_bwd_z_preferred(Ce, Cin, k, H2, W2, s))


# BN1 of the wide expand convs (blocks 9-25: Cin 96-384 -> Ce 576-2304 on pwgemm.hip's wide kernel, no statistics
# epilogue) from G = x^T x and sx = sum x -- the same wgrad(x, x) / colsum(x) the dz-mode expand backward needs, now
# computed once in the forward and handed to the backward -- instead of a bn_stats pass over the 6x wider y1
# (65-130 us per block: profiles/r4_pmc_bytes.md).  gram_bn=0: the bn_stats pass.
GRAM_BN = switches.on("gram_bn")


def gram_bn_preferred(Cin: int, Ce: int) -> bool:
    ext = _ext()
    return (GRAM_BN and Cin % 8 == 0 and not ext.pw_stats_supported(Cin, Ce) and ext.pw_gemm_supported(Cin, Ce)
            and (WGRAD_MFMA and wgrad_mfma_preferred(1 << 20, Cin, Cin)))


def gram_moments(x2d: torch.Tensor):
    """(G = x^T x fp32 [Cin, Cin], sx = sum_rows x fp32 [Cin]): one pass of the MFMA wgrad kernel that also sums the
    rows it stages, one fixed-order sum of both partial sets (bindings.cpp gram; ``gram_sx=0``: wgrad + colsum(x))."""
    if not (GRAM_SX and WGRAD_MFMA and wgrad_mfma_preferred(*x2d.shape, x2d.shape[1])):
        return wgrad(x2d, x2d), _ext().colsum(x2d)
    x2d = x2d.contiguous()
    cfg = _WGRAD_TILE.get((x2d.shape[1], x2d.shape[1]))
    if cfg is None:
        G, sx = _ext().gram(x2d)
    else:
        variant, rows_per_split = cfg
        G, sx = _ext().gram(x2d, variant, max(1, min(2048, round(x2d.shape[0] / rows_per_split))))
    return G, sx


GRAM_SX = switches.on("gram_sx")


def gram_bn_consts(x2d: torch.Tensor, We_b: torch.Tensor, bnc: "BNCtx"):
    """Train-mode BN1 constants of y1 = x2d @ We_b^T from x2d alone: G = x^T x and sum x in one MFMA pass, the
    quadratic forms in fp64 (csrc/kernels/xexpand.hip); running stats updated in place."""
    bn = bnc.bn
    return tuple(_ext().x_bn_stats(x2d, We_b, bn.weight, bn.bias, bn.eps, bn.momentum, bn.running_mean,
                                   bn.running_var))


# Project convs of the deep blocks on the tiled MFMA GEMM (csrc/kernels/gemm.hip) with the operand prologue
# A = silu(bn2(y2)) * gate and the BN3-statistics epilogue: replaces bn_apply (read y2, write A) + the hipBLASLt GEMM
# (read A) + bn_stats (read y3); A is still stored (by the first N tile) for the weight gradient.  (Ce, Cout) -> tile
# config, from tools/bench_gemm_mfma.py (profiles/r3_gemm_bench.log: 1.38-1.42x over the three launches); the
# K = 2304 / 1392 -> 384 shapes stay on the library (0.7x).
GEMM_PROJ = {(1392, 232): 1, (816, 232): 1} if switches.on("gemm_proj") else {}


def project_gemm(y2: torch.Tensor, Wp_b: torch.Tensor, sc2, sh2, gate, hw: int, bnc: "BNCtx", training: bool,
                 store_a: bool):
    """y3 = (silu(bn2(y2)) * gate) @ Wp^T with BN3's batch statistics from the epilogue -> (y3, consts, A|None)."""
    Ce = y2.shape[-1]
    M2 = y2.numel() // Ce
    res = _ext().gemm(y2.view(M2, Ce), Wp_b, False, None, sc2, sh2, gate, hw, stats=training,
                      cfg=GEMM_PROJ[(Ce, Wp_b.shape[0])], store_a=store_a)
    consts = bnc.train_consts(res[1], res[2], M2) if training else bnc.eval_consts()
    return res[0], consts, (res[-1] if store_a else None)


# ... and their data gradients dA = dy3 @ Wp (NN; profiles/r3_gemm_bench.log "proj19 dgrad": 1.32x over hipBLASLt)
GEMM_PROJ_DGRAD = {(1392, 232): 0, (816, 232): 0} if switches.on("gemm_proj_dgrad") else {}


# the residual path's gradient added in the wide dz-mode dgrad's epilogue instead of an add_scaled_ pass
TALL_RES = switches.on("tall_res")
# ... and, for the non-expand residual block 1, in the unified depthwise backward's store
DW_RES = switches.on("dw_res")
# shapes the wide dz-mode path does not pay for (filled from A/B runs)
_Z_WIDE_OFF = set()


def _few_splits(part: torch.Tensor) -> torch.Tensor:
    """Split partials [S, Co, Ci] as they are for S <= 4 (the consumer sums them), else their fixed-order colsum: a
    per-element loop over the 64-256 splits of the tall z-mode gradients made pw_z_finish latency-bound (40 -> 174 us
    for the 19x19 blocks, gpurun_out/trN vs trN_film)."""
    return part if part.shape[0] <= 4 else _ext().colsum(part)


def expand_bwd_z_wide(dz: torch.Tensor, x: torch.Tensor, We: torch.Tensor, consts: torch.Tensor, res=None, gram=None):
    """Expand-conv backward of a wide block from dz [M, Ce] and the block input x [M, Cin] (y1 is not read):
    dx = dz @ (diag(k1) We) + x @ Mk + r0 and dWe = diag(k1) dz^T x + diag(k2) We G + k0 (x) sx with
    Mk = We^T diag(k2) We, G = x^T x, sx = sum_m x (csrc/kernels/pwbwd.hip pw_z_prep / pw_z_finish, pwtall.hip
    pw_tall_tail).  Replaces bn_bwd_apply (read dA1 and y1, write dy1) + the dgrad / wgrad reads of dy1 by two
    reads of dz and three of the 6x narrower x.  ``res = (dout, fmul, hw)`` adds the residual path's gradient
    dout * fmul[frame] in the dgrad epilogue (no add_scaled_ pass)."""
    ext = _ext()
    wt, mk, r0 = ext.pw_z_prep(We, consts)     # (diag(k1) We)^T, We^T diag(k2) We, k0 @ We in one launch
    if res is not None:
        dx = ext.pw_tall_tail(dz, wt, x, mk, r0, res[0], res[1], res[2])
    else:
        dx = ext.pw_tall_tail(dz, wt, x, mk, r0)
    S = _few_splits(wgrad(dz, x, raw=True))  # up to 4 split partials are summed inside pw_z_finish
    G, sx = gram if gram is not None else gram_moments(x)     # from the forward's BN1 when it used them
    return dx, ext.pw_z_finish(S, G, sx, We, consts)


def expand_bwd_z_gemm(dz: torch.Tensor, x: torch.Tensor, We: torch.Tensor, consts: torch.Tensor, res=None, gram=None):
    """expand_bwd_z_wide with the data gradient on gemm.hip (``Z_GEMM`` shapes): dx = dz @ (diag(k1) We) + x @ Mk + r0
    (+ dout * fmul[frame]) as one two-segment GEMM (csrc/kernels/gemm.hip TAIL); dWe as in expand_bwd_z_wide."""
    ext = _ext()
    wt, mk, r0 = ext.pw_z_prep(We, consts)     # wt [Cin, Ce] = (diag(k1) We)^T, mk [Cin, Cin], r0 [Cin]
    cfg = Z_GEMM.get((We.shape[0], We.shape[1]), -1)
    if res is not None:
        dx = ext.gemm_tail(dz, wt, x, mk, r0, res[0], res[1], res[2], cfg)
    else:
        dx = ext.gemm_tail(dz, wt, x, mk, r0, cfg=cfg)
    S = _few_splits(wgrad(dz, x, raw=True))  # up to 4 split partials are summed inside pw_z_finish
    G, sx = gram if gram is not None else gram_moments(x)     # from the forward's BN1 when it used them
    return dx, ext.pw_z_finish(S, G, sx, We, consts)


def dw_fused_preferred(k: int, H: int, W: int, s: int = 1) -> bool:
    """Per-layer choice between dw_bwd_fused and the unfused sequence, from tools/bench_dw_fused.py at 768 frames.
    The unified kernel (profiles/r2_dw_uni_ab.log) beats the unfused sequence on every stride-1 layer, including the
    19x19 k5 ones (blocks 13-17) where the two-pass kernel ran 12 % slower than unfused
    (profiles/r2_dw_bwd_fused_ab.log)."""
    if not DW_FUSED:
        return False
    if s == 2:
        return DW_S2_FUSED
    return DW_VARIANT != 0 or not (k == 5 and 200 <= H * W <= 1000)


def wgrad(dy: torch.Tensor, x: torch.Tensor, prologue=None, final: bool = False, ok: bool = True,
          raw: bool = False) -> torch.Tensor:
    """Weight gradient dy^T @ a for dy [M, Co], x [M, Ci] bf16 -> fp32 [Co, Ci], on the streaming MFMA kernel
    (csrc/kernels/wgrad.hip).  ``prologue = (scale, shift, gate, act, hw)`` rebuilds a = act(x*scale+shift)*gate
    inside the kernel (the project conv's input A from y2).  ``final``: the result is a parameter's gradient as is
    (``ok``: that parameter requires one), so the split-K partial sum may be left to the flat gather
    (parallel/flat.py defer_partials).  ``raw``: the [splits, Co, Ci] partials themselves, for a consumer kernel
    that sums them (pw_z_finish)."""
    ext = _ext()
    final = final or raw
    if prologue is not None or (WGRAD_MFMA and wgrad_mfma_preferred(dy.shape[0], dy.shape[1], x.shape[1])):
        dy, x = dy.contiguous(), x.contiguous()
        if prologue is None:
            cfg = _WGRAD_TILE.get((dy.shape[1], x.shape[1]))
            if cfg is None:
                out = ext.wgrad(dy, x, partials=final)
            else:
                variant, rows_per_split = cfg
                out = ext.wgrad(dy, x, variant=variant, splits=max(1, min(2048, round(dy.shape[0] / rows_per_split))),
                                partials=final)
        else:
            sc, sh, gate, act, hw = prologue
            out = ext.wgrad(dy, x, sc, sh, gate, act, hw, partials=final)
        if raw:
            return out
        return defer_partials(out, ok) if final else out
    if prologue is not None:
        raise ValueError("wgrad prologue needs the MFMA kernel (bf16, channels % 8)")
    return wgrad_bmm(dy, x, final, ok, raw)


# (Co, Ci) -> (tile variant of csrc/kernels/wgrad.hip VARIANTS, rows per split) of every plain wgrad call of the step,
# from the per-site sweep of tools/bench_wgrad_sites.py at 768 frames (profiles/r5_wgrad_sites.log, variant x split
# count against the automatic pick: the Gram matrix of blocks 19-24 52.0 -> 32.6 us, the 19x19 expand / project
# gradients 108 / 104 -> 99 / 96 us, block 13's project 157 -> 139 us).  (136, 576) and (232, 816) are the deep
# shapes where the MFMA kernel beats hipBLASLt's split-K at all (profiles/r2_wgrad_variants.log).
_WGRAD_TILE = {(136, 576): (1, 2166), (232, 816): (2, 1600)} if switches.on("wgrad_deep") else {}
_WGRAD_TILE.update({(96, 96): (1, 1083), (136, 136): (1, 2166), (576, 96): (2, 2166), (96, 576): (2, 2166),
                    (96, 288): (2, 1083), (232, 232): (1, 1200), (64, 512): (1, 600)})


def wgrad_mfma_preferred(M: int, Co: int, Ci: int) -> bool:
    """Shape rule from the per-site sweeps (profiles/r2_wgrad_variants.log, 768 frames at 300x300): the streaming
    MFMA kernel wins for the mid-resolution layers (Co*Ci <= ~56k, M <= ~5M rows: blocks 2-12, 20-45 % faster) and
    the two deep shapes of _WGRAD_TILE; hipBLASLt's split-K keeps the very tall skinny ones (blocks 0-1) and the other
    wide deep ones (14-25: 1.4-2x faster there)."""
    if Co % 8 or Ci % 8 or M > 5_000_000:
        return False
    return Co * Ci <= 56_000 or (Co, Ci) in _WGRAD_TILE


# (Co, Ci) -> rows per split of the library split-K weight gradient where the per-site sweep beat _wgrad_splits
# (tools/bench_wgrad_sites.py --bmm, profiles/r5_wgrad_bmm_sites.log: block 14-17 project 197 -> 170 us at 64 splits,
# top 156 -> 142 and block-25 expand 204 -> 184 us at 24); the library stays ahead of the MFMA kernel on all of these
_BMM_ROWS = {(136, 816): 4332, (1536, 384): 3200, (384, 2304): 3200}


def wgrad_bmm(dy: torch.Tensor, x: torch.Tensor, final: bool = False, ok: bool = True,
              raw: bool = False) -> torch.Tensor:
    """Weight gradient dy^T @ x for dy [M, Co], x [M, Ci] (M = frames*pixels, up to ~1e7 rows).

    A plain TN GEMM here has only (Co/16)*(Ci/16) output tiles (e.g. 18 for
    144x24) and one workgroup streams all M rows; split-K as a batched GEMM
    over S row chunks gives S times the parallelism, then an fp32 sum."""
    M = dy.shape[0]
    rps = _BMM_ROWS.get((dy.shape[1], x.shape[1]))
    S = max(1, M // rps) if rps else _wgrad_splits(M, dy.shape[1] * x.shape[1])
    if S == 1:
        out = _mm_f32(dy.t(), x)
        return out[None] if raw else out
    rows = M // S
    M1 = rows * S
    a = dy[:M1].view(S, rows, dy.shape[1]).transpose(1, 2)
    b = x[:M1].view(S, rows, x.shape[1])
    try:
        part = torch.bmm(a, b, out_dtype=torch.float32)
    except (TypeError, RuntimeError):
        part = torch.bmm(a, b).float()
    if M1 < M:                                # the leftover rows join the first split
        part[0] += _mm_f32(dy[M1:].t(), x[M1:])
    if raw:
        return part.contiguous()
    if final:
        return defer_partials(part.contiguous(), ok)
    return _ext().colsum(part)                # deterministic fixed-order sum (csrc/kernels/reduce.hip)


def _partials(M: int) -> int:
    return int(max(1, min(1024, (M + 255) // 256)))


class BNCtx:
    """Per-BN bookkeeping shared by forward and backward (not a tensor)."""

    def __init__(self, bn: torch.nn.BatchNorm2d):
        self.bn = bn

    def train_consts(self, psum, psq, count):
        bn = self.bn
        sc, sh, mu, rs = _ext().bn_finalize(psum, psq, float(count), bn.weight, bn.bias, bn.eps, bn.momentum,
                                            bn.running_mean, bn.running_var)
        return sc, sh, mu, rs

    def eval_consts(self):
        bn = self.bn
        rstd = torch.rsqrt(bn.running_var.float() + bn.eps)
        sc = bn.weight.float() * rstd
        sh = bn.bias.float() - bn.running_mean.float() * sc
        return sc.contiguous(), sh.contiguous(), bn.running_mean.float().contiguous(), rstd.contiguous()


def _bn_train_or_eval(bnc: BNCtx, training: bool, y2d: torch.Tensor = None, partials=None):
    if training:
        if partials is None:
            partials = _ext().bn_stats(y2d, _partials(y2d.shape[0]))
        count = y2d.shape[0] if y2d is not None else None
        return bnc.train_consts(partials[0], partials[1], count)
    return bnc.eval_consts()


class StemFn(torch.autograd.Function):
    """frames (uint8/f32 NCHW) -> silu(bn(conv3x3s2(shift(frames))))  [N, Ho, Wo, 40] bf16."""

    @staticmethod
    def forward(ctx, img, shift, w, gamma, beta, bnc: BNCtx, training: bool):
        ext = _ext()
        y, ps, pq = ext.stem_fwd(img, shift, w.reshape(40, 27).float().contiguous(), STEM_FWD_BLOCKS)
        M = y.numel() // 40
        if training:
            sc, sh, mu, rs = bnc.train_consts(ps, pq, M)
        else:
            sc, sh, mu, rs = bnc.eval_consts()
        a = ext.bn_apply(y, sc, sh, ACT_SILU, None, 0)
        ctx.save_for_backward(img, shift if shift is not None else torch.empty(0), y, sc, sh, mu, rs, gamma)
        ctx.has_shift = shift is not None
        return a

    @staticmethod
    def backward(ctx, da):
        ext = _ext()
        img, shift, y, sc, sh, mu, rs, gamma = ctx.saved_tensors
        shift = shift if ctx.has_shift else None
        da = da.contiguous()
        M = y.numel() // 40
        pa, pb = ext.bn_bwd_reduce(da, None, None, 0, y, sc, sh, mu, rs, ACT_SILU, _partials(M))
        mdz, mdzx, dg, db = ext.bn_bwd_finalize_new(pa, pb, float(M))
        dy = ext.bn_bwd_apply(da, None, None, 0, y, sc, sh, mu, rs, gamma.float().contiguous(), ACT_SILU, mdz, mdzx)
        dw = ext.stem_bwd_weight(img, shift, dy, STEM_BWD_BLOCKS).view(40, 3, 3, 3)
        return None, None, dw, dg, db, None, None


class StemPreFn(torch.autograd.Function):
    """frames -> y = conv3x3s2(shift(frames)) [N, Ho, Wo, 40] bf16, PRE-BatchNorm, plus the stem BN's constants
    (sc, sh, mean, rstd; batch statistics from the conv kernel's epilogue in training, running stats in eval).
    The BN + SiLU is applied by block 0 (its depthwise staging prologue, like an expand block's BN1), whose backward
    also returns the stem BN's gradients: the stem never writes the activated tensor (one [N,150,150,40] write + read
    per step) and its BN backward statistics come out of block 0's depthwise backward epilogue."""

    @staticmethod
    def forward(ctx, img, shift, w, bnc: BNCtx, training: bool, link: Optional[StemLink] = None):
        ext = _ext()
        y, ps, pq = ext.stem_fwd(img, shift, w.reshape(40, 27).float().contiguous(), STEM_FWD_BLOCKS)
        M = y.numel() // 40
        sc, sh, mu, rs = bnc.train_consts(ps, pq, M) if training else bnc.eval_consts()
        ctx.save_for_backward(img, shift if shift is not None else torch.empty(0))
        ctx.has_shift = shift is not None
        ctx.link = link
        ctx.mark_non_differentiable(sc, sh, mu, rs)
        ctx.set_materialize_grads(False)        # no zero-filled gradients for the four constants
        return y, sc, sh, mu, rs

    @staticmethod
    def backward(ctx, dy, *_):
        ext = _ext()
        img, shift = ctx.saved_tensors
        shift = shift if ctx.has_shift else None
        link = ctx.link
        if link is not None and link.bn is not None:
            # dy is the gradient of silu(bn(y)); the BN backward-apply runs in the kernel's staging
            x, sc, sh, mu, rs, g, mdz, mdzx = link.bn
            link.bn = None
            dw = ext.stem_bwd_weight(img, shift, dy.contiguous(), STEM_BWD_BLOCKS, x, sc, sh, mu, rs, g, mdz, mdzx)
        else:
            dw = ext.stem_bwd_weight(img, shift, dy.contiguous(), STEM_BWD_BLOCKS)
        return None, None, dw.view(40, 3, 3, 3), None, None, None


class MBConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, fmul, fadd, keep, We, g1, b1, Wd, g2, b2, f1w, f1b, f2w, f2b, Wp, g3, b3, meta):
        ext = _ext()
        spec, bns, training = meta[:3]
        # input-BN mode (block 0 after StemPreFn): x is the stem conv output BEFORE its BatchNorm; (sc, sh, mean,
        # rstd) of that BN arrive in meta, its gamma / beta in the g1 / b1 slots, and the block applies BN + SiLU in
        # the depthwise staging exactly as it applies BN1 to an expand conv's output
        in_consts = meta[3] if len(meta) > 3 else None
        _mark(f"fwd{spec.index}")
        N, H, W, Cin = x.shape
        Ce, Cout, k, s = spec.expand_ch, spec.out_ch, spec.kernel, spec.stride
        M = N * H * W
        expand = We is not None
        in_bn = in_consts is not None and not expand
        p_ = (k - 1) // 2
        H2_, W2_ = (H + 2 * p_ - k) // s + 1, (W + 2 * p_ - k) // s + 1
        xmode = expand and x_mode_preferred(Cin, Ce, k, s, H2_, W2_)
        gram = None                     # (x^T x, sum x) when BN1 came from them: reused by the dz-mode backward
        if xmode:
            # y1 = x @ We^T is never materialised (see XMODE): BN1 from x's Gram matrix, y1 rebuilt in dw_fwd_x
            We_b = _bf(We).reshape(Ce, Cin).contiguous()
            if training:
                sc1, sh1, mu1, rs1 = gram_bn_consts(x.view(M, Cin), We_b, bns[0])
            else:
                sc1, sh1, mu1, rs1 = bns[0].eval_consts()
            y1 = None
            dw_in, dsc, dsh, dact = None, sc1, sh1, ACT_SILU
        elif expand and training and gram_bn_preferred(Cin, Ce):
            We_b = _bf(We).reshape(Ce, Cin).contiguous()
            y1 = _lin(x.view(M, Cin), We_b).view(N, H, W, Ce)
            gram = gram_moments(x.view(M, Cin))
            bn = bns[0].bn
            sc1, sh1, mu1, rs1 = ext.bn_from_gram(gram[0], gram[1], We_b, float(M), bn.weight, bn.bias, bn.eps,
                                                  bn.momentum, bn.running_mean, bn.running_var)
            dw_in, dsc, dsh, dact = y1, sc1, sh1, ACT_SILU
        elif expand:
            y1, (sc1, sh1, mu1, rs1) = _lin_bn(x.view(M, Cin), _bf(We).reshape(Ce, Cin), bns[0], training)
            y1 = y1.view(N, H, W, Ce)
            dw_in, dsc, dsh, dact = y1, sc1, sh1, ACT_SILU
        elif in_bn:
            if spec.has_skip:
                raise ValueError("input-BN mode needs a block without a residual (its input is pre-activation)")
            y1 = None
            sc1, sh1, mu1, rs1 = in_consts
            dw_in, dsc, dsh, dact = x, sc1, sh1, ACT_SILU
        else:
            y1 = sc1 = sh1 = mu1 = rs1 = None
            dw_in, dsc, dsh, dact = x, None, None, ACT_NONE
        bn2, bn3 = bns[-2], bns[-1]
        if xmode:
            y2, ps2, pq2 = ext.dw_fwd_x(x, We_b, Wd.reshape(Ce, k * k).float().contiguous(), sc1, sh1, k, s,
                                        XMODE_BLOCKS)
        else:
            y2, ps2, pq2 = ext.dw_fwd(dw_in, Wd.reshape(Ce, k * k).float().contiguous(), dsc, dsh, dact, k, s,
                                      MAX_BLOCKS)
        _, H2, W2, _ = y2.shape
        HW2 = H2 * W2
        M2 = N * HW2
        if training:
            sc2, sh2, mu2, rs2 = bn2.train_consts(ps2, pq2, M2)
        else:
            sc2, sh2, mu2, rs2 = bn2.eval_consts()
        # squeeze-excitation (fp32, [N, Ce])
        se = spec.se_ch
        f1 = f1w.reshape(se, Ce).float()
        f2 = f2w.reshape(Ce, se).float()
        if se_fused_active():
            # pool sum -> fc1 -> SiLU -> fc2 -> sigmoid in two kernels (csrc/kernels/se.hip se_rowdot + se_rowmat);
            # the returned pool is the frame SUM (the backward applies 1/HW)
            pool, h, gate = ext.se_fwd(ext.frame_pool(y2.view(N, HW2, Ce), None, sc2, sh2, ACT_SILU), 1.0 / HW2,
                                       f1.contiguous(), f1b.float().contiguous(), f2.contiguous(),
                                       f2b.float().contiguous())
            hs = torch.empty(0, device=x.device)
            if _SE_DEBUG and not torch.cuda.is_current_stream_capturing():
                ctx.se_dbg = (pool.clone(), h.clone(), gate.clone())
        else:
            # the pooled SUM is kept; 1/HW rides on the GEMMs' alpha (no divide launch)
            pool = ext.frame_pool(y2.view(N, HW2, Ce), None, sc2, sh2, ACT_SILU)
            h = torch.addmm(f1b.float(), pool, f1.t(), alpha=1.0 / HW2)
            hs = F.silu(h)
            z = torch.addmm(f2b.float(), hs, f2.t())
            gate = torch.sigmoid(z).contiguous()
        if project_fused(Ce, Cout, HW2):
            # operand rebuilt in the GEMM's registers; stored (for dWp) only when a backward will follow
            need_a = (training or Wp.requires_grad or x.requires_grad) and not proj_bwd_fused(Ce, Cout, HW2)
            y3, (sc3, sh3, mu3, rs3), A = _lin_bn(y2.view(M2, Ce), _bf(Wp).reshape(Cout, Ce), bn3, training,
                                                  pro=(sc2, sh2, gate, HW2, need_a))
        elif (Ce, Cout) in GEMM_PROJ and HW2 >= 1 and gate.is_contiguous():
            need_a = training or Wp.requires_grad or x.requires_grad
            y3, (sc3, sh3, mu3, rs3), A = project_gemm(y2, _bf(Wp).reshape(Cout, Ce).contiguous(), sc2, sh2, gate,
                                                       HW2, bn3, training, need_a)
        else:
            A = ext.bn_apply(y2, sc2, sh2, ACT_SILU, gate, HW2)                 # [N, H2, W2, Ce]
            y3, (sc3, sh3, mu3, rs3) = _lin_bn(A.view(M2, Ce), _bf(Wp).reshape(Cout, Ce), bn3, training)
        skip = x if spec.has_skip else None
        keep_t = keep if (keep is not None and spec.has_skip) else None
        out = ext.block_tail(y3.view(N, HW2, Cout), sc3, sh3, keep_t, skip.view(N, HW2, Cout) if skip is not None
                             else None, fmul, fadd)
        ctx.meta = (spec, expand, (N, H, W, Cin, H2, W2), keep_t is not None, in_bn, xmode)
        ctx.gram = gram
        ctx.stem_link = meta[4] if (in_bn and len(meta) > 4) else None
        ctx.save_for_backward(x, fmul, keep_t if keep_t is not None else torch.empty(0), We if expand else torch.empty(0),
                              g1 if (expand or in_bn) else torch.empty(0), Wd, g2, f1w, f2w, Wp, g3,
                              y1 if y1 is not None else torch.empty(0), y2, A if A is not None else torch.empty(0), y3,
                              gate, pool, h, hs,
                              *(t if t is not None else torch.empty(0) for t in (sc1, sh1, mu1, rs1)),
                              sc2, sh2, mu2, rs2, sc3, sh3, mu3, rs3)
        _mark(f"fwd{spec.index}_end")
        return out.view(N, H2, W2, Cout)

    @staticmethod
    def backward(ctx, dout):
        ext = _ext()
        spec, expand, (N, H, W, Cin, H2, W2), has_keep, in_bn, xmode = ctx.meta
        _mark(f"bwd{spec.index}")
        (x, fmul, keep, We, g1, Wd, g2, f1w, f2w, Wp, g3, y1, y2, A, y3, gate, pool, h, hs,
         sc1, sh1, mu1, rs1, sc2, sh2, mu2, rs2, sc3, sh3, mu3, rs3) = ctx.saved_tensors
        keep = keep if has_keep else None
        Ce, Cout, k, s, se = spec.expand_ch, spec.out_ch, spec.kernel, spec.stride, spec.se_ch
        HW2 = H2 * W2
        M, M2 = N * H * W, N * H2 * W2
        dev = x.device
        dout = dout.contiguous().to(BF)
        skip = x.view(N, HW2, Cout) if spec.has_skip else None
        # ---- tail: FiLM grads, BN3 backward
        dmul, dadd, pdz3, pdzx3 = ext.tail_bwd_reduce(dout.view(N, HW2, Cout), y3.view(N, HW2, Cout), sc3, sh3, mu3,
                                                      rs3, keep, skip, fmul)
        mdz3, mdzx3, dg3, db3 = ext.bn_bwd_finalize_new(pdz3, pdzx3, float(M2))
        # ---- BN3 backward-apply + project data gradient
        Wp2 = _bf(Wp).reshape(Cout, Ce)
        pbf = A.numel() == 0 and proj_bwd_fused(Ce, Cout, HW2)
        kp = keep.float().contiguous() if keep is not None else None
        if (Ce, Cout) not in GEMM_PROJ_DGRAD and ext.pw_gemm_bnbwd_supported(Cout, Ce):
            # blocks 0-7: dy3 = BN3-backward(dout, y3) is built in the skinny GEMM's operand prologue and stored once
            # for the project weight gradient (no bn_bwd_apply launch, no second read of dy3)
            dA, dy3 = ext.pw_gemm_bnbwd(dout.view(M2, Cout), y3.view(M2, Cout), Wp2.t().contiguous(), fmul, kp, HW2,
                                        g3.float().contiguous(), mu3, rs3, mdz3, mdzx3, _pw_blocks(M2))
        else:
            # the drop-path mask scales the FiLM row multiplier inside the kernel (fmul * keep[frame])
            dy3 = ext.bn_bwd_apply(dout.view(M2, Cout), fmul, None, HW2, y3, sc3, sh3, mu3, rs3,
                                   g3.float().contiguous(), ACT_NONE, mdz3, mdzx3, kp)
            if (Ce, Cout) in GEMM_PROJ_DGRAD:
                dA = ext.gemm(dy3.view(M2, Cout), Wp2.contiguous(), True, cfg=GEMM_PROJ_DGRAD[(Ce, Cout)])[0]
            else:
                dA = _lin(dy3, Wp2.t())                                          # [M2, Ce]
        if pbf:
            # SE + BN2 backward sums and dWp from (dy3, y2) in one pass per frame, the dA-weighted sums contracted
            # through dA = dy3 @ Wp (csrc/kernels/projbwd.hip); the operand A was never stored
            red, dWp = ext.proj_bwd(dy3, y2.view(N, HW2, Ce), Wp2.contiguous(), gate, sc2, sh2, mu2, rs2)
            dWp = dWp.view_as(Wp)
        else:
            if A.numel() == 0:                    # forward ran without storing the operand
                A = ext.bn_apply(y2, sc2, sh2, ACT_SILU, gate, HW2)
            dWp = wgrad(dy3, A.view(M2, Ce), final=True, ok=ctx.needs_input_grad[14]).view_as(Wp)
            # ---- squeeze-excitation + BN2 backward statistics: ONE pass over (dA, y2)
            red = ext.se_bn_bwd_reduce(dA.view(N, HW2, Ce), y2.view(N, HW2, Ce), sc2, sh2, mu2, rs2)  # [5, N, Ce]
        f1 = f1w.reshape(se, Ce).float()
        f2 = f2w.reshape(Ce, se).float()
        # SE + BN2 backward glue in three kernels around the four small GEMMs (csrc/kernels/se.hip):
        #   dz = sum_hw(dA * a2) * g(1-g);  dh = (dz f2) * silu'(h);  rb = (dh f1) / HW (grad of a2 via the pool);
        #   BN2 sums: sum dz = sum_n gate*S1 + rb*S2,  sum dz*xhat = sum_n gate*S3 + rb*S4
        if se_fused_active():
            # per-frame chain + reductions over frames in two kernels (se_bwd_frame, se_bwd_wsum)
            df2w, df2b, df1w, df1b, rb, db2, dg2, mdz2, mdzx2 = ext.se_bwd(red, gate, h, pool, 1.0 / HW2,
                                                                          f1.contiguous(), f2.contiguous(), float(M2))
            dbg = getattr(ctx, "se_dbg", None)
            if dbg is not None and not torch.cuda.is_current_stream_capturing():
                _se_debug_check(ext, spec.index, dbg, (red, gate, h, pool, 1.0 / HW2, f1.contiguous(),
                                                       f2.contiguous(), float(M2)),
                                (df2w, df2b, df1w, df1b, rb, db2, dg2, mdz2, mdzx2))
                ctx.se_dbg = None
            df2w, df1w = df2w.view_as(f2w), df1w.view_as(f1w)
        else:
            dz, df2b = ext.se_bwd_dz(red[0], gate)
            df2w = (dz.t() @ hs).view_as(f2w)
            dh, df1b = ext.se_bwd_dh(dz @ f2, h)
            df1w = torch.addmm(_scalar_zero(dev), dh.t(), pool, beta=0.0, alpha=1.0 / HW2).view_as(f1w)
            rb, db2, dg2, mdz2, mdzx2 = ext.se_bwd_bnsum(red, gate, dh @ f1, 1.0 / HW2, float(M2))
        wd = Wd.reshape(Ce, k * k).float().contiguous()
        pre = expand or in_bn          # the depthwise input is BN + SiLU of a stored pre-activation tensor
        x1 = y1 if expand else x
        zmode = expand and (xmode or pw_bwd_z_preferred(Ce, Cin, k, H2, W2, s))
        skip_done = False
        if xmode:
            # y1 recomputed per tile from (x, We) on MFMA; the kernel stores dz for pw_bwd_z
            res = ext.dw_bwd_fused_x(dA.view(N, H2, W2, Ce), y2, gate, rb.contiguous(), sc2, sh2, mu2, rs2,
                                     g2.float().contiguous(), mdz2, mdzx2, wd, k, x, _bf(We).reshape(Ce, Cin).contiguous(),
                                     sc1, sh1, mu1, rs1, XMODE_BLOCKS, True)
            dy2 = None
            dWd = res[1].view_as(Wd)
            dA1, pa1, pb1 = res[0], res[2], res[3]
        elif dw_fused_preferred(k, H2, W2, s):
            # BN2 backward-apply + depthwise data AND weight gradients in one pass; dy2 never reaches HBM
            # (csrc/kernels/dwconv.hip dw_bwd_uni_kernel / dw_bwd_uni_s2_kernel)
            # non-expand residual block (block 1): the residual gradient dout * fmul joins dx in the kernel's store
            dw_res = DW_RES and not pre and spec.has_skip and s == 1 and DW_VARIANT != 0
            res = ext.dw_bwd_fused(dA.view(N, H2, W2, Ce), y2, gate, rb.contiguous(), sc2, sh2, mu2, rs2,
                                   g2.float().contiguous(), mdz2, mdzx2, wd, k, x1,
                                   sc1 if pre else None, sh1 if pre else None,
                                   ACT_SILU if pre else ACT_NONE, mu1 if pre else None,
                                   rs1 if pre else None, _DW_BWD_BLOCKS.get((H2, Ce), MAX_BLOCKS), DW_VARIANT, zmode,
                                   dout.view(N, H, W, Cin) if dw_res else None,
                                   fmul.float().contiguous() if dw_res else None)
            skip_done = dw_res
            dy2 = None
            dWd = res[1].view_as(Wd)
            if pre:
                dA1, pa1, pb1 = res[0], res[2], res[3]
            else:
                dx = res[0]
        else:
            dy2 = ext.bn_bwd_apply(dA, gate, rb, HW2, y2, sc2, sh2, mu2, rs2, g2.float().contiguous(), ACT_SILU,
                                   mdz2, mdzx2).view(N, H2, W2, Ce)
        # ---- depthwise backward
        if expand:
            if dy2 is not None:
                dA1, pa1, pb1 = ext.dw_bwd_data(dy2, wd, H, W, k, s, y1, sc1, sh1, mu1, rs1, MAX_BLOCKS)
                dWd = ext.dw_bwd_weight(dy2, y1, sc1, sh1, ACT_SILU, k, s, _dw_wgrad_blocks(Ce)).view_as(Wd)
            if zmode and not ext.pw_bwd_supported(Ce, Cin):
                mdz1, mdzx1, dg1, db1, consts = ext.bn_bwd_finalize_pw(pa1, pb1, float(M), sc1, sh1,
                                                                       g1.float().contiguous(), mu1, rs1)
                res = spec.has_skip and TALL_RES
                zfn = expand_bwd_z_gemm if z_gemm_preferred(Ce, Cin) else expand_bwd_z_wide
                dx2, dWe = zfn(dA1.view(M, Ce), x.view(M, Cin), _bf(We).reshape(Ce, Cin), consts.contiguous(),
                               (dout.view(M, Cin), fmul.float().contiguous(), H * W) if res else None, ctx.gram)
                ctx.gram = None
                dx = dx2.view(N, H, W, Cin)
                dWe = dWe.view_as(We)
                skip_done = res
            elif zmode:
                # dA1 holds dz = dA1 * silu'(bn1(y1)); dgrad / wgrad over x instead of y1 (csrc/kernels/pwbwd.hip)
                mdz1, mdzx1, dg1, db1, consts = ext.bn_bwd_finalize_pw(pa1, pb1, float(M), sc1, sh1,
                                                                       g1.float().contiguous(), mu1, rs1)
                res = spec.has_skip
                dx2, dWe = ext.pw_bwd_z(dA1.view(M, Ce), x.view(M, Cin), _bf(We).reshape(Ce, Cin), consts.contiguous(),
                                        dout.view(M, Cin) if res else None, fmul.float().contiguous() if res else None,
                                        H * W, _pw_bwd_blocks(M, z=True))
                dx = dx2.view(N, H, W, Cin)
                dWe = dWe.view_as(We)
                skip_done = res
            elif ext.pw_bwd_supported(Ce, Cin):
                # SiLU/BN1 backward + dgrad + wgrad of the expand conv in ONE pass (csrc/kernels/pwbwd.hip); its five
                # per-channel constants come out of the BN1 finalize launch
                mdz1, mdzx1, dg1, db1, consts = ext.bn_bwd_finalize_pw(pa1, pb1, float(M), sc1, sh1,
                                                                       g1.float().contiguous(), mu1, rs1)
                res = spec.has_skip
                dx2, dWe = ext.pw_bwd(dA1.view(M, Ce), y1.view(M, Ce), x.view(M, Cin), _bf(We).reshape(Ce, Cin),
                                      consts.contiguous(), dout.view(M, Cin) if res else None,
                                      fmul.float().contiguous() if res else None, H * W, _pw_bwd_blocks(M))
                dx = dx2.view(N, H, W, Cin)
                dWe = dWe.view_as(We)
                skip_done = res
            else:
                mdz1, mdzx1, dg1, db1 = ext.bn_bwd_finalize_new(pa1, pb1, float(M))
                dy1 = ext.bn_bwd_apply(dA1, None, None, 0, y1, sc1, sh1, mu1, rs1, g1.float().contiguous(), ACT_SILU,
                                       mdz1, mdzx1).view(M, Ce)
                dx = _lin(dy1, _bf(We).reshape(Ce, Cin).t()).view(N, H, W, Cin)
                dWe = wgrad(dy1, x.view(M, Cin), final=True, ok=ctx.needs_input_grad[4]).view_as(We)
        elif in_bn:
            if dy2 is not None:
                dA1, pa1, pb1 = ext.dw_bwd_data(dy2, wd, H, W, k, s, x, sc1, sh1, mu1, rs1, MAX_BLOCKS)
                dWd = ext.dw_bwd_weight(dy2, x, sc1, sh1, ACT_SILU, k, s, _dw_wgrad_blocks(Ce)).view_as(Wd)
            # the stem BN's backward: statistics from the depthwise epilogue, then apply -> grad of the stem conv output
            mdz1, mdzx1, dg1, db1 = ext.bn_bwd_finalize_new(pa1, pb1, float(M))
            if ctx.stem_link is not None:
                # the stem's weight-gradient kernel applies this BN backward while staging (StemPreFn.backward)
                ctx.stem_link.bn = (x, sc1, sh1, mu1, rs1, g1.float().contiguous(), mdz1, mdzx1)
                dx = dA1.view(N, H, W, Cin)
            else:
                dx = ext.bn_bwd_apply(dA1, None, None, 0, x, sc1, sh1, mu1, rs1, g1.float().contiguous(), ACT_SILU,
                                      mdz1, mdzx1).view(N, H, W, Cin)
            dWe = None
        else:
            if dy2 is not None:
                (dx,) = ext.dw_bwd_data(dy2, wd, H, W, k, s, None, None, None, None, None, MAX_BLOCKS)
                dWd = ext.dw_bwd_weight(dy2, x, None, None, ACT_NONE, k, s, _dw_wgrad_blocks(Ce)).view_as(Wd)
            dg1 = db1 = dWe = None
        if spec.has_skip and not skip_done:
            ext.add_scaled_(dx.view(N, HW2, Cout), dout.view(N, HW2, Cout), fmul.float().contiguous())
        _mark(f"bwd{spec.index}_end")
        return (dx, dmul, dadd, None, dWe, dg1, db1, dWd, dg2, db2, df1w, df1b, df2w, df2b, dWp, dg3, db3, None)


def _scalar_zero(device):
    """0-dim zero: the ignored (beta = 0) bias operand of an addmm used as a scaled mm."""
    key = ("z0", str(device))
    hit = _LAYOUT_CACHE.get(key)
    if hit is None:
        hit = torch.zeros((), device=device)
        _LAYOUT_CACHE[key] = hit
    return hit


def _ones_zeros(E: int, device):
    """Constant identity BN / FiLM vectors of the top's block_tail calls (cached: no fill kernels per step)."""
    key = ("oz", E, str(device))
    hit = _LAYOUT_CACHE.get(key)
    if hit is None:
        hit = (torch.ones(E, device=device), torch.zeros(E, device=device))
        _LAYOUT_CACHE[key] = hit
    return hit


def _zeros2(N: int, E: int, device):
    """Cached [N, E] fp32 zeros (the FiLM shift slot of block_tail used as a per-frame row scale)."""
    key = ("z2", N, E, str(device))
    hit = _LAYOUT_CACHE.get(key)
    if hit is None:
        hit = torch.zeros(N, E, device=device)
        _LAYOUT_CACHE[key] = hit
    return hit


class TopFn(torch.autograd.Function):
    """x [N,h,w,384] -> silu(bn(x @ Wt^T)) @ W1^T -> * fmul + fadd   => [N, h*w, 512] bf16."""

    @staticmethod
    def forward(ctx, x, Wt, gt, bt, W1, fmul, fadd, bnc: BNCtx, training: bool):
        ext = _ext()
        N, H, W, Cin = x.shape
        Ct, E = Wt.shape[0], W1.shape[0]
        M = N * H * W
        # BN statistics from the wide GEMM's epilogue (no bn_stats pass over the 1536-wide y)
        y, (sc, sh, mu, rs) = _lin_bn(x.view(M, Cin), _bf(Wt).reshape(Ct, Cin), bnc, training)
        a = ext.bn_apply(y, sc, sh, ACT_SILU, None, 0)
        f = _lin(a, _bf(W1).reshape(E, Ct))        # [M, E]
        ones, zeros = _ones_zeros(E, x.device)
        out = ext.block_tail(f.view(N, H * W, E), ones, zeros, None, None, fmul, fadd)
        ctx.save_for_backward(x, Wt, gt, W1, fmul, y, a, f, sc, sh, mu, rs)
        ctx.shape = (N, H, W, Cin, Ct, E)
        return out

    @staticmethod
    def backward(ctx, dout):
        ext = _ext()
        x, Wt, gt, W1, fmul, y, a, f, sc, sh, mu, rs = ctx.saved_tensors
        N, H, W, Cin, Ct, E = ctx.shape
        M, HW = N * H * W, H * W
        dev = x.device
        dout = dout.contiguous().to(BF)
        ones, zeros = _ones_zeros(E, dev)
        dmul, dadd, _, _ = ext.tail_bwd_reduce(dout.view(N, HW, E), f.view(N, HW, E), ones, zeros, zeros, ones,
                                               None, None, None)
        # df = dout * fmul[frame] as one flat pass (block_tail with identity BN and a zero FiLM shift; bitwise the
        # torch expression, which ran as an fp32 multiply + a bf16 cast: 88 us at b128)
        zeros_ne = _zeros2(N, E, dev)
        df = ext.block_tail(dout.view(N, HW, E), ones, zeros, None, None, fmul.float().contiguous(), zeros_ne).view(M, E)
        W1m = _bf(W1).reshape(E, Ct)
        dW1 = wgrad(df, a, final=True, ok=ctx.needs_input_grad[4]).view_as(W1)
        da = _lin(df, W1m.t())                                                   # [M, Ct]
        pa, pb = ext.bn_bwd_reduce(da, None, None, 0, y, sc, sh, mu, rs, ACT_SILU, _partials(M))
        mdz, mdzx, dg, db = ext.bn_bwd_finalize_new(pa, pb, float(M))
        dy = ext.bn_bwd_apply(da, None, None, 0, y, sc, sh, mu, rs, gt.float().contiguous(), ACT_SILU, mdz, mdzx)
        dWt = wgrad(dy, x.view(M, Cin), final=True, ok=ctx.needs_input_grad[1]).view_as(Wt)
        dx = _lin(dy, _bf(Wt).reshape(Ct, Cin).t()).view(N, H, W, Cin)
        return dx, dWt, dg, db, dW1, dmul, dadd, None, None


class FilmFn(torch.autograd.Function):
    """Every FiLM projection of the encoder (26 block FiLMs + the final one; reference
    ``film_efficientnet/film_conditioning_layer.py:39-51``) as ONE MFMA GEMM: gb = ctx @ W_all^T + b_all, with the "+1"
    of the multiplicative halves and the block-by-block layout in the epilogue (``rt1_gemm_cmap``: each block's
    (1 + gamma) / beta comes out as its own contiguous [N, C] slice of one flat buffer).  The backward reads that
    layout directly (``rt1_wgrad_dymap``: fp32 gradient rounded to bf16 while staged, the bias gradient from the same
    pass in fp32).  Operands: the context in bf16 and the bf16 weight shadow, packed per step by FusedRT1 (as torch
    autocast runs these Linears).  It replaces an fp32 hipBLASLt addmm (64 us), the index_select into the block
    layout and its index_add backward, the fp32 weight-gradient GEMM (60 us) and the bias column sum."""

    @staticmethod
    def forward(ctx, xe, wpack, bpack, cmap, rows, *params):
        ext = _ext()
        out = ext.film_fwd(xe, xe.shape[1], wpack, bpack, cmap, xe.shape[0] * wpack.shape[0], FILM_FWD_CFG)
        ctx.save_for_backward(xe, cmap)
        ctx.rows = rows
        return out

    @staticmethod
    def backward(ctx, g):
        if ctx.needs_input_grad[0]:
            raise NotImplementedError("FilmFn: no gradient for the context embedding (RT-1 feeds a frozen encoder's)")
        xe, cmap = ctx.saved_tensors
        dW, db = _ext().film_wgrad(g.contiguous(), cmap, xe, xe.shape[1], FILM_WGRAD_SPLITS, FILM_WGRAD_TILE)
        nw = len(ctx.rows) // 2
        grads = [dW[r0:r1] for r0, r1 in ctx.rows[:nw]] + [db[r0:r1] for r0, r1 in ctx.rows[nw:]]
        return (None, None, None, None, None, *grads)


# gemm.hip tile config of the forward (128 x 64: 19.6 us vs 21.4-22.9 for the others) and row splits of the weight
# gradient (1: 31.5 us vs 47-55 for 2-4), tools/bench_film.py at 768 frames (profiles/r6_film_bench.log)
FILM_FWD_CFG = 4
FILM_WGRAD_SPLITS = 1
FILM_WGRAD_TILE = 0
_FILM_PACK = {}   # data_ptr(first FiLM weight) -> (wpack bf16 [sum C, 512], bpack fp32 [sum C]), filled per step


def set_film_packs(packs):
    global _FILM_PACK
    _FILM_PACK = packs


def film_params(net, encoder):
    """All FiLM projections (26 block FiLMs + the encoder's final FiLM) as one weight matrix."""
    films = list(net.films) + [encoder.film_layer]
    ws, bs, sizes = [], [], []
    for fl in films:
        ws += [fl._projection_mult.weight, fl._projection_add.weight]
        bs += [fl._projection_mult.bias, fl._projection_add.bias]
        sizes += [fl.num_channels, fl.num_channels]
    return ws, bs, sizes


def encoder_forward(encoder, frames: torch.Tensor, context: Optional[torch.Tensor], shift: Optional[torch.Tensor],
                    training: bool) -> torch.Tensor:
    """FiLM-EfficientNet-B3 + conv1x1 + final FiLM on ``frames`` (N,3,H,W) -> [N, h*w, 512] bf16."""
    net = encoder.net
    N = frames.shape[0]
    stem = net.convNormAct0
    first = net.blocks[0]
    stem_into_block0 = STEM_IN_BLOCK0 and first.expand is None and not first.spec.has_skip
    link = StemLink() if (stem_into_block0 and STEM_BN_BWD_FUSED) else None
    if stem_into_block0:
        x, *stem_consts = StemPreFn.apply(frames, shift, stem[0].weight, BNCtx(stem[1]), training, link)
    else:
        x = StemFn.apply(frames, shift, stem[0].weight, stem[1].weight, stem[1].bias, BNCtx(stem[1]), training)
    # every FiLM gamma/beta of the encoder in ONE GEMM: ctx (N, 512) x W_all^T (512, 2*sum C), with the "+1" of the
    # multiplicative halves folded into the bias; one gather then lays the [N, 2*sum C] product out block by block, so
    # each block's (1 + gamma) and beta are contiguous [N, C] views (it was 27 adds + 54 strided copies per step)
    ws, bs, sizes = film_params(net, encoder)
    xe = (context if context is not None else torch.zeros(N, 512, device=frames.device)).to(BF).contiguous()
    cmap, rows = _film_layout(sizes, N, frames.device)
    pk = _FILM_PACK.get(ws[0].data_ptr())
    wpack, bpack = pk if pk is not None else (torch.cat([_bf(w) for w in ws], 0), torch.cat(bs, 0).float())
    gb = FilmFn.apply(xe, wpack, bpack, cmap, rows, *ws, *bs)
    parts = [c.view(N, n) for c, n in zip(gb.split([n * N for n in sizes]), sizes)]
    keeps = _drop_path_masks(net, N, frames.device) if training else {}
    for i, blk in enumerate(net.blocks):
        sp = blk.spec
        fmul = parts[2 * i]
        fadd = parts[2 * i + 1]
        keep = keeps.get(i)
        e = blk.expand
        dw, se, pj = blk.depthwise, blk.se, blk.project
        bns = ([BNCtx(e[1])] if e is not None else []) + [BNCtx(dw[1]), BNCtx(pj[1])]
        if i == 0 and stem_into_block0:
            # the stem BN's gamma / beta ride in the (absent) expand BN's slots; its constants in meta
            g1_, b1_, meta = stem[1].weight, stem[1].bias, (sp, bns, training, tuple(stem_consts), link)
        else:
            g1_ = e[1].weight if e is not None else None
            b1_ = e[1].bias if e is not None else None
            meta = (sp, bns, training)
        x = MBConvFn.apply(x, fmul, fadd, keep, e[0].weight if e is not None else None, g1_, b1_,
                           dw[0].weight, dw[1].weight, dw[1].bias,
                           se.fc1.weight, se.fc1.bias, se.fc2.weight, se.fc2.bias,
                           pj[0].weight, pj[1].weight, pj[1].bias, meta)
    top = net.convNormAct1
    fmul = parts[-2]
    fadd = parts[-1]
    out = TopFn.apply(x, top[0].weight, top[1].weight, top[1].bias, encoder.conv1x1.weight, fmul, fadd,
                      BNCtx(top[1]), training)
    if training:
        bump_batches_tracked(net)
    return out


_LAYOUT_CACHE = {}


def _film_layout(sizes, N: int, device):
    """Column map of the FiLM GEMM's epilogue (int32 [sum(sizes) / 4, 4]: for each 4-column group the flat offset of
    its first element at row 0, the row stride and the bits of the 1.0 added to the multiplicative halves -- even
    entries of ``sizes``) so the [N, sum(sizes)] product lands as consecutive [N, size] blocks; plus the weight rows of
    each projection (the same list for the biases)."""
    key = (tuple(sizes), N, str(device))
    hit = _LAYOUT_CACHE.get(key)
    if hit is None:
        assert all(n % 8 == 0 for n in sizes), sizes
        one = int(torch.tensor(1.0).view(torch.int32))
        groups, rows, c0, off = [], [], 0, 0
        for j, n in enumerate(sizes):
            for cl in range(0, n, 4):
                groups.append((off + cl, n, one if j % 2 == 0 else 0, 0))
            rows.append((c0, c0 + n))
            c0 += n
            off += n * N
        hit = (torch.tensor(groups, dtype=torch.int32).to(device), tuple(rows) + tuple(rows))
        _LAYOUT_CACHE[key] = hit
    return hit


def _drop_path_masks(net, N: int, device):
    """Per-frame drop-path keep masks (bernoulli(1-p) / (1-p)) of every residual block from ONE uniform draw."""
    # the module's p (what StochasticDepth.keep_mask used; callers may zero it), not the spec's rate
    blocks = [(i, float(blk.dropout.p)) for i, blk in enumerate(net.blocks)
              if blk.spec.has_skip and blk.spec.drop_rate > 0 and blk.dropout.p > 0]
    if not blocks:
        return {}
    key = ("drop", tuple(p for _, p in blocks), str(device))
    kp = _LAYOUT_CACHE.get(key)
    if kp is None:
        kp = torch.tensor([1.0 - p for _, p in blocks], device=device)[:, None]
        _LAYOUT_CACHE[key] = kp
    u = torch.rand(len(blocks), N, device=device)
    keep = (u < kp).float().div_(kp)
    return {i: keep[j] for j, (i, _) in enumerate(blocks)}


def bump_batches_tracked(net):
    """num_batches_tracked += 1 on every BatchNorm of ``net`` in one foreach launch.  The counter list is cached on
    the module itself, so it dies with the module (an id()-keyed global cache kept freed models' tensors alive and
    could hand a dead model's counters to a new model reusing the id)."""
    lst = getattr(net, "_rt1_tracked", None)
    if lst is None:
        lst = [m.num_batches_tracked for m in net.modules()
               if isinstance(m, torch.nn.BatchNorm2d) and m.num_batches_tracked is not None]
        object.__setattr__(net, "_rt1_tracked", lst)
    torch._foreach_add_(lst, 1)
