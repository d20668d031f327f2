"""Skinny MFMA pointwise-conv GEMM (csrc/kernels/pwgemm.hip) vs an fp32 PyTorch reference (MI355X only)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

BF = torch.bfloat16
# every (K, N) of the B3 high-resolution 1x1 convs in both orientations, plus odd M tails
SHAPES = [(40, 24), (24, 40), (24, 24), (24, 144), (144, 24), (144, 32), (32, 144), (32, 192), (192, 32),
          (192, 48), (48, 192), (48, 288), (288, 48)]


@pytest.fixture(scope="module")
def ext():
    from pytorch_rt1_for_distributed_training_amd import ops
    return ops.load()


@pytest.mark.parametrize("K,N", SHAPES)
@pytest.mark.parametrize("M", [1, 37, 1000, 4099])
def test_pw_gemm_matches_fp32(ext, K, N, M):
    assert ext.pw_gemm_supported(K, N)
    torch.manual_seed(K * 1000 + N + M)
    a = torch.randn(M, K, device="cuda").to(BF)
    # asymmetric, non-constant weights so a transposed / mis-indexed store cannot pass
    b = (torch.randn(N, K, device="cuda") + torch.arange(N, device="cuda")[:, None] * 0.01).to(BF)
    c = ext.pw_gemm(a, b, 2048)[0]
    ref = a.float() @ b.float().t()
    assert c.shape == (M, N) and c.dtype == BF
    err = (c.float() - ref).norm() / ref.norm()
    assert err < 6e-3, float(err)


def test_pw_gemm_grid_stride(ext):
    """few workgroups: every wave walks many strips (prefetch path)"""
    torch.manual_seed(0)
    a = torch.randn(50000, 24, device="cuda").to(BF)
    b = torch.randn(144, 24, device="cuda").to(BF)
    c = ext.pw_gemm(a, b, 3)[0]
    ref = a.float() @ b.float().t()
    assert (c.float() - ref).norm() / ref.norm() < 6e-3


@pytest.mark.parametrize("K,N", [(40, 24), (24, 144), (192, 32), (48, 288), (288, 48)])
def test_pw_gemm_bn_stat_epilogue(ext, K, N):
    torch.manual_seed(1)
    M = 5003
    a = torch.randn(M, K, device="cuda").to(BF)
    b = (torch.randn(N, K, device="cuda") * 0.2 + 0.05).to(BF)
    c, ps, pq = ext.pw_gemm(a, b, 64, True)
    assert torch.equal(c, ext.pw_gemm(a, b, 64)[0])
    cf = c.float()
    torch.testing.assert_close(ps.sum(0), cf.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(pq.sum(0), (cf * cf).sum(0), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("K,N,hw,frames,mb", [(40, 24, 150, 5, 64), (24, 24, 130, 7, 3), (144, 32, 5625 // 25, 9, 64),
                                               (192, 32, 361, 6, 2048), (192, 48, 1444 // 4, 5, 16),
                                               (288, 48, 1444, 3, 64)])
def test_pw_gemm_project_prologue(ext, K, N, hw, frames, mb):
    """operand prologue: pw_gemm(y, W, scale, shift, gate, hw) == pw_gemm(bn_apply(y, scale, shift, SiLU, gate), W)
    bit for bit (same formula and rounding), BN partials included, and both close to the fp32 reference."""
    torch.manual_seed(K + N + hw)
    M = hw * frames
    y = (torch.randn(M, K, device="cuda") * 1.5).to(BF)
    w = (torch.randn(N, K, device="cuda") * 0.2 + torch.arange(N, device="cuda")[:, None] * 0.01).to(BF)
    sc, sh = torch.rand(K, device="cuda") + 0.5, torch.randn(K, device="cuda") * 0.3
    gate = torch.rand(frames, K, device="cuda")
    a = ext.bn_apply(y, sc, sh, 1, gate, hw)
    c0, ps0, pq0 = ext.pw_gemm(a, w, mb, True)
    c1, ps1, pq1 = ext.pw_gemm(y, w, mb, True, sc, sh, gate, hw)
    assert torch.equal(c0, c1)
    assert torch.equal(ps0, ps1) and torch.equal(pq0, pq1)
    assert torch.equal(ext.pw_gemm(y, w, mb, False, sc, sh, gate, hw)[0], c1)
    c2, ps2, pq2, a2 = ext.pw_gemm(y, w, mb, True, sc, sh, gate, hw, True)      # + the stored operand
    assert torch.equal(c2, c1) and torch.equal(ps2, ps1) and torch.equal(a2, a)
    af = torch.nn.functional.silu(y.float() * sc + sh) * gate.repeat_interleave(hw, 0)
    ref = af @ w.float().t()
    assert float((c1.float() - ref).norm() / ref.norm()) < 1e-2


@pytest.mark.parametrize("CE,CIN", [(144, 24), (192, 32), (288, 48)])
@pytest.mark.parametrize("M,skip", [(4099, False), (3000, True), (64, False)])
def test_pw_bwd_fused_expand_backward(ext, CE, CIN, M, skip):
    """pwbwd.hip: SiLU + BN backward prologue, dgrad and wgrad of the expand conv in one kernel."""
    assert ext.pw_bwd_supported(CE, CIN)
    torch.manual_seed(CE + M)
    dA = torch.randn(M, CE, device="cuda").to(BF)
    y = (torch.randn(M, CE, device="cuda") * 2 + 0.3).to(BF)
    x = torch.randn(M, CIN, device="cuda").to(BF)
    We = (torch.randn(CE, CIN, device="cuda") * 0.2).to(BF)
    sc, sh = torch.rand(CE, device="cuda") + 0.5, torch.randn(CE, device="cuda") * 0.3
    k1, k2, k0 = torch.rand(CE, device="cuda") + 0.2, torch.randn(CE, device="cuda") * 0.1, torch.randn(CE, device="cuda") * 0.1
    consts = torch.stack([sc, sh, k1, k2, k0]).contiguous()
    HW = 1000 if skip else 1
    dout = torch.randn(M, CIN, device="cuda").to(BF) if skip else None
    fmul = torch.randn(M // HW, CIN, device="cuda") if skip else None
    dx, dWe = ext.pw_bwd(dA, y, x, We, consts, dout, fmul, HW, 64)
    u = y.float() * sc + sh
    s = torch.sigmoid(u)
    dz = dA.float() * s * (1 + u * (1 - s))
    dy = (k1 * dz + k2 * y.float() + k0).to(BF).float()
    dx_ref = dy @ We.float()
    if skip:
        dx_ref = dx_ref + dout.float() * fmul.repeat_interleave(HW, 0)
    dWe_ref = dy.t() @ x.float()
    assert dx.shape == (M, CIN) and dWe.shape == (CE, CIN)
    assert float((dx.float() - dx_ref).norm() / dx_ref.norm()) < 8e-3
    assert float((dWe - dWe_ref).norm() / dWe_ref.norm()) < 2e-3


@pytest.mark.parametrize("CE,CIN", [(144, 24), (192, 32), (288, 48)])
@pytest.mark.parametrize("M,skip", [(4099, False), (3000, True), (64, False), (70001, False)])
def test_pw_bwd_z_matches_fp32(ext, CE, CIN, M, skip):
    """pwbwd.hip pw_bwd_z: the expand backward from (dz, x) only -- dy1 = k1*dz + k2*(x @ We^T) + k0 rewritten as
    (k1*dz) @ We + x @ Mk + r0 and diag(k1) dz^T x + diag(k2) We G + k0 sx^T -- vs the fp32 chain.  x has a non-zero
    mean so the G / sx terms are large and cancel against the dz term."""
    assert ext.pw_bwd_supported(CE, CIN)
    torch.manual_seed(CE + M + 1)
    dz = torch.randn(M, CE, device="cuda").to(BF)
    x = (torch.randn(M, CIN, device="cuda") + 0.5).to(BF)
    We = (torch.randn(CE, CIN, device="cuda") * 0.2).to(BF)
    sc, sh = torch.rand(CE, device="cuda") + 0.5, torch.randn(CE, device="cuda") * 0.3
    k1, k2, k0 = torch.rand(CE, device="cuda") + 0.2, torch.randn(CE, device="cuda") * 0.1, torch.randn(CE, device="cuda") * 0.1
    consts = torch.stack([sc, sh, k1, k2, k0]).contiguous()
    HW = 1000 if skip else 1
    dout = torch.randn(M, CIN, device="cuda").to(BF) if skip else None
    fmul = torch.randn(M // HW, CIN, device="cuda") if skip else None
    dx, dWe = ext.pw_bwd_z(dz, x, We, consts, dout, fmul, HW, 64)
    y1 = x.float() @ We.float().t()
    dy = k1 * dz.float() + k2 * y1 + k0
    dx_ref = dy @ We.float()
    if skip:
        dx_ref = dx_ref + dout.float() * fmul.repeat_interleave(HW, 0)
    dWe_ref = dy.t() @ x.float()
    assert dx.shape == (M, CIN) and dWe.shape == (CE, CIN)
    assert float((dx.float() - dx_ref).norm() / dx_ref.norm()) < 8e-3
    assert float((dWe - dWe_ref).norm() / dWe_ref.norm()) < 3e-3


@pytest.mark.parametrize("CE,CIN,M", [(576, 96, 5000), (816, 136, 3001), (576, 96, 70001), (816, 136, 4096)])
def test_expand_bwd_z_wide_matches_fp32(ext, CE, CIN, M):
    """ops.backbone.expand_bwd_z_wide (pw_z_prep, MFMA wgrad for Mk / G / dz^T x, pw_tall_tail, pw_z_finish) vs the
    fp32 expand backward chain."""
    from pytorch_rt1_for_distributed_training_amd.ops.backbone import expand_bwd_z_wide
    torch.manual_seed(CE + M)
    dz = torch.randn(M, CE, device="cuda").to(BF)
    x = (torch.randn(M, CIN, device="cuda") + 0.3).to(BF)
    We = (torch.randn(CE, CIN, device="cuda") * 0.1).to(BF)
    sc, sh = torch.rand(CE, device="cuda") + 0.5, torch.randn(CE, device="cuda") * 0.3
    k1, k2, k0 = torch.rand(CE, device="cuda") + 0.2, torch.randn(CE, device="cuda") * 0.1, torch.randn(CE, device="cuda") * 0.1
    consts = torch.stack([sc, sh, k1, k2, k0]).contiguous()
    dx, dWe = expand_bwd_z_wide(dz, x, We, consts)
    y1 = x.float() @ We.float().t()
    dy = k1 * dz.float() + k2 * y1 + k0
    dx_ref = dy @ We.float()
    dWe_ref = dy.t() @ x.float()
    assert dx.shape == (M, CIN) and dWe.shape == (CE, CIN)
    assert float((dx.float() - dx_ref).norm() / dx_ref.norm()) < 1e-2
    assert float((dWe - dWe_ref).norm() / dWe_ref.norm()) < 3e-3


@pytest.mark.parametrize("CE,CIN", [(576, 96), (816, 136), (1392, 232), (2304, 384), (200, 30), (64, 33)])
def test_pw_z_prep_matches_fp32(ext, CE, CIN):
    """pwbwd.hip pw_z_prep (one launch): Wt = (diag(k1) We)^T, Mk = We^T diag(k2) We (bf16), r0 = k0 @ We (fp32)
    against fp64 PyTorch on the same bf16 weights; odd CIN (scalar loads, partial 32 x 32 tiles) included; Mk bitwise
    reproducible (fixed slice order)."""
    torch.manual_seed(CE + CIN)
    We = (torch.randn(CE, CIN, device="cuda") * CIN ** -0.5).to(BF)
    consts = torch.randn(5, CE, device="cuda")
    wt, mk, r0 = ext.pw_z_prep(We, consts.view(-1))
    W = We.double()
    k1, k2, k0 = consts[2].double(), consts[3].double(), consts[4].double()
    torch.testing.assert_close(wt.double(), (W * k1[:, None]).t(), rtol=1e-2, atol=1e-3)
    mk_ref = W.t() @ (W * k2[:, None])
    torch.testing.assert_close(mk.double(), mk_ref, rtol=1e-2, atol=1e-2 * mk_ref.abs().max().item())
    r0_ref = k0 @ W
    torch.testing.assert_close(r0.double(), r0_ref, rtol=1e-4, atol=1e-4 * r0_ref.abs().max().item())
    again = ext.pw_z_prep(We, consts.view(-1))
    assert torch.equal(again[1], mk) and torch.equal(again[2], r0) and torch.equal(again[0], wt)


@pytest.mark.parametrize("M,K,N,K2", [(5003, 576, 96, 96), (4099, 816, 136, 136), (300, 816, 136, 136),
                                     (3600, 576, 96, 96)])
def test_pw_tall_tail_matches_fp32(ext, M, K, N, K2):
    """pwtall.hip second reduction segment: A @ W^T + A2 @ W2^T + bias."""
    torch.manual_seed(M + K)
    a = torch.randn(M, K, device="cuda").to(BF)
    w = (torch.randn(N, K, device="cuda") * 0.1).to(BF)
    a2 = torch.randn(M, K2, device="cuda").to(BF)
    w2 = (torch.randn(N, K2, device="cuda") * 0.1).to(BF)
    bias = torch.randn(N, device="cuda")
    c = ext.pw_tall_tail(a, w, a2, w2, bias)
    ref = a.float() @ w.float().t() + a2.float() @ w2.float().t() + bias
    assert float((c.float() - ref).norm() / ref.norm()) < 6e-3
    if M % 100 == 0:                                   # + residual epilogue (frames of 100 rows)
        res = torch.randn(M, N, device="cuda").to(BF)
        rmul = torch.randn(M // 100, N, device="cuda")
        c2 = ext.pw_tall_tail(a, w, a2, w2, bias, res, rmul, 100)
        ref2 = ref + res.float() * rmul.repeat_interleave(100, 0)
        assert float((c2.float() - ref2).norm() / ref2.norm()) < 6e-3


@pytest.mark.parametrize("K,N", [(96, 576), (136, 816), (232, 1392), (384, 2304), (384, 1536), (96, 288)])
@pytest.mark.parametrize("M", [37, 3001])
def test_pw_wide_matches_fp32(ext, K, N, M):
    """wide-N MFMA GEMM (mid-resolution 1x1 convs) vs fp32; includes partial 64-column chunks (816, 1392)."""
    assert ext.pw_gemm_supported(K, N)
    torch.manual_seed(K + N + M)
    a = torch.randn(M, K, device="cuda").to(BF)
    b = (torch.randn(N, K, device="cuda") + torch.arange(N, device="cuda")[:, None] * 0.01).to(BF)
    c = ext.pw_gemm(a, b, 64)[0]
    ref = a.float() @ b.float().t()
    assert c.shape == (M, N)
    assert float((c.float() - ref).norm() / ref.norm()) < 6e-3


@pytest.mark.parametrize("M,K,N", [(5003, 576, 96), (4099, 816, 136), (3001, 1392, 232), (2053, 2304, 384),
                                   (4096, 288, 96), (777, 1536, 384), (1000, 256, 16), (1500, 520, 200)])
def test_pw_tall_matches_fp32(ext, M, K, N):
    """pwtall.hip: wide-K / narrow-N MFMA GEMM incl. K tails (816, 520), N tails (136, 232, 200) and M tails."""
    assert ext.pw_tall_supported(K, N)
    torch.manual_seed(M + K + N)
    a = torch.randn(M, K, device="cuda").to(BF)
    b = (torch.randn(N, K, device="cuda") + torch.arange(N, device="cuda")[:, None] * 0.01).to(BF)
    c = ext.pw_tall(a, b)[0]
    ref = a.float() @ b.float().t()
    assert c.shape == (M, N) and c.dtype == BF
    err = (c.float() - ref).norm() / ref.norm()
    assert err < 6e-3, float(err)
    # per-row check: a dropped K chunk or mis-stored column shows up in some row even if the global norm hides it
    rerr = ((c.float() - ref).norm(dim=1) / ref.norm(dim=1)).max()
    assert rerr < 2e-2, float(rerr)


def test_pw_tall_rejects_unsupported(ext):
    assert not ext.pw_tall_supported(96, 576)      # narrow K: the skinny/wide kernels' job
    assert not ext.pw_tall_supported(1536, 512)    # N > 384
    assert not ext.pw_tall_supported(300, 96)      # K % 8


@pytest.mark.parametrize("frames,HW,K,N", [(16, 361, 576, 96), (12, 361, 816, 136), (9, 1444, 288, 96),
                                          (40, 100, 1392, 232), (7, 100, 520, 200)])
def test_pw_tall_operand_prologue(ext, frames, HW, K, N):
    """pw_tall with the project-conv operand prologue a = silu(y*scale+shift)*gate[frame] (and its stored copy)
    is bit-identical to bn_apply followed by the plain pw_tall."""
    torch.manual_seed(K + N)
    M = frames * HW
    y = torch.randn(M, K, device="cuda").to(BF)
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(BF)
    sc, sh = torch.rand(K, device="cuda") + 0.5, torch.randn(K, device="cuda") * 0.3
    gate = torch.rand(frames, K, device="cuda")
    c, a = ext.pw_tall(y, w, sc, sh, gate, HW, True)
    a_ref = ext.bn_apply(y, sc, sh, 1, gate, HW)
    assert torch.equal(a, a_ref.view(M, K))
    assert torch.equal(c, ext.pw_tall(a_ref.view(M, K), w)[0])
    (c2,) = ext.pw_tall(y, w, sc, sh, gate, HW, False)
    assert torch.equal(c2, c)


@pytest.mark.parametrize("K,N", [(24, 40), (24, 24), (32, 144), (32, 192), (48, 192), (48, 288)])
@pytest.mark.parametrize("with_keep", [False, True])
def test_pw_gemm_bnbwd_equals_apply_then_gemm(ext, K, N, with_keep):
    """Project data gradient with the BN3 backward in the operand prologue == bn_bwd_apply then the plain skinny
    GEMM, bit for bit (dA and the stored dy3), including a drop-path mask and frames straddling strips (the wide
    form for blocks 9-17 was measured slower and removed: profiles/r5_pw_wide_bnbwd_ab.log)."""
    assert ext.pw_gemm_bnbwd_supported(K, N)
    torch.manual_seed(K * 7 + N)
    frames, hw = 13, 121
    M = frames * hw
    dout = torch.randn(M, K, device="cuda").to(BF)
    y3 = torch.randn(M, K, device="cuda").to(BF)
    W = torch.randn(N, K, device="cuda").to(BF)
    fmul = torch.rand(frames, K, device="cuda") + 0.5
    keep = ((torch.rand(frames, device="cuda") > 0.3).float() / 0.7) if with_keep else None
    gamma, mean = torch.rand(K, device="cuda") + 0.5, torch.randn(K, device="cuda") * 0.1
    rstd, mdz, mdzx = torch.rand(K, device="cuda") + 0.5, torch.randn(K, device="cuda") * 0.1, torch.randn(K, device="cuda") * 0.1
    sc, sh = torch.ones(K, device="cuda"), torch.zeros(K, device="cuda")
    dA, dy3 = ext.pw_gemm_bnbwd(dout, y3, W, fmul, keep, hw, gamma, mean, rstd, mdz, mdzx, 2048)
    rs = (fmul * keep[:, None]).contiguous() if with_keep else fmul
    ref_dy = ext.bn_bwd_apply(dout, rs, None, hw, y3, sc, sh, mean, rstd, gamma, 0, mdz, mdzx)
    ref_dA = ext.pw_gemm(ref_dy, W, 2048)[0]
    assert torch.equal(dy3, ref_dy)
    assert torch.equal(dA, ref_dA)


@pytest.mark.parametrize("CE,CIN", [(576, 96), (1392, 232), (200, 33), (64, 70)])
def test_pw_z_finish_matches_fp64(ext, CE, CIN):
    """pw_z_finish: dWe = k1 S + k2 We G + k0 sx against fp64, partial 32 x 32 tiles and a cj tail
    included; bitwise reproducible."""
    torch.manual_seed(CE * 3 + CIN)
    S = torch.randn(CE, CIN, device="cuda")
    G = torch.randn(CIN, CIN, device="cuda") * 4.0
    sx = torch.randn(CIN, device="cuda") * 10.0
    We = (torch.randn(CE, CIN, device="cuda") * CIN ** -0.5).to(BF)
    consts = torch.randn(5, CE, device="cuda")
    out = ext.pw_z_finish(S, G, sx, We, consts.view(-1))
    k1, k2, k0 = consts[2].double(), consts[3].double(), consts[4].double()
    ref = k1[:, None] * S.double() + k2[:, None] * (We.double() @ G.double()) + k0[:, None] * sx.double()[None]
    torch.testing.assert_close(out.double(), ref, rtol=1e-4, atol=1e-4 * ref.abs().max().item())
    assert torch.equal(ext.pw_z_finish(S, G, sx, We, consts.view(-1)), out)


@pytest.mark.parametrize("splits", [1, 3, 16])
def test_pw_z_finish_sums_split_partials(ext, splits):
    """pw_z_finish on the wgrad kernel's [splits, CE, CIN] partials (ops/backbone.py wgrad(raw=True)) equals the
    call on their fp32 sum up to summation order."""
    CE, CIN = 816, 136
    torch.manual_seed(splits)
    parts = torch.randn(splits, CE, CIN, device="cuda")
    G = torch.randn(CIN, CIN, device="cuda")
    sx = torch.randn(CIN, device="cuda")
    We = (torch.randn(CE, CIN, device="cuda") * CIN ** -0.5).to(BF)
    consts = torch.randn(5 * CE, device="cuda")
    out = ext.pw_z_finish(parts, G, sx, We, consts)
    ref = ext.pw_z_finish(parts.double().sum(0).float(), G, sx, We, consts)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
