"""y1-free expand blocks ("x-mode"): the depthwise kernels recompute y1 = x @ We^T on MFMA per staged tile, and BN1's
batch statistics come from x's Gram matrix.  Checked against the stored-y1 kernels (same math with y1 materialised)
and plain fp32 PyTorch (MI355X only)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

BF = torch.bfloat16

# (Cin, Ce, k, s): the x-mode shapes of FiLM-EfficientNet-B3 (blocks 2, 3-4, 5, 6-7, 8)
SHAPES = [(24, 144, 3, 2), (32, 192, 3, 1), (32, 192, 5, 2), (48, 288, 5, 1), (48, 288, 3, 2)]


@pytest.fixture(scope="module")
def ext():
    from pytorch_rt1_for_distributed_training_amd import ops
    return ops.load()


def rel_err(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-12))


def _inputs(Cin, Ce, N, H, W, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = (torch.randn(N, H, W, Cin, device="cuda", generator=g) + 0.3).to(BF)
    we = (torch.randn(Ce, Cin, device="cuda", generator=g) * Cin ** -0.5).to(BF)
    y1 = (x.float().view(-1, Cin) @ we.float().t()).to(BF).view(N, H, W, Ce)
    return x, we, y1


@pytest.mark.parametrize("Cin,Ce,k,s", SHAPES)
@pytest.mark.parametrize("N,H,W,mb", [(3, 19, 23, 64), (2, 38, 38, 2048), (1, 75, 75, 16)])
def test_dw_fwd_x_matches_stored_y1(ext, Cin, Ce, k, s, N, H, W, mb):
    assert ext.dw_x_supported(Cin, Ce, k, s)
    x, we, y1 = _inputs(Cin, Ce, N, H, W)
    w = torch.randn(Ce, k * k, device="cuda") * 0.3
    sc1, sh1 = torch.rand(Ce, device="cuda") + 0.5, torch.randn(Ce, device="cuda") * 0.2
    out_x, ps_x, pq_x = ext.dw_fwd_x(x, we, w, sc1, sh1, k, s, mb)
    out_r, ps_r, pq_r = ext.dw_fwd(y1, w, sc1, sh1, 1, k, s, mb)
    assert out_x.shape == out_r.shape
    # y1 from MFMA vs from torch's GEMM: a few elements may round to the neighbouring bf16
    assert rel_err(out_x, out_r) < 2e-3
    torch.testing.assert_close(ps_x.sum(0), ps_r.sum(0), rtol=2e-3, atol=2e-2)
    torch.testing.assert_close(pq_x.sum(0), pq_r.sum(0), rtol=2e-3, atol=2e-2)
    # fp32 reference of the whole chain
    a = F.silu(y1.float() * sc1 + sh1).permute(0, 3, 1, 2)
    ref = F.conv2d(a, w.view(Ce, 1, k, k), stride=s, padding=(k - 1) // 2, groups=Ce)
    assert rel_err(out_x.permute(0, 3, 1, 2), ref) < 1e-2


@pytest.mark.parametrize("Cin,Ce,k,s", SHAPES)
@pytest.mark.parametrize("N,H,W,mb", [(3, 19, 23, 64), (2, 38, 38, 2048), (1, 76, 76, 8)])
def test_dw_bwd_fused_x_matches_stored_y1(ext, Cin, Ce, k, s, N, H, W, mb):
    torch.manual_seed(1)
    dev = "cuda"
    x, we, y1 = _inputs(Cin, Ce, N, H, W, seed=1)
    p = (k - 1) // 2
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    C = Ce
    dA = torch.randn(N, Ho, Wo, C, device=dev).to(BF)
    y2 = (torch.randn(N, Ho, Wo, C, device=dev) * 1.5).to(BF)
    gate, rb = torch.rand(N, C, device=dev), torch.randn(N, C, device=dev) * 0.1
    sc2, sh2 = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.2
    mu2, rs2, g2 = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5, torch.rand(C, device=dev) + 0.5
    mdz2, mdzx2 = torch.randn(C, device=dev) * 0.05, torch.randn(C, device=dev) * 0.05
    w = torch.randn(C, k * k, device=dev) * 0.3
    sc1, sh1 = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.2
    mu1, rs1 = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
    rx = ext.dw_bwd_fused_x(dA, y2, gate, rb, sc2, sh2, mu2, rs2, g2, mdz2, mdzx2, w, k, x, we, sc1, sh1, mu1, rs1, mb,
                            True)
    rr = ext.dw_bwd_fused(dA, y2, gate, rb, sc2, sh2, mu2, rs2, g2, mdz2, mdzx2, w, k, y1, sc1, sh1, 1, mu1, rs1, mb,
                          -1 if s == 2 else 1, zout=True)
    assert rx[0].shape == (N, H, W, C)
    assert rel_err(rx[0], rr[0]) < 2e-3
    assert rel_err(rx[1], rr[1]) < 2e-3
    torch.testing.assert_close(rx[2].sum(0), rr[2].sum(0), rtol=1e-2, atol=1e-1)
    torch.testing.assert_close(rx[3].sum(0), rr[3].sum(0), rtol=1e-2, atol=1e-1)


@pytest.mark.parametrize("Cin,M", [(24, 200_003), (32, 4_096), (48, 77_777), (64, 1_000)])
def test_xgram(ext, Cin, M):
    """G = x^T x and sum x in one pass (fp64 output) vs fp64 torch."""
    torch.manual_seed(Cin)
    x = (torch.randn(M, Cin, device="cuda") + torch.rand(Cin, device="cuda")).to(BF)
    out = ext.xgram(x)
    xd = x.double()
    torch.testing.assert_close(out[:Cin * Cin].view(Cin, Cin), xd.t() @ xd, rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(out[Cin * Cin:], xd.sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("Cin,Ce", [(24, 144), (32, 192), (48, 288)])
@pytest.mark.parametrize("offset", [0.0, 2.0])
def test_x_bn_stats(ext, Cin, Ce, offset):
    """BN1 batch statistics (and the running-stat update) from x's Gram moments vs the statistics of y1 itself."""
    torch.manual_seed(Cin)
    M = 200_000
    x = (torch.randn(M, Cin, device="cuda") * 0.7 + offset + torch.rand(Cin, device="cuda")).to(BF)
    we = (torch.randn(Ce, Cin, device="cuda") * Cin ** -0.5).to(BF)
    gamma, beta = torch.rand(Ce, device="cuda") + 0.5, torch.randn(Ce, device="cuda") * 0.1
    rm, rv = torch.zeros(Ce, device="cuda"), torch.ones(Ce, device="cuda")
    sc, sh, mu, rs = ext.x_bn_stats(x, we, gamma, beta, 1e-5, 0.1, rm, rv)
    y = x.double() @ we.double().t()
    mean, var = y.mean(0), y.var(0, unbiased=False)
    torch.testing.assert_close(mu.double(), mean, rtol=1e-5, atol=1e-5 * float(var.sqrt().mean()))
    torch.testing.assert_close((1.0 / rs.double() ** 2 - 1e-5), var, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(sc.double(), gamma.double() / (var + 1e-5).sqrt(), rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(sh.double(), beta.double() - mean * sc.double(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(rm.double(), 0.1 * mean, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(rv.double(), 0.9 + 0.1 * var * M / (M - 1), rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("Cin,Ce,M", [(96, 576, 277_248), (136, 816, 277_248), (232, 1392, 76_800), (384, 2304, 76_800),
                                        (64, 20, 5_000)])
@pytest.mark.parametrize("offset", [0.0, 1.5])
def test_bn_from_gram_wide(ext, Cin, Ce, M, offset):
    """BN1 of the wide expand convs from (wgrad(x, x), colsum(x)) in fp32 (ops/backbone.py GRAM_BN) vs the statistics
    of y1 itself, at the real row counts (768 frames at 19x19 / 10x10)."""
    from pytorch_rt1_for_distributed_training_amd.ops import backbone
    torch.manual_seed(Cin + M)
    x = (torch.randn(M, Cin, device="cuda") * 0.7 + offset + torch.rand(Cin, device="cuda")).to(BF)
    we = (torch.randn(Ce, Cin, device="cuda") * Cin ** -0.5).to(BF)
    gamma, beta = torch.rand(Ce, device="cuda") + 0.5, torch.randn(Ce, device="cuda") * 0.1
    rm, rv = torch.zeros(Ce, device="cuda"), torch.ones(Ce, device="cuda")
    if Ce >= 576 and Cin <= 232:
        assert backbone.gram_bn_preferred(Cin, Ce)          # the step's wide blocks take this path
    G, sx = backbone.gram_moments(x)
    sc, sh, mu, rs = ext.bn_from_gram(G, sx, we, float(M), gamma, beta, 1e-5, 0.1, rm, rv)
    y = x.double() @ we.double().t()
    mean, var = y.mean(0), y.var(0, unbiased=False)
    torch.testing.assert_close(mu.double(), mean, rtol=1e-4, atol=1e-4 * float(var.sqrt().mean()))
    torch.testing.assert_close((1.0 / rs.double() ** 2 - 1e-5), var, rtol=2e-3, atol=1e-5)
    torch.testing.assert_close(sc.double(), gamma.double() / (var + 1e-5).sqrt(), rtol=1e-3, atol=1e-6)
    torch.testing.assert_close(rm.double(), 0.1 * mean, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(rv.double(), 0.9 + 0.1 * var * M / (M - 1), rtol=1e-3, atol=1e-6)


@pytest.mark.parametrize("C,M,variant,splits", [(96, 277_248, 1, 256), (136, 277_248, 1, 128), (232, 76_800, 1, 64),
                                                (232, 76_800, -1, 0), (64, 5_000, 0, 3), (128, 1_000, 2, 1),
                                                (256, 70_001, 3, 16)])
def test_gram_one_pass(ext, C, M, variant, splits):
    """ext.gram: G = x^T x and sx = sum x from one wgrad pass (the first ci tile's workgroups sum the rows they stage)
    and one fixed-order split sum, vs fp64 torch; several ci tiles per row (C > tile width) and odd row counts."""
    torch.manual_seed(C + M)
    x = (torch.randn(M, C, device="cuda") * 0.7 + torch.rand(C, device="cuda")).to(BF)
    G, sx = ext.gram(x, variant, splits)
    xd = x.double()
    torch.testing.assert_close(G.double(), xd.t() @ xd, rtol=1e-5, atol=1e-5 * M)
    torch.testing.assert_close(sx.double(), xd.sum(0), rtol=1e-5, atol=1e-5 * M ** 0.5)
    # the same numbers the two-launch path (wgrad + colsum) gives, to fp32 summation-order differences
    torch.testing.assert_close(G, ext.wgrad(x, x, variant=variant, splits=splits), rtol=1e-5, atol=1e-5 * M ** 0.5)


def test_mbconv_xmode_vs_stored(ext, monkeypatch):
    """MBConvFn of blocks 2-8 with x-mode on and off: same outputs, gradients and running statistics (the only
    difference is fp32 vs bf16-tensor BN1 statistics and MFMA vs library y1 rounding)."""
    import copy
    from pytorch_rt1_for_distributed_training_amd.models.efficientnet import FiLMEfficientNet
    from pytorch_rt1_for_distributed_training_amd.ops import backbone
    from pytorch_rt1_for_distributed_training_amd.ops.backbone import BNCtx, MBConvFn
    torch.manual_seed(0)
    net = FiLMEfficientNet().cuda().train()
    N = 6
    shapes = {2: (24, 60, 60), 3: (32, 30, 30), 5: (32, 30, 30), 6: (48, 15, 15), 8: (48, 15, 15)}
    for i, (cin, H, W) in shapes.items():
        blk = net.blocks[i]
        sp = blk.spec
        assert blk.expand is not None and sp.in_ch == cin
        x = (torch.randn(N, H, W, cin, device="cuda") + 0.2).to(BF)
        fmul = torch.rand(N, sp.out_ch, device="cuda") + 0.5
        fadd = torch.randn(N, sp.out_ch, device="cuda") * 0.1
        g = None
        outs = []
        monkeypatch.setattr(backbone, "XMODE_SHAPES", None)           # every supported block
        for xm in (True, False):
            monkeypatch.setattr(backbone, "XMODE", xm)
            b = copy.deepcopy(blk)
            e, dw, se, pj = b.expand, b.depthwise, b.se, b.project
            bns = [BNCtx(e[1]), BNCtx(dw[1]), BNCtx(pj[1])]
            xf = x.clone().requires_grad_(True)
            out = MBConvFn.apply(xf, fmul, fadd, None, e[0].weight, e[1].weight, e[1].bias, dw[0].weight, dw[1].weight,
                                 dw[1].bias, se.fc1.weight, se.fc1.bias, se.fc2.weight, se.fc2.bias, pj[0].weight,
                                 pj[1].weight, pj[1].bias, (sp, bns, True))
            if g is None:
                g = torch.randn_like(out.float()).to(BF)
            grads = torch.autograd.grad(out, [xf, e[0].weight, e[1].weight, e[1].bias, dw[0].weight, pj[0].weight], g)
            outs.append((out, grads, e[1].running_mean.clone(), e[1].running_var.clone()))
        (o1, g1, m1, v1), (o0, g0, m0, v0) = outs
        assert rel_err(o1, o0) < 1e-2, i
        for a, b_ in zip(g1, g0):
            assert rel_err(a, b_) < 2e-2, i
        torch.testing.assert_close(m1, m0, rtol=1e-3, atol=1e-4)
        torch.testing.assert_close(v1, v0, rtol=1e-2, atol=1e-4)


def test_block2_xmode_pair_at_bench_resolution(ext):
    """Block 2's y1-free stride-2 pair (Cin 24 -> Ce 144, k3 s2) at the REAL 150x150 input of the 300x300 bench, with
    the production grid cap (backbone.XMODE_BLOCKS): forward and fused backward against the stored-y1 kernels and
    the forward against fp32 PyTorch."""
    from pytorch_rt1_for_distributed_training_amd.ops import backbone
    Cin, Ce, k, s = 24, 144, 3, 2
    N, H, W, mb = 6, 150, 150, backbone.XMODE_BLOCKS
    x, we, y1 = _inputs(Cin, Ce, N, H, W, seed=4)
    w = torch.randn(Ce, k * k, device="cuda") * 0.3
    sc1, sh1 = torch.rand(Ce, device="cuda") + 0.5, torch.randn(Ce, device="cuda") * 0.2
    out_x, ps_x, pq_x = ext.dw_fwd_x(x, we, w, sc1, sh1, k, s, mb)
    out_r, ps_r, pq_r = ext.dw_fwd(y1, w, sc1, sh1, 1, k, s, mb)
    assert out_x.shape == (N, 75, 75, Ce)
    assert rel_err(out_x, out_r) < 2e-3
    torch.testing.assert_close(ps_x.sum(0), ps_r.sum(0), rtol=2e-3, atol=5e-2)
    torch.testing.assert_close(pq_x.sum(0), pq_r.sum(0), rtol=2e-3, atol=5e-2)
    a = F.silu(y1.float() * sc1 + sh1).permute(0, 3, 1, 2)
    ref = F.conv2d(a, w.view(Ce, 1, k, k), stride=s, padding=1, groups=Ce)
    assert rel_err(out_x.permute(0, 3, 1, 2), ref) < 1e-2
    # fused backward (dz-mode, as the step runs it)
    dev = "cuda"
    C, Ho, Wo = Ce, 75, 75
    dA = torch.randn(N, Ho, Wo, C, device=dev).to(BF)
    y2 = (torch.randn(N, Ho, Wo, C, device=dev) * 1.5).to(BF)
    gate, rb = torch.rand(N, C, device=dev), torch.randn(N, C, device=dev) * 0.1
    sc2, sh2 = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.2
    mu2, rs2, g2 = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5, torch.rand(C, device=dev) + 0.5
    mdz2, mdzx2 = torch.randn(C, device=dev) * 0.05, torch.randn(C, device=dev) * 0.05
    mu1, rs1 = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
    rx = ext.dw_bwd_fused_x(dA, y2, gate, rb, sc2, sh2, mu2, rs2, g2, mdz2, mdzx2, w, k, x, we, sc1, sh1, mu1, rs1, mb,
                            True)
    rr = ext.dw_bwd_fused(dA, y2, gate, rb, sc2, sh2, mu2, rs2, g2, mdz2, mdzx2, w, k, y1, sc1, sh1, 1, mu1, rs1, mb,
                          -1, zout=True)
    assert rx[0].shape == (N, H, W, C)
    assert rel_err(rx[0], rr[0]) < 2e-3
    assert rel_err(rx[1], rr[1]) < 2e-3
    torch.testing.assert_close(rx[2].sum(0), rr[2].sum(0), rtol=1e-2, atol=1e-1)
    torch.testing.assert_close(rx[3].sum(0), rr[3].sum(0), rtol=1e-2, atol=1e-1)
    # the weight gradient against fp32 autograd of the same chain (dy rebuilt by BN2-backward-apply in fp32)
    z2 = y2.float() * sc2 + sh2
    sg = torch.sigmoid(z2)
    k1 = g2 * rs2
    dy = (k1 * (dA.float() * gate[:, None, None, :] + rb[:, None, None, :]) * sg * (1 + z2 * (1 - sg))
          - k1 * rs2 * mdzx2 * y2.float() - k1 * (mdz2 - mu2 * rs2 * mdzx2))
    a = F.silu(y1.float() * sc1 + sh1).permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    wf = w.view(Ce, 1, k, k).clone().requires_grad_(True)
    o = F.conv2d(a, wf, stride=s, padding=1, groups=Ce)
    o.backward(dy.permute(0, 3, 1, 2))
    assert rel_err(rx[1].view(Ce, k * k), wf.grad.view(Ce, k * k)) < 2e-2
