"""256-row LDS-DMA MFMA GEMM (csrc/kernels/gemm256.hip) vs fp32 PyTorch: NT / NN operands at both N tiles, ragged M / N /
K edges (the zero-source DMA lanes), bias, the BN-statistics epilogue and the BN + SiLU + gate operand prologue (bit for
bit against bn_apply + the same product, and the stored operand against bn_apply)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

BF = torch.bfloat16


@pytest.fixture(scope="module")
def ext():
    from pytorch_rt1_for_distributed_training_amd import ops
    return ops.load()


def rel_err(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-12))


@pytest.mark.parametrize("M,N,K", [(76800 // 8, 2304, 384), (9600, 1392, 232), (5000, 384, 2304), (4000, 512, 1536),
                                   (8448, 3072, 512), (777, 264, 72), (300, 40, 136), (256, 256, 64), (1, 8, 8)])
@pytest.mark.parametrize("nn", [False, True])
@pytest.mark.parametrize("bn", [256, 128])
def test_gemm256_layouts(ext, M, N, K, nn, bn):
    torch.manual_seed(M + N + K)
    a = torch.randn(M, K, device="cuda").to(BF)
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(BF)          # a Linear weight [N, K]
    b = w.t().contiguous() if nn else w                                 # NN: the [K, N] operand
    (c,) = ext.gemm256(a, b, nn, bn=bn)
    ref = a.float() @ w.float().t()
    assert c.dtype == BF and c.shape == (M, N)
    assert rel_err(c, ref) < 6e-3
    if not nn:
        bias = torch.randn(N, device="cuda")
        (cb,) = ext.gemm256(a, b, False, bias, bn=bn)
        assert rel_err(cb, ref + bias) < 6e-3


def test_gemm256_exact_small_integers(ext):
    """Integer-valued operands: every product and sum is exact in fp32, so the output must equal the reference
    exactly -- catches a wrong lane / swizzle mapping that a tolerance could hide.  Asymmetric B (row != column)."""
    M, N, K = 520, 264, 200
    a = torch.randint(-3, 4, (M, K), device="cuda").to(BF)
    w = (torch.arange(N, device="cuda")[:, None] % 5 - 2 + (torch.arange(K, device="cuda")[None, :] % 3)).to(BF)
    ref = (a.float() @ w.float().t()).to(BF)
    for bn in (256, 128):
        assert torch.equal(ext.gemm256(a, w, False, bn=bn)[0], ref)
        assert torch.equal(ext.gemm256(a, w.t().contiguous(), True, bn=bn)[0], ref)


@pytest.mark.parametrize("M,N,K,bn", [(76800 // 8, 1536, 384, 256), (9600, 1392, 232, 256), (5000, 384, 2304, 128),
                                      (3000, 232, 1392, 256)])
def test_gemm256_stats_epilogue(ext, M, N, K, bn):
    torch.manual_seed(1)
    a = torch.randn(M, K, device="cuda").to(BF)
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(BF)
    c, ps, pq = ext.gemm256(a, w, False, stats=True, bn=bn)
    assert ps.shape == ((M + 255) // 256, N)
    cf = c.float()
    torch.testing.assert_close(ps.sum(0), cf.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(pq.sum(0), (cf * cf).sum(0), rtol=1e-4, atol=1e-2)
    assert rel_err(c, a.float() @ w.float().t()) < 6e-3


@pytest.mark.parametrize("M,N,K,hw,bn", [(7600, 232, 1392, 100, 256), (7600, 384, 2304, 100, 128),
                                         (1083, 136, 576, 361, 256), (2000, 512, 1536, 100, 256)])
@pytest.mark.parametrize("stats", [False, True])
def test_gemm256_bn_silu_gate_prologue(ext, M, N, K, hw, bn, stats):
    """A = silu(y * scale + shift) * gate[m / hw] rebuilt in LDS == bn_apply + the plain product, bit for bit."""
    torch.manual_seed(2)
    y = (torch.randn(M, K, device="cuda") * 1.5).to(BF)
    sc, sh = torch.rand(K, device="cuda") + 0.5, torch.randn(K, device="cuda") * 0.3
    gate = torch.rand(M // hw, K, device="cuda")
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(BF)
    res = ext.gemm256(y, w, False, None, sc, sh, gate, hw, stats=stats, store_a=True, bn=bn)
    a = ext.bn_apply(y, sc, sh, 1, gate, hw)                  # the pass the prologue replaces (same rounding)
    (ref,) = ext.gemm256(a, w, False, bn=bn)
    assert torch.equal(res[0], ref)
    assert torch.equal(res[-1], a)
    af = torch.nn.functional.silu(y.float() * sc + sh) * gate.repeat_interleave(hw, 0)
    assert rel_err(res[0], af @ w.float().t()) < 6e-3
    if stats:
        cf = res[0].float()
        torch.testing.assert_close(res[1].sum(0), cf.sum(0), rtol=1e-4, atol=1e-2)
