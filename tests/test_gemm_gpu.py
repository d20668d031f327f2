"""Tiled MFMA GEMM (csrc/kernels/gemm.hip) vs fp32 PyTorch: NT / NN operand layouts, every tile configuration,
ragged M / N / K edges, bias, fp32 output, the BN-statistics epilogue and the BN + SiLU + gate operand prologue."""
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


@pytest.mark.parametrize("M,N,K", [(8448, 3072, 512), (8448, 512, 1024), (1000, 232, 1392), (777, 1536, 384),
                                   (300, 40, 24), (129, 264, 72)])
@pytest.mark.parametrize("nn", [False, True])
@pytest.mark.parametrize("cfg", [0, 1, 2])
def test_gemm_layouts(ext, M, N, K, nn, cfg):
    torch.manual_seed(M + N + K)
    a = torch.randn(M, K, device="cuda").to(BF)
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(BF)          # a Linear weight [N, K]
    b = w.t().contiguous() if nn else w                                 # NN: the [K, N] operand
    bias = torch.randn(N, device="cuda")
    (c,) = ext.gemm(a, b, nn, bias, cfg=cfg)
    ref = a.float() @ w.float().t() + bias
    assert c.dtype == BF and c.shape == (M, N)
    assert rel_err(c, ref) < 8e-3
    (c32,) = ext.gemm(a, b, nn, None, out_f32=True, cfg=cfg)
    assert c32.dtype == torch.float32
    assert rel_err(c32, a.float() @ w.float().t()) < 1e-5


@pytest.mark.parametrize("M,N,K,cfg", [(76800 // 8, 232, 1392, -1), (5000, 384, 2304, 0), (4000, 512, 1536, 1),
                                       (3000, 64, 96, 2)])
def test_gemm_stats_epilogue(ext, M, N, K, cfg):
    torch.manual_seed(1)
    a = torch.randn(M, K, device="cuda").to(BF)
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(BF)
    c, ps, pq = ext.gemm(a, w, False, stats=True, cfg=cfg)
    cf = c.float()
    torch.testing.assert_close(ps.sum(0), cf.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(pq.sum(0), (cf * cf).sum(0), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("M,N,K,hw", [(7600, 232, 1392, 100), (7600, 384, 2304, 100), (1083, 136, 576, 361)])
@pytest.mark.parametrize("stats", [False, True])
def test_gemm_bn_silu_gate_prologue(ext, M, N, K, hw, stats):
    """A = silu(y * scale + shift) * gate[m / hw] rebuilt in the operand load == bn_apply + plain GEMM."""
    torch.manual_seed(2)
    y = (torch.randn(M, K, device="cuda") * 1.5).to(BF)
    sc, sh = torch.rand(K, device="cuda") + 0.5, torch.randn(K, device="cuda") * 0.3
    gate = torch.rand(M // hw, K, device="cuda")
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(BF)
    res = ext.gemm(y, w, False, None, sc, sh, gate, hw, stats=stats)
    a = ext.bn_apply(y, sc, sh, 1, gate, hw)                  # the pass the prologue replaces (same rounding)
    (ref,) = ext.gemm(a, w, False)
    assert torch.equal(res[0], ref)
    af = torch.nn.functional.silu(y.float() * sc + sh) * gate.repeat_interleave(hw, 0)
    assert rel_err(res[0], af @ w.float().t()) < 8e-3
    if stats:
        cf = res[0].float()
        torch.testing.assert_close(res[1].sum(0), cf.sum(0), rtol=1e-4, atol=1e-2)
    # the rebuilt operand stored for the weight gradient == bn_apply's output, bit for bit
    for cfg in (0, 1):
        out = ext.gemm(y, w, False, None, sc, sh, gate, hw, stats=stats, cfg=cfg, store_a=True)
        assert torch.equal(out[0], ref) and torch.equal(out[-1], a)


@pytest.mark.parametrize("M,N,K,K2,hw,res,cfg", [(7600, 232, 1392, 232, 100, True, -1), (3610, 136, 816, 136, 361, True, -1),
                                                 (1000, 232, 1392, 232, 100, False, 0), (777, 64, 200, 40, 7, True, 2),
                                                 (640, 384, 2304, 384, 64, True, 1)])
def test_gemm_tail_two_segments_residual(ext, M, N, K, K2, hw, res, cfg):
    """C = A B^T + A2 B2^T + bias + res * rmul[m / hw] (the dz-mode expand dgrad of blocks 18-24) vs fp32."""
    torch.manual_seed(3)
    a = torch.randn(M, K, device="cuda").to(BF)
    b = (torch.randn(N, K, device="cuda") * K ** -0.5).to(BF)
    a2 = torch.randn(M, K2, device="cuda").to(BF)
    b2 = (torch.randn(N, K2, device="cuda") * K2 ** -0.5).to(BF)
    bias = torch.randn(N, device="cuda")
    r = torch.randn(M, N, device="cuda").to(BF) if res else None
    rm = torch.rand(M // hw, N, device="cuda") if res else None
    c = ext.gemm_tail(a, b, a2, b2, bias, r, rm, hw, cfg)
    ref = a.float() @ b.float().t() + a2.float() @ b2.float().t() + bias
    if res:
        ref = ref + (r.float().view(M // hw, hw, N) * rm[:, None, :]).view(M, N)
    assert c.dtype == BF and c.shape == (M, N)
    assert rel_err(c, ref) < 8e-3


