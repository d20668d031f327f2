"""gemm.hip v2 (csrc/kernels/gemm2.hip: persistent, LDS-DMA ring) against fp32 PyTorch references of the same ops."""
import pytest
import torch

pytestmark = pytest.mark.gpu

BF = torch.bfloat16


def _ext():
    from pytorch_rt1_for_distributed_training_amd import ops
    return ops.load()


@pytest.mark.parametrize("M,N,K", [(128, 64, 64), (300, 192, 72), (1000, 128, 520), (4096, 512, 1536),
                                   (8448, 3072, 512), (76800, 384, 2304)])
def test_gemm2_bf16_matches_fp32(M, N, K):
    torch.manual_seed(M + N + K)
    a = torch.randn(M, K, device="cuda").to(BF)
    w = (torch.randn(N, K, device="cuda") * 0.05).to(BF)
    bias = torch.randn(N, device="cuda")
    ref = a.float() @ w.float().t() + bias
    (c,) = _ext().gemm2(a, w, bias)
    assert c.dtype == BF and c.shape == (M, N)
    err = (c.float() - ref).abs().max() / ref.abs().max()
    assert err < 1e-2, float(err)
    for v in (1, 2, 3):                  # the other pipeline variants: identical math, identical bits
        assert torch.equal(_ext().gemm2(a, w, bias, variant=v)[0], c), v
    # no bias, different grids (persistence: fewer workgroups than tiles, and one per tile)
    for grid in (8, 37, 0):
        (c2,) = _ext().gemm2(a, w, None, grid=grid)
        assert torch.equal(c2, _ext().gemm2(a, w, None, grid=0)[0])
        ref0 = a.float() @ w.float().t()
        assert (c2.float() - ref0).abs().max() / ref0.abs().max() < 1e-2


def test_gemm2_stats_partials():
    torch.manual_seed(1)
    M, N, K = 1000, 192, 256
    a = torch.randn(M, K, device="cuda").to(BF)
    w = (torch.randn(N, K, device="cuda") * 0.1).to(BF)
    c, ps, pq = _ext().gemm2(a, w, None, stats=True)
    assert ps.shape == (2 * ((M + 127) // 128), N)
    cf = c.float()                    # the statistics describe the stored bf16 values
    torch.testing.assert_close(ps.sum(0), cf.sum(0), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(pq.sum(0), (cf * cf).sum(0), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_gemm2_residual_dropout_matches_tf_resid(p):
    """fp32 C = R + dropout(A W^T + bias) with transformer.hip's hash: equal (up to the bf16 rounding of the
    unfused GEMM output) to the tf_resid path it replaces, and the same dropped positions."""
    from pytorch_rt1_for_distributed_training_amd.ops import rng
    torch.manual_seed(2)
    M, N, K = 8448, 512, 1024
    ext = _ext()
    a = torch.randn(M, K, device="cuda").to(BF)
    w = (torch.randn(N, K, device="cuda") * 0.05).to(BF)
    bias = torch.randn(N, device="cuda")
    R = torch.randn(M, N, device="cuda")
    ctr = rng.counter("cuda")
    (c,) = ext.gemm2(a, w, bias, out_f32=True, R=R, p=p, salt=1234, seed_dev=ctr)
    ref = ext.tf_resid(R, torch.mm(a, w.t()), bias, p, 1234, ctr)
    assert c.dtype == torch.float32
    if p > 0:
        # same dropped set (the dropped outputs equal R exactly on both paths)
        assert torch.equal(c == R, ref == R)
    torch.testing.assert_close(c, ref, rtol=2e-2, atol=2e-2)
    h = a.float() @ w.float().t() + bias
    keep = (ref != R).float() if p > 0 else torch.ones_like(R)
    torch.testing.assert_close(c, R + keep * h / (1 - p), rtol=1e-3, atol=2e-3)
