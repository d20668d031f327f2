"""Full-row transformer GEMMs with fused residual / dropout / LayerNorm epilogues (csrc/kernels/tfrow.hip) vs fp32
PyTorch: forward x + dropout(A W^T + b) and the next LayerNorm, backward A W followed by the LayerNorm backward
(dx, dgamma, dbeta) and the bf16 copy + column sums of dx."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

BF = torch.bfloat16


@pytest.fixture(scope="module")
def ext():
    from pytorch_rt1_for_distributed_training_amd import ops
    return ops.load()


def rel_err(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-12))


@pytest.mark.parametrize("T,K", [(8448, 1024), (8448, 512), (1000, 512), (45, 1024), (33, 72)])
@pytest.mark.parametrize("ln", [False, True])
def test_tf_row_fwd(ext, T, K, ln):
    torch.manual_seed(T + K)
    a = torch.randn(T, K, device="cuda").to(BF)
    w = (torch.randn(512, K, device="cuda") * K ** -0.5).to(BF)
    x = torch.randn(T, 512, device="cuda")
    b = torch.randn(512, device="cuda") * 0.1
    lg, lb = torch.rand(512, device="cuda") + 0.5, torch.randn(512, device="cuda") * 0.1
    out = ext.tf_row_fwd(a, w, x, b, lg=lg if ln else None, lb=lb if ln else None, eps=1e-6)
    ref = x + a.float() @ w.float().t() + b
    assert rel_err(out[0], ref) < 1e-5
    if ln:
        xo = out[0]
        ref_n = F.layer_norm(xo, (512,), lg, lb, 1e-6)
        assert rel_err(out[1], ref_n) < 5e-3
        torch.testing.assert_close(out[2], xo.mean(1), rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(out[3], torch.rsqrt(xo.var(1, unbiased=False) + 1e-6), rtol=1e-4, atol=1e-4)


def test_tf_row_fwd_dropout_matches_drop_bwd_mask(ext):
    """The epilogue's dropout mask is the counter hash tf_drop_bwd regenerates (same seed, same device counter)."""
    torch.manual_seed(3)
    T, K, p, seed = 2000, 512, 0.1, 12345
    a = torch.randn(T, K, device="cuda").to(BF)
    w = (torch.randn(512, K, device="cuda") * K ** -0.5).to(BF)
    x = torch.randn(T, 512, device="cuda")
    b = torch.randn(512, device="cuda") * 0.1
    ctr = torch.tensor([7], dtype=torch.int32, device="cuda")
    (xo,) = ext.tf_row_fwd(a, w, x, b, p, seed, ctr)
    keep, _ = ext.tf_drop_bwd(torch.ones(T, 512, device="cuda"), p, seed, ctr)
    kept = keep.float() != 0
    assert 0.85 < float(kept.float().mean()) < 0.95
    ref = x + torch.where(kept, (a.float() @ w.float().t() + b) / (1 - p), torch.zeros_like(x))
    assert rel_err(xo, ref) < 1e-5


@pytest.mark.parametrize("T,K", [(8448, 3072), (8448, 512), (1000, 512), (45, 3072), (33, 72)])
@pytest.mark.parametrize("dres,want_bf", [(True, True), (False, False)])
def test_tf_row_bwd(ext, T, K, dres, want_bf):
    torch.manual_seed(T * 7 + K)
    a = (torch.randn(T, K, device="cuda") * 0.1).to(BF)
    w = (torch.randn(K, 512, device="cuda") * K ** -0.5).to(BF)          # [K, 512]: dxn = a @ w
    xin = torch.randn(T, 512, device="cuda") * 2 + 0.5
    g = torch.rand(512, device="cuda") + 0.5
    mu = xin.mean(1)
    rs = torch.rsqrt(xin.var(1, unbiased=False) + 1e-6)
    r = torch.randn(T, 512, device="cuda") if dres else None
    out = ext.tf_row_bwd(a, w, xin, mu, rs, g, r, want_bf)
    dxn = a.float() @ w.float()
    xr = xin.clone().requires_grad_(True)
    gr = g.clone().requires_grad_(True)
    br = torch.zeros(512, device="cuda", requires_grad=True)
    F.layer_norm(xr, (512,), gr, br, 1e-6).backward(dxn)
    ref_dx = xr.grad + (r if dres else 0)
    assert rel_err(out[0], ref_dx) < 2e-4
    assert rel_err(out[1], gr.grad) < 2e-4
    assert rel_err(out[2], br.grad) < 2e-4
    if want_bf:
        assert torch.equal(out[3], out[0].to(BF))
        torch.testing.assert_close(out[4], out[3].float().sum(0), rtol=1e-4, atol=1e-3)
