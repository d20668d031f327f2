"""MFMA depthwise forward (csrc/kernels/dwmfma.hip) vs a plain PyTorch fp32 reference (MI355X only).

ext.dw_fwd_mfma runs the MFMA kernel (ext.dw_fwd takes it only with RT1_DW_MFMA=1: it measured slower than the
vector-ALU forward, profiles/r3_dw_mfma_ab.md); these cases pin
the real low-resolution layer shapes of the b128 step plus the edges of the patch / chunk tiling: maps that are not
a multiple of 4, a partial last 32-channel chunk (816, 1392 = 16 mod 32), a 16-channel-chunk map (38 x 38, > 2
patch groups), frames walked by fewer workgroups than frames (mb < N), and the prologue-free (copy) variant."""
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


CASES = [
    # k, C, H, W, prologue, N, mb
    (5, 816, 19, 19, True, 6, 64),     # blocks 14-17
    (5, 576, 19, 19, True, 5, 3),      # block 13 (frames walked by 3 workgroups)
    (5, 1392, 10, 10, True, 7, 64),    # blocks 19-23
    (5, 288, 38, 38, True, 3, 64),     # blocks 6-7 (16-channel chunks, 7 patch groups)
    (3, 576, 19, 19, True, 4, 64),     # blocks 9-12
    (3, 2304, 10, 10, True, 3, 2),     # block 25
    (3, 1392, 10, 10, True, 3, 64),    # block 24
    (5, 40, 13, 7, False, 3, 64),      # copy prologue, odd map, partial chunk of 8
    (3, 24, 5, 9, True, 2, 64),
    (5, 136, 1, 1, True, 2, 64),       # 1 x 1 map
    (3, 48, 33, 21, True, 2, 64),      # > 20: 16-channel chunks
]


@pytest.mark.parametrize("k,C,H,W,prologue,N,mb", CASES)
def test_dw_fwd_mfma_matches_fp32(ext, k, C, H, W, prologue, N, mb):
    torch.manual_seed(0)
    x = torch.randn(N, H, W, C, device="cuda").to(BF)
    w = torch.randn(C, 1, k, k, device="cuda") * 0.3
    scale = (torch.rand(C, device="cuda") + 0.5) if prologue else None
    shift = (torch.randn(C, device="cuda") * 0.2) if prologue else None
    out, ps, pq = ext.dw_fwd_mfma(x, w.view(C, k * k), scale, shift, 1 if prologue else 0, k, mb)
    xr = x.float().permute(0, 3, 1, 2)
    a = F.silu(xr * scale[None, :, None, None] + shift[None, :, None, None]) if prologue else xr
    ref = F.conv2d(a, w, padding=(k - 1) // 2, groups=C)
    assert out.shape == (N, H, W, C)
    assert torch.isfinite(out.float()).all()
    assert rel_err(out.permute(0, 3, 1, 2), ref) < 1e-2
    # the statistics describe the stored bf16 tensor
    o = out.float()
    torch.testing.assert_close(ps.sum(0), o.sum((0, 1, 2)), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(pq.sum(0), (o ** 2).sum((0, 1, 2)), rtol=1e-3, atol=1e-2)


def test_dw_fwd_mfma_deterministic(ext):
    torch.manual_seed(1)
    x = torch.randn(16, 19, 19, 816, device="cuda").to(BF)
    w = torch.randn(816, 25, device="cuda") * 0.3
    sc, sh = torch.rand(816, device="cuda") + 0.5, torch.randn(816, device="cuda") * 0.2
    a = ext.dw_fwd_mfma(x, w, sc, sh, 1, 5, 8)
    b = ext.dw_fwd_mfma(x, w, sc, sh, 1, 5, 8)
    for u, v in zip(a, b):
        assert torch.equal(u, v)
