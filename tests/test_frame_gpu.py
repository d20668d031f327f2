"""Per-frame reductions of csrc/kernels/block.hip (frame_pool, se_bn_bwd_reduce, tail_bwd_reduce) against fp64 PyTorch
on the same bf16 inputs (MI355X only).  Shapes cover both work layouts: wave mode (maps <= 1500 px, C >= 64, the
software-pipelined loop, 1-pixel maps included) and block mode (large maps: pixel splits, whole-row channel groups for
widths that are not a multiple of 64 channels -- C = 144 / 136 / 40 -- and 8-vector groups otherwise), plus the fixed
summation order (bitwise repeat)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

BF = torch.bfloat16
SHAPES = [(3, 5625, 144), (2, 5625, 192), (2, 22500, 40), (3, 2000, 136), (5, 100, 1392), (4, 361, 576), (7, 1, 96),
          (3, 1444, 288), (6, 100, 232)]


@pytest.fixture(scope="module")
def ext():
    from pytorch_rt1_for_distributed_training_amd import ops
    return ops.load()


def _inputs(N, HW, C, seed):
    torch.manual_seed(seed)
    dev = "cuda"
    y = (torch.randn(N, HW, C, device=dev) * 1.3 + 0.2).to(BF)
    g = (torch.randn(N, HW, C, device=dev) * 0.1).to(BF)
    sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.2
    mu, rs = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
    return y, g, sc, sh, mu, rs


def _close(a, ref, name):
    scale = ref.abs().max().item() + 1e-12
    torch.testing.assert_close(a.double(), ref, rtol=1e-4, atol=2e-5 * scale, msg=name)


@pytest.mark.parametrize("N,HW,C", SHAPES)
def test_frame_pool_matches_fp64(ext, N, HW, C):
    y, g, sc, sh, _, _ = _inputs(N, HW, C, N * HW + C)
    z = y.double() * sc.double() + sh.double()
    act = z * torch.sigmoid(z)
    _close(ext.frame_pool(y, None, sc, sh, 1), act.sum(1), "silu pool")
    _close(ext.frame_pool(y, g, sc, sh, 1), (act * g.double()).sum(1), "gated pool")
    _close(ext.frame_pool(y, None, None, None, 0), y.double().sum(1), "raw pool")
    a = ext.frame_pool(y, g, sc, sh, 1)
    assert torch.equal(a, ext.frame_pool(y, g, sc, sh, 1))


@pytest.mark.parametrize("N,HW,C", SHAPES)
def test_se_bn_bwd_reduce_matches_fp64(ext, N, HW, C):
    y, g, sc, sh, mu, rs = _inputs(N, HW, C, 3 * N + HW + C)
    out = ext.se_bn_bwd_reduce(g, y, sc, sh, mu, rs)
    yd, gd = y.double(), g.double()
    z = yd * sc.double() + sh.double()
    s = torch.sigmoid(z)
    act, sg = z * s, s * (1 + z * (1 - s))
    xh = (yd - mu.double()) * rs.double()
    ref = [gd * act, gd * sg, sg, gd * sg * xh, sg * xh]
    for k in range(5):
        _close(out[k], ref[k].sum(1), f"out[{k}]")
    assert torch.equal(out, ext.se_bn_bwd_reduce(g, y, sc, sh, mu, rs))


@pytest.mark.parametrize("N,HW,C", SHAPES)
@pytest.mark.parametrize("with_extras", [False, True])
def test_tail_bwd_reduce_matches_fp64(ext, N, HW, C, with_extras):
    y, d, sc, sh, mu, rs = _inputs(N, HW, C, 5 * N + HW + C)
    dev = "cuda"
    keep = (torch.rand(N, device=dev) > 0.3).float() / 0.7 if with_extras else None
    skip = torch.randn(N, HW, C, device=dev).to(BF) if with_extras else None
    fmul = torch.rand(N, C, device=dev) + 0.5 if with_extras else None
    dmul, dadd, pdz, pdzx = ext.tail_bwd_reduce(d, y, sc, sh, mu, rs, keep, skip, fmul)
    yd, dd = y.double(), d.double()
    kp = keep.double()[:, None, None] if keep is not None else 1.0
    h = (yd * sc.double() + sh.double()) * kp + (skip.double() if skip is not None else 0.0)
    dz = dd * (fmul.double()[:, None, :] if fmul is not None else 1.0) * kp
    xh = (yd - mu.double()) * rs.double()
    _close(dmul, (dd * h).sum(1), "dmul")
    _close(dadd, dd.sum(1), "dadd")
    _close(pdz, dz.sum(1), "sum dz")
    _close(pdzx, (dz * xh).sum(1), "sum dz*xh")
