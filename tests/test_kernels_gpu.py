"""HIP kernel numerics vs plain PyTorch fp32 references (MI355X only)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ext():
    from pytorch_rt1_for_distributed_training_amd import ops
    return ops.load()


def test_flat_adam_matches_reference(ext):
    from pytorch_rt1_for_distributed_training_amd.ops.adam import flat_adam_step, reference_adam_step
    torch.manual_seed(0)
    n = 1_000_003 + 1  # not a multiple of 4 -> exercises the scalar tail
    p = torch.randn(n, device="cuda")
    g = torch.randn(n, device="cuda")
    m = torch.randn(n, device="cuda") * 0.1
    v = torch.rand(n, device="cuda") * 0.1
    ref = [t.clone() for t in (p, g, m, v)]
    for step in (1, 2, 7):
        kw = dict(lr=5e-4, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.01 if step == 7 else 0.0, step=step,
                  grad_scale=0.25)
        flat_adam_step(p, g, m, v, **kw)
        reference_adam_step(ref[0], ref[1], ref[2], ref[3], **kw)
    torch.testing.assert_close(p, ref[0], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(m, ref[2], rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(v, ref[3], rtol=1e-5, atol=1e-8)


def test_engine_step_hip_backend_small(ext):
    from pytorch_rt1_for_distributed_training_amd.config import RT1Config
    from pytorch_rt1_for_distributed_training_amd.data.synthetic import make_batch
    from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine
    from pytorch_rt1_for_distributed_training_amd.models import build_rt1
    torch.manual_seed(0)
    cfg = RT1Config(height=96, width=96, seq_len=2, backend="hip")
    eng = TrainEngine(build_rt1(cfg), cfg, order_probe=False)
    assert eng.backend == "hip"
    batch = make_batch(2, 2, 96, 96, device="cuda")
    losses = [float(eng.train_step(batch)) for _ in range(3)]
    assert all(math.isfinite(x) for x in losses), losses


@pytest.mark.parametrize("T", [6, 2, 15])
def test_rt1_attention_matches_eager(ext, T):
    from pytorch_rt1_for_distributed_training_amd.models.transformer import masked_attention, rt1_attention_mask
    from pytorch_rt1_for_distributed_training_amd.ops.attention import RT1AttentionFn
    torch.manual_seed(0)
    B, H, D, L, K = 3, 8, 128, 11, 8
    S = T * L
    qkv = torch.randn(B, S, 3, H, D, device="cuda").to(torch.bfloat16).requires_grad_(True)
    out = RT1AttentionFn.apply(qkv, L, K, 0.0, 0)
    q, k, v = qkv.detach().float().permute(2, 0, 3, 1, 4).unbind(0)
    q, k, v = (t.clone().requires_grad_(True) for t in (q, k, v))
    mask = rt1_attention_mask(T, K, L - K).cuda()
    ref, _ = masked_attention(q, k, v, mask, 0.0, False)
    ref = ref.permute(0, 2, 1, 3)
    err = float((out.float() - ref).norm() / ref.norm())
    assert err < 1e-2, err
    g = torch.randn_like(ref)
    out.backward(g.to(torch.bfloat16))
    ref.backward(g)
    dref = torch.stack([q.grad, k.grad, v.grad], 0).permute(1, 3, 0, 2, 4)
    derr = float((qkv.grad.float() - dref).norm() / dref.norm())
    assert derr < 2e-2, derr


def test_rt1_attention_dropout_mask_consistent(ext):
    """Forward dropout (in-kernel hash) == explicit keep-mask applied to the eager softmax."""
    from pytorch_rt1_for_distributed_training_amd.models.transformer import rt1_attention_mask
    from pytorch_rt1_for_distributed_training_amd.ops.attention import RT1AttentionFn
    torch.manual_seed(1)
    B, H, D, L, K, T = 2, 8, 128, 11, 8, 6
    S = T * L
    qkv = torch.randn(B, S, 3, H, D, device="cuda").to(torch.bfloat16)
    out = RT1AttentionFn.apply(qkv, L, K, 0.1, 1234)
    q, k, v = qkv.float().permute(2, 0, 3, 1, 4).unbind(0)
    mask = rt1_attention_mask(T, K, L - K).cuda()
    s = (q @ k.transpose(-1, -2) / D ** 0.5).masked_fill(mask == 0, float("-inf"))
    keep = ext.attn_keepmask(B * H, S, 0.1, 1234, qkv).view(B, H, S, S).float()
    assert 0.85 < float(keep.mean()) < 0.95
    ref = (torch.softmax(s, -1) * keep / 0.9) @ v
    err = float((out.float() - ref.permute(0, 2, 1, 3)).norm() / ref.norm())
    assert err < 1e-2, err


def test_native_rccl_communicator_single_rank():
    """csrc/comm.cpp: RCCL communicator on its own stream (world = 1 on the one-GPU box)."""
    from pytorch_rt1_for_distributed_training_amd.parallel.native_comm import NativeComm
    c = NativeComm.single(0)
    t = torch.arange(1000, device="cuda", dtype=torch.float32)
    ref = t.clone()
    w = c.all_reduce_(t)
    w.wait()
    torch.cuda.synchronize()
    assert torch.equal(t, ref)
    b = torch.randn(77, device="cuda").to(torch.bfloat16)
    b0 = b.clone()
    c.broadcast_(b, 0)
    parts = [torch.ones(10, device="cuda"), torch.full((3,), 2.0, device="cuda")]
    c.all_reduce_coalesced_(parts).wait()
    torch.cuda.synchronize()
    assert torch.equal(b, b0) and float(parts[1][0]) == 2.0
    c.destroy()
