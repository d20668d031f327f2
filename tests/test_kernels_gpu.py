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
