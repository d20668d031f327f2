"""Data parallel over torch.distributed (gloo on CPU, 2 ranks) — correctness of the
bucketed all-reduce, parameter broadcast, buffer broadcast and gradient-order probe."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

import pytorch_rt1_for_distributed_training_amd as rt1
from pytorch_rt1_for_distributed_training_amd.data.synthetic import make_batch


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg():
    return rt1.preset("tiny").replace(seq_len=2)


def _batch(b):
    g = torch.Generator().manual_seed(123)
    return make_batch(b, 2, 64, 64, uint8=False, generator=g)


def _shard(batch, lo, hi):
    if isinstance(batch, dict):
        return {k: _shard(v, lo, hi) for k, v in batch.items()}
    return batch[lo:hi]


def _worker(rank, world, port, out_dir, bucket_mb):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(2)
    from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine, split_batch
    from pytorch_rt1_for_distributed_training_amd.models import build_rt1
    from pytorch_rt1_for_distributed_training_amd.parallel import dist as pdist
    ctx = pdist.init_distributed("cpu")
    torch.manual_seed(1000 + rank)  # different init per rank: the broadcast must fix it
    model = build_rt1(_cfg())
    eng = TrainEngine(model, _cfg(), bucket_cap_mb=bucket_mb, order_probe=True)
    assert len(eng.ddp.buckets) >= 1
    full = _batch(4)
    per = 4 // world
    shard = _shard(full, rank * per, (rank + 1) * per)
    eng.ddp.prepare()
    eng.optimizer.zero_grad()
    model.eval()
    loss_bt, _ = model.train_forward(*split_batch(shard), shift=(0, 0), with_aux=False)
    loss_bt.mean().backward()
    eng.ddp.finish()
    grads = {n: (p.grad * eng.ddp.grad_scale).clone() for n, p in model.named_parameters() if p.requires_grad}
    params = {n: p.detach().clone() for n, p in model.named_parameters()}
    torch.save({"grads": grads, "params": params, "nbuckets": len(eng.ddp.buckets)},
               os.path.join(out_dir, f"rank{rank}.pt"))
    pdist.shutdown()


@pytest.mark.parametrize("bucket_mb", [0.5, 64.0])
def test_dp_gradients_match_single_process(tmp_path, bucket_mb):
    world = 2
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, str(tmp_path), bucket_mb), nprocs=world, join=True,
                       start_method="spawn")
    r0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "rank1.pt", weights_only=True)
    if bucket_mb < 1:
        assert r0["nbuckets"] > 3
    # identical parameters after the rank-0 broadcast
    for n in r0["params"]:
        assert torch.equal(r0["params"][n], r1["params"][n]), n
    # single-process reference with rank 0's (broadcast) weights on the full batch
    from pytorch_rt1_for_distributed_training_amd.engine.step import split_batch
    from pytorch_rt1_for_distributed_training_amd.models import build_rt1
    model = build_rt1(_cfg())
    with torch.no_grad():
        for n, p in model.named_parameters():
            p.copy_(r0["params"][n])
    model.eval()
    loss_bt, _ = model.train_forward(*split_batch(_batch(4)), shift=(0, 0), with_aux=False)
    loss_bt.mean().backward()
    # the reference normalises CE by the PER-RANK batch (b*t*11), so DP grads = world x single-process grads
    for n, p in model.named_parameters():
        if not p.requires_grad:
            continue
        torch.testing.assert_close(r0["grads"][n], world * p.grad, rtol=2e-4, atol=1e-7, msg=n)
        torch.testing.assert_close(r1["grads"][n], r0["grads"][n], rtol=0, atol=0, msg=n)
