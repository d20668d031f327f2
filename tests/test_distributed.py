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


class _FakeCapture:
    """Stands in for engine.graphs.SegmentedCapture on CPU: records where the graph would be cut."""

    def __init__(self):
        self.stream = None
        self.cuts = []

    def bucket_ready(self, index):
        self.cuts.append(index)


def _worker4(rank, world, port, out_dir, comm_dtype):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(2)
    from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine, split_batch
    from pytorch_rt1_for_distributed_training_amd.models import build_rt1
    from pytorch_rt1_for_distributed_training_amd.parallel import dist as pdist
    pdist.init_distributed("cpu")
    torch.manual_seed(7)
    model = build_rt1(_cfg())
    # a trainable parameter the forward never touches: its bucket can only complete through finish()'s flush
    model.register_parameter("unused_probe", torch.nn.Parameter(torch.ones(5)))
    dtype = {"fp32": torch.float32, "bf16": torch.bfloat16}[comm_dtype]
    eng = TrainEngine(model, _cfg(), bucket_cap_mb=0.25, order_probe=True, grad_comm_dtype=dtype)
    full = _batch(4)
    per = 4 // world
    shard = _shard(full, rank * per, (rank + 1) * per)

    def fwd_bwd():
        model.eval()
        loss_bt, _ = model.train_forward(*split_batch(shard), shift=(0, 0), with_aux=False)
        loss_bt.mean().backward()

    eng.ddp.prepare()
    eng.optimizer.zero_grad()
    fwd_bwd()
    eng.ddp.finish()
    log = list(eng.ddp.launch_log)
    grads = {n: (p.grad * eng.ddp.grad_scale).clone() for n, p in model.named_parameters() if p.requires_grad}
    # capture-mode hooks (what the segmented hipGraph DP step relies on) on the same backward
    fake = _FakeCapture()
    eng.optimizer.zero_grad()
    with eng.ddp.capture_cuts(fake):
        fwd_bwd()
    rest = eng.ddp.unlaunched_buckets()
    eng.flat.gather_grads()
    gathered_local = eng.flat.grad.clone()
    params = {n: p.detach().clone() for n, p in model.named_parameters()}
    torch.save({"grads": grads, "params": params, "nbuckets": len(eng.ddp.buckets), "log": log, "cuts": fake.cuts,
                "rest": rest, "local": gathered_local,
                "unused_bucket": eng.ddp._param_bucket[eng.flat.index[id(model.unused_probe)]]},
               os.path.join(out_dir, f"rank{rank}.pt"))
    pdist.shutdown()


@pytest.mark.parametrize("comm_dtype", ["fp32", "bf16"])
def test_dp_four_ranks_bucket_order_flush_and_compression(tmp_path, comm_dtype):
    world = 4
    port = _free_port()
    mp.start_processes(_worker4, args=(world, port, str(tmp_path), comm_dtype), nprocs=world, join=True,
                       start_method="spawn")
    rs = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    nb = rs[0]["nbuckets"]
    assert nb >= 4
    for r in rs:
        # every bucket issued exactly once; buckets are laid out in gradient-ready order, so they are issued in
        # increasing order -- except the bucket holding the never-used parameter, flushed by finish() at the end
        assert sorted(r["log"]) == list(range(nb)), r["log"]
        ub = r["unused_bucket"]
        assert r["log"][-1] == ub
        assert [b for b in r["log"] if b != ub] == sorted(b for b in r["log"] if b != ub)
        # capture mode: every bucket except the one that can never complete reports a cut, in order
        assert r["cuts"] == [b for b in range(nb) if b != ub]
        assert r["rest"] == [ub]
    # single-process reference on the full batch with the same weights
    from pytorch_rt1_for_distributed_training_amd.engine.step import split_batch
    from pytorch_rt1_for_distributed_training_amd.models import build_rt1
    model = build_rt1(_cfg())
    model.register_parameter("unused_probe", torch.nn.Parameter(torch.ones(5)))
    with torch.no_grad():
        for n, p in model.named_parameters():
            p.copy_(rs[0]["params"][n])
    model.eval()
    loss_bt, _ = model.train_forward(*split_batch(_batch(4)), shift=(0, 0), with_aux=False)
    loss_bt.mean().backward()
    tol = dict(rtol=2e-4, atol=1e-7) if comm_dtype == "fp32" else dict(rtol=2e-2, atol=2e-5)
    for n, p in model.named_parameters():
        if not p.requires_grad:
            continue
        if n == "unused_probe":
            for r in rs:
                assert torch.count_nonzero(r["grads"][n]) == 0
            continue
        torch.testing.assert_close(rs[0]["grads"][n], world * p.grad, msg=n, **tol)
        for r in rs[1:]:
            torch.testing.assert_close(r["grads"][n], rs[0]["grads"][n], rtol=0, atol=0, msg=n)
