#!/usr/bin/env python3
"""Data-parallel correctness on ONE GPU box: 2 ranks share cuda:0, collectives over gloo (RCCL refuses
two ranks on one device).  Exercises the real hip backend + DataParallel bucket hooks + fused Adam:
after K steps on different data per rank, every rank must hold bit-identical parameters and BN buffers.

  torchrun --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/dp_gpu_check.py [--graph]

``--graph`` also runs the hipGraph DP step (forward+backward captured as graph segments cut at bucket
boundaries, each bucket's all-reduce issued between segment replays) side by side with the eager bucketed path
on the same data, and requires the all-reduced flat gradient and the parameters to be BITWISE equal after every
step (the kernels are deterministic, dropout / drop-path / random shift are off); on a mismatch it names the
buckets and parameters that differ.  ``--eager2`` does the same with two eager DP engines (eager == eager: the
run-to-run reproducibility of the data-parallel step).  ``--steps K`` (default 4).  Exit code 2 = mismatch.
"""
from __future__ import annotations

import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pytorch_rt1_for_distributed_training_amd as rt1  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.data.synthetic import make_batch  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.models import build_rt1  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.parallel import dist as pdist  # noqa: E402

BUCKET_MB = float(os.environ.get("RT1_DPCHECK_BUCKET_MB", "4.0"))   # debug: bucket size of the check


def _run(ctx, cfg, graph: bool, steps: int):
    torch.manual_seed(0)
    model = build_rt1(cfg)
    eng = TrainEngine(model, cfg, order_probe=True, bucket_cap_mb=BUCKET_MB, graph=graph)
    assert eng.ddp.enabled and (len(eng.ddp.buckets) > 1 or BUCKET_MB > 4.0), "expected several gradient buckets"
    g = torch.Generator().manual_seed(100 + ctx.rank)
    losses = []
    for _ in range(steps):
        batch = make_batch(4, cfg.seq_len, 128, 128, device=ctx.device, generator=g)
        losses.append(float(eng.train_step(batch)))
    torch.cuda.synchronize()
    return eng, losses


def _named_diffs(eng, a, b, limit=8):
    names = {id(p): n for n, p in eng.model.named_parameters()}
    out = []
    for bi, bk in enumerate(eng.ddp.buckets if eng.ddp.enabled else []):
        if not torch.equal(a[bk.start:bk.end], b[bk.start:bk.end]):
            bad = []
            for i in bk.members:
                off, n = eng.flat.segment(i)
                d = float((a[off:off + n] - b[off:off + n]).abs().max())
                if d != 0:
                    bad.append(f"{names.get(id(eng.flat.params[i]), i)}:{d:.2e}")
            out.append(f"bucket {bi}: " + ", ".join(bad[:limit]))
    return out


def _keep_local_grads(eng):
    """Snapshot every bucket's LOCAL (pre-all-reduce) gradient as its all-reduce is issued (debug: tells a difference
    in this rank's backward from one introduced by the collective)."""
    eng.local_grad = torch.zeros_like(eng.flat.grad)
    orig = eng.ddp._all_reduce

    def wrapped(t):
        off = t.data_ptr() - eng.flat.grad.data_ptr()
        eng.local_grad[off // 4: off // 4 + t.numel()].copy_(t)
        return orig(t)
    eng.ddp._all_reduce = wrapped


def _se_debug_report(tag: str):
    from pytorch_rt1_for_distributed_training_amd.ops import backbone
    bad = [(n, int(v)) for n, v in backbone.SE_DEBUG_LOG if int(v) != 0]
    backbone.SE_DEBUG_LOG.clear()
    if bad:
        print(f"   [{tag}] SE debug mismatches: {bad}", flush=True)


def _pair_vs(ctx, cfg, steps: int, graph_a: bool) -> bool:
    """Engine A (graph DP if ``graph_a`` else eager DP) and eager-DP engine B stepped on the same batches from the same
    initial state; bitwise comparison of the reduced flat gradient, the local (pre-all-reduce) gradient, the
    parameters and the loss after every step."""
    torch.manual_seed(0)
    eg = TrainEngine(build_rt1(cfg), cfg, order_probe=True, bucket_cap_mb=BUCKET_MB, graph=graph_a)
    torch.manual_seed(0)
    ee = TrainEngine(build_rt1(cfg), cfg, order_probe=True, bucket_cap_mb=BUCKET_MB, graph=False)
    assert eg.ddp.enabled and (len(eg.ddp.buckets) > 1 or BUCKET_MB > 4.0), "expected several gradient buckets"
    _keep_local_grads(eg)
    _keep_local_grads(ee)
    g = torch.Generator().manual_seed(100 + ctx.rank)
    ok = True
    name_a = "graph" if graph_a else "eagerA"
    for step in range(steps):
        batch = make_batch(4, cfg.seq_len, 128, 128, device=ctx.device, generator=g)
        lg = float(eg.train_step(batch))
        _se_debug_report(f"rank{ctx.rank} {name_a} step {step + 1}")
        le = float(ee.train_step(batch))
        _se_debug_report(f"rank{ctx.rank} eager step {step + 1}")
        torch.cuda.synchronize()
        gsame = torch.equal(eg.flat.grad, ee.flat.grad)
        lsame = torch.equal(eg.local_grad, ee.local_grad)
        psame = torch.equal(eg.flat.data, ee.flat.data)
        flags = torch.tensor([float(not lsame)], device=ctx.device)
        dist.all_reduce(flags)
        if not lsame:
            for line in _named_diffs(eg, eg.local_grad, ee.local_grad):
                print(f"   rank{ctx.rank} local grad " + line, flush=True)
        if ctx.rank == 0:
            nseg = eg._segments.num_segments if eg._segments is not None else 0
            print(f"step {step + 1}: loss {name_a} {lg:.8f} eager {le:.8f}  grads equal {gsame}  params equal {psame}"
                  f"  local grads equal on all ranks {float(flags) == 0}"
                  f"  (graph segments {nseg}, buckets {len(eg.ddp.buckets)})", flush=True)
            if not gsame:
                for line in _named_diffs(eg, eg.flat.grad, ee.flat.grad):
                    print("   grad " + line, flush=True)
        ok = ok and gsame and psame and lg == le
    if graph_a:
        assert eg._segments is not None and eg._segments.num_segments > 1, "graph DP step was not segmented"
    return ok


def _graph_vs_eager(ctx, cfg, steps: int) -> bool:
    return _pair_vs(ctx, cfg, steps, True)


def main():
    ctx = pdist.init_distributed("cuda", backend="gloo")
    # no random ops, so the graph and eager runs see identical math (their RNG streams differ)
    cfg = rt1.RT1Config(height=128, width=128, seq_len=6, backend="hip", dropout_rate=0.0, drop_connect_rate=0.0,
                        crop_ratio=0.0)
    graph = "--graph" in sys.argv
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 4
    if graph or "--eager2" in sys.argv:
        ok = _pair_vs(ctx, cfg, steps, graph)
        pdist.shutdown()
        sys.exit(0 if ok else 2)
    eng, losses = _run(ctx, cfg, False, steps)
    flat = eng.flat.data
    hi, lo = flat.clone(), flat.clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    pdiff = float((hi - lo).abs().max())
    bufs = eng.ddp.buffers
    bdiff = 0.0
    if bufs is not None:
        bh, bl = bufs.clone(), bufs.clone()
        dist.all_reduce(bh, op=dist.ReduceOp.MAX)
        dist.all_reduce(bl, op=dist.ReduceOp.MIN)
        bdiff = float((bh - bl).abs().max())
    if ctx.rank == 0:
        print(f"losses {losses}  max |param diff| across ranks {pdiff:.3e}  buffer diff {bdiff:.3e}", flush=True)
    ok = pdiff == 0.0 and all(l == l for l in losses)
    pdist.shutdown()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
