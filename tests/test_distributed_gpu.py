"""Data-parallel correctness of the hip backend on one GPU box.

* 2 ranks on cuda:0 over gloo (RCCL refuses two ranks on one device): eager bucketed DP keeps bit-identical ranks,
  and the segmented hipGraph DP step -- the path ``bench.py --gpus N`` runs -- is bitwise equal to eager DP.
* ``bench.py --gpus 2`` itself (gloo rehearsal): its JSON line, graph segmentation and cross-rank consistency check.
* a single-rank RCCL communicator (``comm="native"``) driving the whole bucketed DP path through ``TrainEngine``:
  RCCL collectives on the communicator's stream between graph-segment replays, against the plain graph step.
"""
import json
import os
import re
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _torchrun(script_args, port, timeout=600, env_extra=None):
    env = dict(os.environ, PYTHONPATH=ROOT, **(env_extra or {}))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port)] + script_args
    return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)


def test_dp_two_ranks_identical_params_hip_backend():
    r = _torchrun([os.path.join(ROOT, "tools", "dp_gpu_check.py")], 29547)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "max |param diff| across ranks 0.000e+00" in r.stdout


def test_graph_dp_bitwise_equals_eager_dp():
    """Segmented hipGraph DP (forward+backward as graph segments cut at bucket boundaries, each bucket's all-reduce
    issued between segment replays) vs eager bucketed DP on the same batches: flat gradients, parameters and losses
    bitwise equal after every step, with more than one segment."""
    r = _torchrun([os.path.join(ROOT, "tools", "dp_gpu_check.py"), "--graph"], 29548)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-4000:])
    steps = [ln for ln in r.stdout.splitlines() if ln.startswith("step ")]
    assert len(steps) == 4, r.stdout[-2000:]
    for ln in steps:
        assert "grads equal True" in ln and "params equal True" in ln, ln
        nseg = int(re.search(r"graph segments (\d+)", ln).group(1))
        assert nseg > 1, ln


def test_eager_dp_bitwise_reproducible_with_fused_se():
    """Two eager bucketed-DP engines on the same batches from the same state: flat gradients, parameters and losses
    bitwise equal for 8 steps, with the fused SE kernels on (the default for any world size).  Before the packed-fp32
    op_sel fix (profiles/r4_se_dp_rootcause.md) single SE fc1 weight gradients differed run to run here."""
    from pytorch_rt1_for_distributed_training_amd.ops import backbone
    assert backbone.se_fused_active()
    r = _torchrun([os.path.join(ROOT, "tools", "dp_gpu_check.py"), "--eager2", "--steps", "8"], 29546)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-4000:])
    steps = [ln for ln in r.stdout.splitlines() if ln.startswith("step ")]
    assert len(steps) == 8, r.stdout[-2000:]
    assert all("grads equal True" in ln and "params equal True" in ln for ln in steps), r.stdout[-3000:]


def test_bench_two_ranks_gloo_rehearsal():
    """``bench.py --gpus 2`` spawning its own ranks (gloo on one GPU): one JSON line for the whole job, the segmented
    graph step, and bit-identical parameters on both ranks after the timed steps."""
    env = dict(os.environ, PYTHONPATH=ROOT, RT1_DIST_BACKEND="gloo", MASTER_PORT="29549")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "2",
           "--batch_per_gpu", "16"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["dist_backend"] == "gloo"
    assert out["config"]["hipgraph"] is True
    assert out["config"]["graph_segments"] > 1
    assert out["config"]["ranks_consistent"] is True
    # the timed graph-DP step re-run against the eager bucketed DP step on one batch from the same state: bitwise
    assert out["config"]["graph_eq_eager"] is True, out["config"]["graph_eq_eager_detail"]
    assert len(out["config"]["rank_ms_per_step"]) == 2 and out["config"]["rank_spread_ms"] >= 0
    assert len(out["config"]["comm_exposed_ms_per_step"]) == 2
    assert out["config"]["step"] == "graph-dp" and out["config"]["graph_fallback"] is None
    bk = out["config"]["bucket_launch_to_ready_ms_rank0"]
    assert bk and all(b["launch_to_ready_ms"] >= 0 and b["mb"] > 0 for b in bk)
    assert "error" not in out
    assert out["value"] > 0 and out["steps"] == 2


def test_native_comm_single_rank_engine_matches_graph_step():
    """TrainEngine(comm='native') at world 1: a single-rank RCCL communicator runs the bucketed DP path (gradient
    hooks, segmented graph, RCCL all-reduce per bucket on its own stream, Adam after the last wait).  Losses and
    parameters must equal the plain one-graph step bitwise."""
    import pytorch_rt1_for_distributed_training_amd as rt1
    from pytorch_rt1_for_distributed_training_amd.data.synthetic import make_batch
    from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine
    from pytorch_rt1_for_distributed_training_amd.models import build_rt1
    cfg = rt1.RT1Config(height=128, width=128, seq_len=6, backend="hip", dropout_rate=0.0, drop_connect_rate=0.0,
                        crop_ratio=0.0)
    engines = []
    for comm in ("native", "torch"):
        torch.manual_seed(0)
        engines.append(TrainEngine(build_rt1(cfg), cfg, order_probe=True, bucket_cap_mb=4.0, comm=comm, graph=True))
    en, et = engines
    assert en.ddp.enabled and en.ddp.comm is not None and len(en.ddp.buckets) > 1
    assert not et.ddp.enabled
    g = torch.Generator().manual_seed(7)
    try:
        for step in range(4):
            batch = make_batch(4, cfg.seq_len, 128, 128, device="cuda", generator=g)
            ln, lt = float(en.train_step(batch)), float(et.train_step(batch))
            torch.cuda.synchronize()
            assert ln == lt, (step, ln, lt)
            assert torch.equal(en.flat.data, et.flat.data), step
        assert en._segments is not None and en._segments.num_segments > 1
        assert et._graph is not None
        assert not en.ddp.comm.timed_out
    finally:
        en.ddp.comm.destroy()


def _bench_gloo2(env_extra, port):
    env = dict(os.environ, PYTHONPATH=ROOT, RT1_DIST_BACKEND="gloo", MASTER_PORT=str(port), **env_extra)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "2",
           "--batch_per_gpu", "8", "--height", "128", "--width", "128"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0]), r.stderr


def test_bench_graph_mismatch_drops_captured_segments():
    """The fallback bench.py relies on, on the real path: the graph-DP segments ARE captured on both ranks, the forced
    graph == eager mismatch drops them (drop_graph: segments gone, gradients re-attached to the flat buffer) and the
    eager bucketed DP step is warmed up and timed; ranks stay bit-identical."""
    out, err = _bench_gloo2({"RT1_BENCH_TEST_GRAPH_MISMATCH": "1"}, 29551)
    cfg = out["config"]
    assert cfg["step"] == "eager-dp" and cfg["graph_fallback"] and cfg["hipgraph"] is False
    assert cfg["graph_eq_eager"] is False and cfg["graph_eq_eager_detail"]["forced_by_test_hook"]
    assert cfg["graph_segments"] == 0                                  # the captured segments are gone
    assert cfg["ranks_consistent"] is True and out["value"] > 0 and "error" not in out
    assert "timing the eager step instead" in err


def test_bench_capture_failure_on_one_rank_is_collective():
    """Rank 1's segmented capture raises (RT1_TEST_CAPTURE_FAIL=1): the capture decision is collective, so BOTH ranks
    continue with the eager bucketed DP step (no hang, no mismatched collectives) and stay bit-identical."""
    out, err = _bench_gloo2({"RT1_TEST_CAPTURE_FAIL": "1"}, 29552)
    cfg = out["config"]
    assert cfg["step"] == "eager-dp" and cfg["hipgraph"] is False and cfg["graph_segments"] == 0
    assert cfg["ranks_consistent"] is True and out["value"] > 0 and "error" not in out
    assert "every rank continues eagerly" in err


def test_drop_graph_on_captured_single_rank_engine():
    """drop_graph() on an engine whose segmented graph-DP step was captured (world-1 RCCL communicator): later steps
    run the eager hook-driven DP step and track an eager engine bitwise."""
    import pytorch_rt1_for_distributed_training_amd as rt1
    from pytorch_rt1_for_distributed_training_amd.data.synthetic import make_batch
    from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine
    from pytorch_rt1_for_distributed_training_amd.models import build_rt1
    cfg = rt1.RT1Config(height=128, width=128, seq_len=2, backend="hip", dropout_rate=0.0, drop_connect_rate=0.0,
                        crop_ratio=0.0)
    torch.manual_seed(0)
    en = TrainEngine(build_rt1(cfg), cfg, order_probe=True, bucket_cap_mb=4.0, comm="native", graph=True)
    torch.manual_seed(0)
    ee = TrainEngine(build_rt1(cfg), cfg, order_probe=True, graph=False)   # same flat layout (gradient-ready order)
    g = torch.Generator().manual_seed(3)
    try:
        for step in range(5):
            batch = make_batch(4, cfg.seq_len, 128, 128, device="cuda", generator=g)
            if step == 3:
                assert en._segments is not None and en._segments.num_segments > 1
                en.drop_graph()
                assert en._segments is None and not en.graph
            ln, le = float(en.train_step(batch)), float(ee.train_step(batch))
            torch.cuda.synchronize()
            assert ln == le, (step, ln, le)
            assert torch.equal(en.flat.data, ee.flat.data), step
    finally:
        en.ddp.comm.destroy()


def test_bench_single_rank_rccl_process_group_graph_dp():
    """RT1_PG_WORLD1=1: a ONE-rank torch process group over RCCL drives the exact N > 1 path of bench.py -- segmented
    hipGraph DP step, per-bucket ProcessGroup all-reduces issued between segment replays, graph == eager check,
    cross-rank fingerprint -- on the one GPU of this box (the N = 2..8 runs are the driver's)."""
    env = dict(os.environ, PYTHONPATH=ROOT, RT1_PG_WORLD1="1", MASTER_PORT="29583")
    env.pop("RANK", None)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "3", "--warmup", "2",
           "--batch_per_gpu", "8", "--height", "128", "--width", "128", "--bucket_cap_mb", "8"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    cfg = out["config"]
    assert out["dist_backend"] == "nccl" and out["rccl_world"] == 1 and out["comm"] == "torch"
    assert cfg["step"] == "graph-dp" and cfg["graph_segments"] > 1 and cfg["graph_fallback"] is None
    assert cfg["graph_eq_eager"] is True, cfg["graph_eq_eager_detail"]
    assert out["value"] is not None and out["value"] > 0 and "error" not in out
