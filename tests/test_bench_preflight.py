"""bench.py's multi-rank pre-flight on CPU (gloo, 2 ranks, RT-1-tiny): whatever happens in the first multi-GPU run,
the driver must get ONE JSON line.  (1) A rank that stalls (the way a rank stuck in a collective looks to the others)
ends the job with exit code 4 and a JSON error record naming the phase, before the process-group timeout.  (2) When
the timed step's graph == eager check fails, every rank times the eager bucketed DP step and labels it."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BASE = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu", "--preset", "tiny",
        "--batch_per_gpu", "2", "--height", "64", "--width", "64", "--seq_len", "2", "--steps", "2", "--warmup", "1",
        "--bucket_cap_mb", "1"]


def _run(extra_args, extra_env, timeout=240):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    env.pop("RANK", None)
    env.update(extra_env)
    t0 = time.time()
    r = subprocess.run(BASE + extra_args, env=env, capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, lines, time.time() - t0


def test_bench_stalled_rank_leaves_json_record():
    r, lines, dt = _run(["--stall_timeout", "12", "--pg_timeout", "120"], {"RT1_BENCH_TEST_STALL": "1:timed"})
    assert r.returncode != 0, r.stdout[-2000:]
    assert len(lines) == 1, (r.stdout[-2000:], r.stderr[-3000:])
    out = json.loads(lines[0])
    assert out["value"] is None and "no progress" in out["error"], out
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert dt < 110, dt          # ended by the stall watchdog, not by the 120 s process-group timeout


def test_bench_graph_mismatch_times_eager_dp():
    r, lines, _ = _run([], {"RT1_BENCH_TEST_GRAPH_MISMATCH": "1"})
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["value"] is not None and out["value"] > 0 and "error" not in out
    cfg = out["config"]
    assert cfg["step"] == "eager-dp" and cfg["graph_eq_eager"] is False and cfg["graph_fallback"]
    assert cfg["ranks_consistent"] is True and cfg["rank_devices"] == ["cpu", "cpu"]


BASE8 = [a if a != "2" or i != 3 else "8" for i, a in enumerate(BASE)]     # --gpus 8


def _run8(extra_args, extra_env, timeout=400):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    env.pop("RANK", None)
    env.update(extra_env)
    t0 = time.time()
    r = subprocess.run(BASE8 + extra_args, env=env, capture_output=True, text=True, timeout=timeout)
    return r, [ln for ln in r.stdout.splitlines() if ln.startswith("{")], time.time() - t0


def test_bench_eight_ranks_rehearsal():
    """The N=8 launch shape on CPU (gloo, 8 local ranks, RT-1-tiny): bench.py spawns the ranks itself, rank 0 prints
    ONE JSON line with the whole-job value, dp8, one device entry and one step time per rank, and the ranks hold
    bit-identical parameters after the timed steps (no hipGraph on CPU: graph_segments 0, the eager bucketed step)."""
    assert BASE8[3] == "8"
    r, lines, _ = _run8([], {})
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    cfg = out["config"]
    assert out["n_gpus"] == 8 and cfg["parallelism"] == "dp8" and cfg["global_batch"] == 16
    assert out["value"] is not None and out["value"] > 0 and "error" not in out
    assert cfg["ranks_consistent"] is True and cfg["graph_segments"] == 0 and cfg["step"] == "eager-dp"
    assert len(cfg["rank_ms_per_step"]) == 8 and cfg["rank_devices"] == ["cpu"] * 8
    assert out["dist_backend"] == "gloo"


def test_bench_eight_ranks_stall_on_last_rank():
    """Rank 7 of 8 hangs in the timed region (the way a rank stuck in a collective looks to the others): the stall
    watchdog still leaves exactly one JSON error record from rank 0 and a non-zero exit, before the pg timeout."""
    r, lines, dt = _run8(["--stall_timeout", "15", "--pg_timeout", "150"], {"RT1_BENCH_TEST_STALL": "7:timed"})
    assert r.returncode != 0, r.stdout[-2000:]
    assert len(lines) == 1, (r.stdout[-2000:], r.stderr[-3000:])
    out = json.loads(lines[0])
    assert out["value"] is None and "no progress" in out["error"] and out["n_gpus"] == 8, out
    assert dt < 140, dt


def test_bench_single_rank_process_group_runs_dp_path():
    """RT1_PG_WORLD1=1 (the one-GPU rehearsal of the N > 1 path): a one-rank torch process group is created and the
    bucketed DP step runs on it -- gradient hooks, per-bucket all-reduces through the process group -- labelled
    comm torch / eager-dp, on CPU gloo here (RCCL on the GPU box: tests/test_distributed_gpu.py)."""
    BASE1 = [a if a != "2" or i != 3 else "1" for i, a in enumerate(BASE)]     # --gpus 1
    assert BASE1[3] == "1"
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2", RT1_PG_WORLD1="1", MASTER_PORT="29581")
    env.pop("RANK", None)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run(BASE1, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    cfg = out["config"]
    assert out["n_gpus"] == 1 and cfg["parallelism"] == "dp1" and out["dist_backend"] == "gloo"
    assert out["comm"] == "torch" and cfg["step"] == "eager-dp"
    assert out["value"] is not None and out["value"] > 0 and "error" not in out
