"""Multi-rank entrypoints on CPU (gloo): ``bench.py --gpus N`` must really run N ranks, and the local launcher
must propagate a failing rank's exit code and stop the others."""
import json
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = dict(os.environ)
    env.pop("RANK", None)
    env.pop("WORLD_SIZE", None)
    env.pop("MASTER_PORT", None)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    return env


def test_bench_gpus2_spawns_two_ranks():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu", "--preset", "tiny",
           "--height", "64", "--width", "64", "--seq_len", "2", "--batch_per_gpu", "2", "--steps", "1",
           "--warmup", "1", "--dtype", "fp32"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout                      # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["config"]["parallelism"] == "dp2"
    assert out["config"]["global_batch"] == 4
    assert out["dist_backend"] == "gloo"
    assert out["value"] > 0


def test_bench_refuses_mismatched_world(tmp_path):
    # a launcher that says WORLD_SIZE=1 while --gpus 2 is asked for must fail loudly, not report 1 GPU as 2
    env = _env()
    env.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu", "--preset", "tiny",
           "--height", "64", "--width", "64", "--seq_len", "2", "--batch_per_gpu", "1", "--steps", "1",
           "--warmup", "0", "--dtype", "fp32"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode != 0
    assert "refusing" in (r.stderr + r.stdout)


def test_spawn_local_propagates_failure(tmp_path):
    script = tmp_path / "worker.py"
    script.write_text(textwrap.dedent("""
        import os, sys, time
        r = int(os.environ["RANK"])
        assert os.environ["WORLD_SIZE"] == "3" and os.environ["MASTER_ADDR"] == "127.0.0.1"
        if r == 1:
            sys.exit(7)
        time.sleep(120)     # would block forever in a collective; the launcher must stop it
    """))
    sys.path.insert(0, ROOT)
    from pytorch_rt1_for_distributed_training_amd.parallel.launch import spawn_local
    import time
    t0 = time.time()
    rc = spawn_local(3, [str(script)], grace_s=5.0)
    assert rc == 7
    assert time.time() - t0 < 60
