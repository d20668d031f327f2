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
    assert out["config"]["ranks_consistent"] is True
    assert out["config"]["graph_eq_eager"] is None          # no captured graph on the CPU: nothing to compare
    assert len(out["config"]["rank_ms_per_step"]) == 2 and out["config"]["rank_spread_ms"] >= 0
    assert "error" not in out


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


def test_spawn_local_sigterm_tears_down_ranks(tmp_path):
    """SIGTERM sent to the launcher alone stops every rank (no orphans left in a collective) and exits 128+15."""
    worker = tmp_path / "worker.py"
    worker.write_text(textwrap.dedent("""
        import os, time
        open(os.path.join(os.environ["OUT"], "pid%s" % os.environ["RANK"]), "w").write(str(os.getpid()))
        time.sleep(300)
    """))
    parent = tmp_path / "parent.py"
    parent.write_text(textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {ROOT!r})
        from pytorch_rt1_for_distributed_training_amd.parallel.launch import spawn_local
        sys.exit(spawn_local(2, [{str(worker)!r}], grace_s=5.0))
    """))
    import signal
    import time
    env = _env()
    env["OUT"] = str(tmp_path)
    p = subprocess.Popen([sys.executable, str(parent)], env=env)
    pids = []
    deadline = time.time() + 60
    while time.time() < deadline and len(pids) < 2:
        pids = [tmp_path / f"pid{r}" for r in range(2) if (tmp_path / f"pid{r}").exists()]
        time.sleep(0.1)
    assert len(pids) == 2, "ranks did not start"
    time.sleep(0.3)
    child_pids = [int(f.read_text()) for f in pids]
    p.send_signal(signal.SIGTERM)
    assert p.wait(timeout=30) == 128 + signal.SIGTERM
    for cp in child_pids:
        for _ in range(50):
            try:
                os.kill(cp, 0)
            except ProcessLookupError:
                break
            time.sleep(0.1)
        else:
            raise AssertionError(f"rank pid {cp} survived the launcher's SIGTERM")
