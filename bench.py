#!/usr/bin/env python3
"""Headline benchmark: RT-1 train samples/sec for the whole node.

Metric and config come from BASELINE.json: full RT-1 (FiLM-EfficientNet-B3 +
TokenLearner + 8-layer transformer, 35.3M params), history T=6, 300x300
frames, bf16 compute, data-parallel over RCCL with a global batch of 1024 on 8
GPUs (128 windows per GPU; weak scaling).  Synthetic data of the real shapes,
random-init weights.  A timed step is the full training step: pinned uint8
host batch -> HBM copy (double-buffered), forward, backward, bucketed
all-reduce, fused Adam.

  python bench.py                                   # 1 GPU, defaults
  python bench.py --gpus N                          # spawns N local ranks itself (parallel/launch.py)
  torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

With ``--gpus N > 1`` and no launcher environment the parent process only parses arguments and starts N fresh
child ranks (it never touches the GPU); under torchrun the launcher's WORLD_SIZE must equal ``--gpus`` or the
run fails loudly.

Rank 0 prints ONE JSON line.  ``value`` = total samples/s over all ranks =
N * batch_per_gpu / max-over-ranks(step time).

Before timing, the captured step (one graph; the segmented graph-DP step with several ranks) is compared bitwise with
the eager step on one batch from one state on every rank; if any rank differs, every rank times the eager bucketed
step instead ("step": "eager-dp"), which is what ``distribute_train.py`` would then train with.  A stall watchdog
(``--stall_timeout``, below the process-group timeout ``--pg_timeout``, both below the driver's 600 s) turns a hung
collective into a JSON error record and exit code 4; ranks sharing one GPU under RCCL are refused (exit 5).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

METRIC = "train samples/sec (whole node), RT-1 Language-Table, 1/2/4/8 MI355X"
BASELINE_VALUE = None  # the reference publishes no throughput


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch_per_gpu", type=int, default=128)
    ap.add_argument("--height", type=int, default=300)
    ap.add_argument("--width", type=int, default=300)
    ap.add_argument("--seq_len", type=int, default=6)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--backend", default="auto", choices=["auto", "hip", "torch"])
    ap.add_argument("--bucket_cap_mb", type=float, default=32.0)
    ap.add_argument("--comm", choices=["torch", "native"], default="torch",
                    help="gradient collectives: torch ProcessGroup (RCCL) or the native C++ RCCL communicator")
    ap.add_argument("--device", default="auto")
    ap.add_argument("--graph", choices=["auto", "on", "off"], default="auto",
                    help="hipGraph step (auto = on): 1 GPU captures the whole step; with data parallelism the "
                         "forward+backward is captured and the RCCL all-reduce + Adam run after each replay")
    ap.add_argument("--profile_steps", type=int, default=0, help="extra per-phase timing report (stderr)")
    ap.add_argument("--no_check", action="store_true",
                    help="skip the post-run graph == eager step comparison (it runs after the timed region)")
    ap.add_argument("--pg_timeout", type=float, default=240.0,
                    help="process-group collective timeout (s), well under the driver's 600 s bench limit")
    ap.add_argument("--stall_timeout", type=float, default=150.0,
                    help="no progress for this long (s): rank 0 prints a one-line JSON error record and every rank "
                         "exits non-zero (a hung collective must still leave a record)")
    ap.add_argument("--preset", default="full", choices=["full", "tiny"],
                    help="full = BASELINE RT-1; tiny = RT-1-tiny plumbing config (2 layers; CPU rehearsals only)")
    return ap.parse_args()


class Heartbeat:
    """Per-rank stall watchdog.  ``beat(phase)`` marks progress; a daemon thread checks it every few seconds.  After
    ``timeout`` s without a beat, rank 0 prints ONE JSON line (``value`` null, ``error`` naming the phase it stalled
    in) and every rank leaves with exit code 4 through ``os._exit`` -- a collective that never returns (a hung RCCL
    ring, a rank that died) cannot be interrupted from Python, but the process can still end with a record.  Ranks
    other than 0 wait ``grace`` s longer so rank 0's record is written first."""

    def __init__(self, timeout: float, rank: int, record, grace: float = 20.0):
        import threading
        self.timeout = float(timeout)
        self.limit = self.timeout + (0.0 if rank == 0 else grace)
        self.rank = rank
        self.record = record                # callable(phase, stalled_s) -> dict (rank 0 prints it)
        self.phase = "start"
        self.t = time.monotonic()
        self._stop = threading.Event()
        if self.timeout > 0:
            threading.Thread(target=self._run, daemon=True, name="bench-stall-watchdog").start()

    def beat(self, phase: str):
        self.phase = phase
        self.t = time.monotonic()

    def stop(self):
        self._stop.set()

    def _run(self):
        while not self._stop.wait(min(5.0, max(0.5, self.timeout / 10))):
            stalled = time.monotonic() - self.t
            if stalled > self.limit:
                if self.rank == 0:
                    try:
                        print(json.dumps(self.record(self.phase, stalled)), flush=True)
                    except Exception as e:           # never let the record itself keep the process alive
                        print(json.dumps({"metric": METRIC, "value": None, "error": f"stalled in {self.phase}; "
                                          f"record failed: {e}"}), flush=True)
                print(f"[bench] rank {self.rank}: no progress for {stalled:.0f} s in phase '{self.phase}': exiting 4",
                      file=sys.stderr, flush=True)
                os._exit(4)


def _test_stall(phase: str, rank: int):
    """Test hook (CPU rehearsals): RT1_BENCH_TEST_STALL=<rank>:<phase> parks that rank forever at that phase, the way
    a rank stuck in a collective looks to the others."""
    spec = os.environ.get("RT1_BENCH_TEST_STALL")
    if spec:
        r, ph = spec.split(":", 1)
        if int(r) == rank and ph == phase:
            print(f"[bench] test hook: rank {rank} stalls at {phase}", file=sys.stderr, flush=True)
            while True:
                time.sleep(3600)


def device_identity(dev) -> str:
    """A string that differs between physical GPUs: the UUID where torch exposes it, else the PCI location."""
    import torch
    if dev.type != "cuda":
        return "cpu"
    p = torch.cuda.get_device_properties(dev)
    uuid = getattr(p, "uuid", None)
    if uuid is not None and str(uuid).strip("0-") != "":
        return f"uuid:{uuid}"
    return "pci:{}:{}:{}".format(getattr(p, "pci_domain_id", "?"), getattr(p, "pci_bus_id", "?"),
                                 getattr(p, "pci_device_id", "?"))


def main():
    a = parse()
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    if a.gpus > 1 and "RANK" not in os.environ:
        # no launcher: become one process per GPU before anything initialises HIP in this process
        from pytorch_rt1_for_distributed_training_amd.parallel.launch import spawn_local
        sys.exit(spawn_local(a.gpus, [os.path.abspath(__file__)] + sys.argv[1:]))
    from pytorch_rt1_for_distributed_training_amd.utils.tuned_gemms import enable_tuned_gemms
    tuned = enable_tuned_gemms()          # recorded hipBLASLt solutions for the remaining library GEMMs
    import torch
    import torch.distributed as dist

    from pytorch_rt1_for_distributed_training_amd.config import RT1Config
    from pytorch_rt1_for_distributed_training_amd.data.prefetch import DevicePrefetcher
    from pytorch_rt1_for_distributed_training_amd.data.synthetic import SyntheticStream
    from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine
    from pytorch_rt1_for_distributed_training_amd.models import build_rt1
    from pytorch_rt1_for_distributed_training_amd.parallel import dist as pdist

    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")   # a failed / timed-out RCCL op ends the rank
    state = {"phase": "init"}

    def stall_record(phase, stalled):
        return {"metric": METRIC, "value": None, "unit": "samples/s", "n_gpus": a.gpus, "steps": a.steps,
                "warmup": a.warmup, "ms_per_step": None, "higher_is_better": True, "scaling": "weak",
                "vs_baseline": None, "dtype": a.dtype, "data": "synthetic",
                "config": {"global_batch": a.gpus * a.batch_per_gpu, "batch_per_gpu": a.batch_per_gpu,
                           "seq_len": a.seq_len, "image": [a.height, a.width], "parallelism": f"dp{a.gpus}"},
                "error": f"no progress for {stalled:.0f} s in phase '{phase}' (collective hang or dead rank); "
                         f"stall_timeout {a.stall_timeout} s, pg_timeout {a.pg_timeout} s"}
    hb = Heartbeat(a.stall_timeout, int(os.environ.get("RANK", 0)), stall_record)
    ctx = pdist.init_distributed(a.device, timeout_s=int(a.pg_timeout))
    world = ctx.world_size
    hb.beat("device check")
    _test_stall("init", ctx.rank)
    # rank -> device: every RCCL rank must own a different physical GPU (a launcher that maps two ranks onto one card
    # would otherwise produce a "scaling" number from a shared GPU)
    ids = pdist.all_gather_objects(device_identity(ctx.device))
    if ctx.backend == "nccl" and len(set(ids)) != len(ids):
        if ctx.is_main:
            print(json.dumps(dict(stall_record("device check", 0.0), error=f"ranks share a GPU: {ids}")), flush=True)
        hb.stop()
        sys.exit(5)
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but the process group has {world} ranks "
                         f"(WORLD_SIZE={os.environ.get('WORLD_SIZE')}); refusing to report a mislabelled number")
    if world > 1:
        assert dist.is_initialized() and dist.get_world_size() == a.gpus
    extra = {}
    if a.preset == "tiny":
        extra = dict(num_layers=2, channels_last=False)
    cfg = RT1Config(height=a.height, width=a.width, seq_len=a.seq_len, dtype=a.dtype, backend=a.backend,
                    **extra)
    torch.manual_seed(0)
    model = build_rt1(cfg)
    use_graph = a.graph in ("on", "auto")
    dp_path = world > 1 or pdist.pg_world1()     # RT1_PG_WORLD1=1: the N > 1 path on a one-rank process group
    engine = TrainEngine(model, cfg, bucket_cap_mb=a.bucket_cap_mb, order_probe=dp_path or a.comm == "native",
                         comm=a.comm, graph=use_graph)
    if "comminit" in os.environ.get("RT1_DP_DIAG", "") and ctx.device.type == "cuda":
        # diagnostic: an idle single-rank RCCL communicator beside the one-graph step (does RCCL's init alone cost?)
        from pytorch_rt1_for_distributed_training_amd.parallel.native_comm import NativeComm
        state["idle_comm"] = NativeComm.single(ctx.device.index)
    stream = SyntheticStream(a.batch_per_gpu, cfg.seq_len, cfg.height, cfg.width, ring=2, uint8=True,
                             seed=ctx.rank)
    batches = iter(DevicePrefetcher(stream, ctx.device, depth=2))

    def sync():
        if ctx.device.type == "cuda":
            torch.cuda.synchronize()

    def progress(msg):
        if ctx.is_main:
            print(msg, file=sys.stderr, flush=True)

    def warm(n, tag):
        for i in range(n):
            hb.beat(f"{tag} {i + 1}/{n}")
            t1 = time.perf_counter()
            engine.train_step(next(batches))
            sync()
            progress(f"[bench] {tag} {i + 1}/{n}: {1e3 * (time.perf_counter() - t1):.1f} ms")
        sync()

    warm(a.warmup, "warmup")
    # the step to time must be the step training would run: the captured graph (graph-DP with several ranks) is
    # compared with the eager step on one batch from one snapshotted state, bitwise, on every rank, BEFORE timing.
    # If any rank differs, every rank drops the graph (engine.drop_graph, as Trainer._check_graph does) and the
    # eager bucketed step is warmed up and timed instead, labelled "step": "eager-dp"
    check = None
    if not a.no_check and engine.graph:
        from pytorch_rt1_for_distributed_training_amd.engine.step import _clone_tree
        hb.beat("graph == eager check")
        b = next(batches)
        sync()
        check = engine.graph_eager_check(_clone_tree(b))
    fake_mismatch = os.environ.get("RT1_BENCH_TEST_GRAPH_MISMATCH") == "1"     # test hook: force the fallback
    if fake_mismatch:
        check = dict(check or {}, equal=False, forced_by_test_hook=True)
    graph_eq_eager = None if check is None else pdist.all_true(check["equal"])
    fallback = graph_eq_eager is False
    if fallback:
        progress("[bench] the graph step differs from the eager step: timing the eager step instead")
        engine.drop_graph()
        warm(max(1, min(a.warmup, 2)), "eager warmup")
    timed_graph = engine.graph
    dp_step = engine.ddp.enabled
    step_kind = ("graph-dp" if dp_step else "graph") if timed_graph else ("eager-dp" if dp_step else "eager")
    hb.beat("pre-timing barrier")
    pdist.barrier()
    sync()
    if engine.ddp.enabled and engine.graph and "notiming" not in os.environ.get("RT1_DP_DIAG", ""):
        engine.comm_timing = []
    _test_stall("timed", ctx.rank)
    t0 = time.perf_counter()
    for i in range(a.steps):
        hb.beat(f"timed step {i + 1}/{a.steps}")
        loss = engine.train_step(next(batches))
        if a.steps <= 20 or (i + 1) % 10 == 0:
            progress(f"[bench] step {i + 1}/{a.steps} issued at {1e3 * (time.perf_counter() - t0):.1f} ms")
    hb.beat("timed sync")
    sync()
    t_rank = time.perf_counter() - t0           # this rank's own time, before the closing barrier
    hb.beat("closing barrier")
    pdist.barrier()
    sync()
    dt_local = time.perf_counter() - t0
    dt = pdist.all_reduce_max(dt_local)
    final_loss = float(loss)
    hb.beat("report")
    comm = None
    buckets = None
    if engine.comm_timing is not None:
        exposed = sum(e0.elapsed_time(e1) for e0, e1 in engine.comm_timing) / max(1, len(engine.comm_timing))
        comm = (exposed, 1e3 * engine.comm_host_wait_s / a.steps)
        engine.comm_timing = None
        buckets = engine.bucket_report()
    per_rank = pdist.all_gather_floats([1e3 * t_rank / a.steps] + list(comm or (0.0, 0.0)))
    # after the timed region: every rank must hold bit-identical parameters (a strided fingerprint of the flat
    # fp32 buffer compared by all-reduce MAX / MIN), the end-to-end check of the data-parallel path that ran
    consistent = None
    if world > 1:
        fp = engine.flat.data[::1021].clone()
        hi, lo = fp.clone(), fp.clone()
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        consistent = bool(torch.equal(hi, lo))
    ms = 1e3 * dt / a.steps
    value = world * a.batch_per_gpu * a.steps / dt
    errors = []
    if consistent is False:
        errors.append("ranks hold different parameters after the timed steps")

    if ctx.is_main:
        step_ms = [r[0] for r in per_rank]
        out = {
            "metric": METRIC,
            "value": None if errors else round(value, 3),
            "unit": "samples/s",
            "n_gpus": world,
            # ranks in the RCCL communicator (0 = the collectives ran on another backend, e.g. a gloo rehearsal)
            "rccl_world": world if ctx.backend == "nccl" else (1 if (world == 1 and ctx.device.type == "cuda") else 0),
            "dist_backend": ctx.backend or "none",
            # world 1 with --comm native: the segmented graph-DP step over a single-rank RCCL communicator
            "comm": a.comm if (world > 1 or engine.ddp.enabled) else "none",
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (value / BASELINE_VALUE) if BASELINE_VALUE else None,
            "dtype": a.dtype,
            "data": "synthetic (uint8 frames + 512-d text emb + action labels of the real shapes; random-init weights)",
            "config": {"model": ("RT-1 (FiLM-EfficientNet-B3 + TokenLearner-8 + 8-layer transformer, 35.3M params)"
                                 if a.preset == "full" else "RT-1-tiny (2-layer transformer; plumbing rehearsal)"),
                       "global_batch": world * a.batch_per_gpu, "batch_per_gpu": a.batch_per_gpu,
                       "seq_len": cfg.seq_len, "tokens": cfg.seq_len * 11, "image": [a.height, a.width],
                       "parallelism": f"dp{world}", "backend": engine.backend, "hipgraph": timed_graph,
                       "step": step_kind,
                       "graph_fallback": (("the captured step differed from the eager step on the check batch; the "
                                           "eager step was timed (what training runs)") if fallback else None),
                       "graph_segments": (engine._segments.num_segments if engine._segments is not None else
                                          (1 if engine._graph is not None else 0)),
                       "ranks_consistent": consistent,
                       "graph_eq_eager": graph_eq_eager,
                       "graph_eq_eager_detail": check,
                       "rank_ms_per_step": [round(x, 3) for x in step_ms],
                       "rank_spread_ms": round(max(step_ms) - min(step_ms), 3),
                       "comm_exposed_ms_per_step": ([round(r[1], 3) for r in per_rank] if comm is not None
                                                    else None),
                       "comm_host_wait_ms_per_step": ([round(r[2], 3) for r in per_rank] if comm is not None
                                                      else None),
                       "bucket_launch_to_ready_ms_rank0": buckets,
                       "rank_devices": ids,
                       "pg_timeout_s": a.pg_timeout, "stall_timeout_s": a.stall_timeout,
                       "tuned_library_gemms": tuned,
                       "frames_per_sec": round(value * cfg.seq_len, 1), "final_loss": final_loss},
        }
        if errors:
            out["error"] = "; ".join(errors)
            out["measured_value_unvalidated"] = round(value, 3)
        print(json.dumps(out), flush=True)
    hb.stop()
    pdist.shutdown()
    if errors:
        sys.exit(3)


if __name__ == "__main__":
    main()
