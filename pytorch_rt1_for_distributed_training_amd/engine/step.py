"""One optimisation step of RT-1 (forward, backward, DP all-reduce, Adam).

Replaces ``RT1_Lightning.training_step`` + Lightning's automatic optimisation
(``distribute_train.py:59-73,99-118``).  Per step:

1. ``ddp.prepare()``  — reset bucket counters, (optionally) broadcast BN buffers;
2. forward under the compute dtype (bf16 on MI355X), loss = mean of the
   per-(b,t) actor loss exactly as ``loss_fn`` (``:112-118``);
3. backward — bucket all-reduces fire from gradient hooks while the rest of
   the backward runs;
4. ``ddp.finish()`` then ONE fused Adam launch over the flat buffer with the
   1/world average folded in.

``graph=True`` (hip backend, one GPU) runs the whole step -- forward, backward,
gradient gather and Adam -- as ONE captured hipGraph (``torch.cuda.CUDAGraph``
is hipGraph on ROCm): the first call runs an eager step and captures, later
calls copy the batch into the static input buffers and replay.  Everything the
step needs from the host is device-resident: the random-shift offsets and
drop-path masks come from torch's graph-safe RNG, dropout seeds from the
``ops.rng`` device counter, Adam's step/lr from ``FlatAdam.dev_state``.
With data parallelism (``graph=True``, world > 1) forward + backward is captured as a CHAIN of graphs cut where
each gradient bucket completes (``engine.graphs.SegmentedCapture``); a step replays segment i, issues bucket i's
RCCL all-reduce on the comm stream, replays segment i+1 while that all-reduce runs, ... then one fused Adam
launch.  Collectives are never captured; they overlap the backward exactly where DDP's hooks would fire them.

No ``network_state`` is fabricated (the reference samples a random one on the
CPU and copies it to the GPU every step only to read its shape).
"""
from __future__ import annotations

import contextlib
import time
from typing import Dict, Optional

import torch
import torch.nn as nn

from ..config import RT1Config
from ..parallel import dist as pdist
from ..parallel.ddp import DataParallel, gradient_ready_order
from ..parallel.flat import deferred_sums
from ..parallel.flat import FlatParameters
from .optim import FlatAdam, multistep_lr


def split_batch(batch: Dict) -> tuple:
    obs = batch["train_observation"]
    return obs["image"], obs.get("natural_language_embedding"), batch["action_label"]


def _clone_tree(batch):
    if isinstance(batch, dict):
        return {k: _clone_tree(v) for k, v in batch.items()}
    return batch.clone() if isinstance(batch, torch.Tensor) else batch


def _copy_into(dst, src):
    if isinstance(dst, dict):
        for k in dst:
            _copy_into(dst[k], src[k])
    elif isinstance(dst, torch.Tensor):
        dst.copy_(src, non_blocking=True)


def _same_shapes(a, b) -> bool:
    if isinstance(a, dict):
        return isinstance(b, dict) and a.keys() == b.keys() and all(_same_shapes(a[k], b[k]) for k in a)
    if isinstance(a, torch.Tensor):
        return isinstance(b, torch.Tensor) and a.shape == b.shape and a.dtype == b.dtype
    return True


def to_device(batch, device, non_blocking=True):
    if isinstance(batch, dict):
        return {k: to_device(v, device, non_blocking) for k, v in batch.items()}
    if isinstance(batch, torch.Tensor):
        return batch.to(device, non_blocking=non_blocking)
    return batch


def synthetic_probe_batch(cfg: RT1Config, b: int, device) -> Dict:
    return {"train_observation": {"image": torch.rand(b, cfg.seq_len, 3, cfg.height, cfg.width, device=device),
                                  "natural_language_embedding": torch.randn(b, cfg.seq_len, 512, device=device)},
            "action_label": {"terminate_episode": torch.zeros(b, cfg.seq_len, dtype=torch.long, device=device),
                             "action": torch.zeros(b, cfg.seq_len, 2, device=device)}}


# Diagnostic knobs of the graph-DP step (RT1_DP_DIAG, comma list; for same-box A/B of its per-step costs only):
#   nosync   -- no per-step BN-buffer broadcast before the replay
#   noreduce -- no bucket all-reduces (world 1 only: the sums are the identity there)
#   relaxed1 -- the one-graph step captured in relaxed mode (as the graph-DP segments are)
#   globalseg -- the graph-DP segments captured in global mode
#   emptycache -- empty_cache() before the segmented capture
_DP_DIAG = set(filter(None, __import__("os").environ.get("RT1_DP_DIAG", "").split(",")))


def _test_capture_failure():
    """Test hook (GPU rehearsals): RT1_TEST_CAPTURE_FAIL=<rank> makes that rank's segmented capture raise, so the
    collective capture decision and the eager fallback of every rank are exercised."""
    import os
    r = os.environ.get("RT1_TEST_CAPTURE_FAIL")
    if r is not None and torch.distributed.is_initialized() and int(r) == torch.distributed.get_rank():
        raise RuntimeError("capture failure forced by RT1_TEST_CAPTURE_FAIL")


class TrainEngine:
    def __init__(self, model: nn.Module, cfg: RT1Config, lr: float = 5e-4, milestones=(50, 75, 90),
                 gamma: float = 0.1, weight_decay: float = 0.0, bucket_cap_mb: float = 32.0,
                 broadcast_buffers: bool = True, device: Optional[torch.device] = None,
                 grad_comm_dtype: torch.dtype = torch.float32, order_probe: bool = True, comm: str = "torch",
                 graph: bool = False):
        ctx = pdist.context()
        self.cfg = cfg
        self.device = device or pdist.default_device()
        self.model = model.to(self.device)
        self.compute_dtype = torch.bfloat16 if (cfg.dtype == "bf16" and self.device.type == "cuda") else torch.float32
        self.backend = self._select_backend(cfg)
        if self.backend == "hip":
            from ..ops import install
            install(self.model, cfg)
        elif self.device.type == "cuda" and cfg.channels_last:
            self.model._image_tokenizer.to(memory_format=torch.channels_last)

        trainable = [p for p in self.model.parameters() if p.requires_grad]
        if order_probe:
            order = self._gradient_order(trainable)
        else:
            order = list(reversed(trainable))
        self.flat = FlatParameters(order, device=self.device)
        # weight-gradient split-K sums folded into the flat gather (parallel/flat.py deferred_sums): one backward per
        # step into an fp32 gradient buffer on the GPU
        self._defer_sums = self.flat.grad.is_cuda and self.flat.grad.dtype == torch.float32
        fused = getattr(self.model, "fused", None)
        if fused is not None and hasattr(fused, "attach_flat"):
            fused.attach_flat(self.flat)
        native = None
        if comm == "native":
            if self.device.type != "cuda":
                raise ValueError("comm='native' (RCCL) needs GPU tensors")
            from ..parallel.native_comm import NativeComm
            dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
            # world 1: a single-rank RCCL communicator, so the bucketed DP path runs (and is testable) on one GPU
            native = (NativeComm(device=dev_index) if ctx.world_size > 1 else NativeComm.single(dev_index))
        elif comm not in ("torch", "native"):
            raise ValueError(f"unknown comm backend {comm!r}")
        self.ddp = DataParallel(self.model, self.flat, bucket_cap_mb=bucket_cap_mb,
                                broadcast_buffers=broadcast_buffers, grad_comm_dtype=grad_comm_dtype, comm=native)
        self.optimizer = FlatAdam(self.flat, lr=lr, weight_decay=weight_decay,
                                  all_params=list(self.model.parameters()))
        self.scheduler = multistep_lr(self.optimizer, list(milestones), gamma)
        self.global_step = 0
        # one GPU: the whole step is one graph; data parallel: forward+backward is the graph, the gradient
        # all-reduce and Adam run after each replay (collectives are never captured)
        self.graph = bool(graph) and self.backend == "hip" and self.device.type == "cuda"
        self._graph = None
        self._segments = None      # SegmentedCapture of the data-parallel graph step
        self._static_batch = None
        self._static_loss = None
        # graph-DP comm timing (bench.py): (event before the final waits, event after) per replayed step
        self.comm_timing = None
        self.comm_host_wait_s = 0.0
        self.bucket_timing = []    # per replayed step: [(bucket, launch event, ready event)] while comm_timing is on

    # ------------------------------------------------------------------ setup helpers
    def _select_backend(self, cfg: RT1Config) -> str:
        if cfg.backend == "torch" or self.device.type != "cuda":
            return "torch"
        if cfg.backend == "hip":
            return "hip"
        from ..ops import available
        return "hip" if available() else "torch"

    def _gradient_order(self, trainable):
        """Probe gradient-ready order on rank 0 with a 1-sample batch; broadcast it."""
        index = {id(p): i for i, p in enumerate(trainable)}
        order_idx = None
        if pdist.context().is_main:
            probe = synthetic_probe_batch(self.cfg, 1, self.device)

            def run():
                with self.autocast():
                    loss, _ = self.model.train_forward(*split_batch(probe), with_aux=False)
                loss.mean().backward()
            was = self.model.training
            self.model.train()
            order = gradient_ready_order(self.model, run, trainable)
            self.model.train(was)
            order_idx = [index[id(p)] for p in order]
        order_idx = pdist.broadcast_object(order_idx)
        return [trainable[i] for i in order_idx]

    def autocast(self):
        if self.compute_dtype == torch.float32 or self.backend == "hip":
            return contextlib.nullcontext()
        return torch.autocast(device_type=self.device.type, dtype=self.compute_dtype)

    # ------------------------------------------------------------------ steps
    def forward_loss(self, batch: Dict):
        images, ctx, actions = split_batch(batch)
        with self.autocast():
            loss_bt, aux = self.model.train_forward(images, ctx, actions, with_aux=False)
        return loss_bt.mean(), aux

    def _step_body(self, batch: Dict) -> torch.Tensor:
        self.model.train()
        self.ddp.prepare()
        self.optimizer.zero_grad()
        loss, _ = self.forward_loss(batch)
        with deferred_sums(self._defer_sums):
            loss.backward()
        self.ddp.finish()
        self.optimizer.step(grad_scale=self.ddp.grad_scale)
        return loss.detach()

    def train_step(self, batch: Dict) -> torch.Tensor:
        if self.graph and self._static_batch is not None and not _same_shapes(self._static_batch, batch):
            # a batch of another shape (e.g. a short last batch) cannot replay the captured graph: run it eagerly
            loss = self._step_body(batch)
            self.optimizer._dev_step = None            # the eager Adam advanced the device state; re-sync next replay
            self.global_step += 1
            return loss
        if self.graph and self.ddp.enabled:
            return self._graph_dp_step(batch)
        if self.graph:
            return self._graph_step(batch)
        loss = self._step_body(batch)
        self.global_step += 1
        return loss

    # ------------------------------------------------------------------ hipGraph step
    def _graph_step(self, batch: Dict) -> torch.Tensor:
        if self._graph is None:
            loss = self._step_body(batch)            # real step, also warms up lazily-initialised state
            self.global_step += 1
            try:
                self._capture(batch)
            except Exception as e:   # capture is an optimisation: never lose the run to it
                import sys
                print(f"[rt1] hipGraph capture failed ({type(e).__name__}: {e}); continuing eagerly",
                      file=sys.stderr, flush=True)
                self.graph = False
                self._graph = None
            return loss
        _copy_into(self._static_batch, batch)
        opt = self.optimizer
        if opt._dev_lr != float(opt.param_groups[0]["lr"]) or opt._dev_step != opt.step_count:
            opt.sync_device_state()
        self._graph.replay()
        opt.step_count += 1
        opt._dev_step = opt.step_count
        self.global_step += 1
        return self._static_loss.clone()

    def _capture(self, batch: Dict):
        self._static_batch = _clone_tree(batch)
        torch.cuda.synchronize(self.device)
        self.optimizer.sync_device_state()
        g = torch.cuda.CUDAGraph()
        steps_before = self.optimizer.step_count
        try:
            with torch.cuda.graph(g, capture_error_mode="relaxed" if "relaxed1" in _DP_DIAG else "global"):
                self._static_loss = self._step_body(self._static_batch)
        finally:
            # the capture recorded the step; it did not run it (restore even when the capture failed, so an eager
            # fallback continues from the right Adam step and re-syncs the device copy)
            self.optimizer.step_count = steps_before
            self.optimizer._dev_step = None
        self.optimizer.sync_device_state()
        self._graph = g

    # ------------------------------------------------------------------ hipGraph data-parallel step
    def _graph_dp_step(self, batch: Dict) -> torch.Tensor:
        if self._segments is None:
            loss = self._step_body(batch)            # eager step (bucketed, overlapped DP) warms everything up
            self.global_step += 1
            err = None
            try:
                _test_capture_failure()
                self._capture_segments(batch)
            except Exception as e:
                err = e
            # capture success is a COLLECTIVE decision: a rank whose capture failed runs eager steps, whose bucket
            # all-reduces are issued from hooks in a different order and count than the graph-DP replay's, so every
            # rank must take the same path or the collectives stop lining up (summing buckets of different steps, or
            # hanging).  No collective runs during the capture itself, so every rank reaches this all-reduce.
            if not pdist.all_true(err is None):
                import sys
                why = f"{type(err).__name__}: {err}" if err is not None else "failed on another rank"
                print(f"[rt1] segmented hipGraph capture {why}; every rank continues eagerly", file=sys.stderr,
                      flush=True)
                self.drop_graph()
            return loss
        _copy_into(self._static_batch, batch)
        if "nosync" not in _DP_DIAG:
            self.ddp.sync_buffers()                  # rank-0 BN buffers before the forward (DDP parity)
        works = []
        timing = self.comm_timing is not None
        launched = []                                # (bucket indices, event after the segment that completed them)

        def on_buckets(buckets):
            if "noreduce" in _DP_DIAG and self.ddp.world == 1:
                return
            works.extend(self.ddp.launch_bucket(b) for b in buckets)
            if timing:
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
                launched.append((list(buckets), ev))
        # segment i replays on the compute stream; bucket i's all-reduce then runs on the comm stream while
        # segment i+1 computes
        self._segments.replay_with(on_buckets)
        if timing:
            # exposed communication: compute-stream time between the last segment and the end of the last wait;
            # per bucket: its launch point (end of the segment that completed it) -> the compute stream passing its
            # wait (an upper bound on the all-reduce: max(backward left, all-reduce))
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
            h0 = time.perf_counter()
            done = []
            for w in works:
                if w is not None:
                    w.wait()
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
                done.append(ev)
            self.comm_host_wait_s += time.perf_counter() - h0
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            self.comm_timing.append((e0, e1))
            per_bucket = []
            k = 0
            for buckets, ev in launched:
                for b in buckets:
                    per_bucket.append((b, ev, done[k]))
                    k += 1
            self.bucket_timing.append(per_bucket)
        else:
            self.ddp.wait_all(works)
        self.optimizer.step(grad_scale=self.ddp.grad_scale)
        self.global_step += 1
        return self._static_loss.clone()

    def _capture_segments(self, batch: Dict):
        from .graphs import SegmentedCapture
        import gc
        self._static_batch = _clone_tree(batch)
        torch.cuda.synchronize(self.device)
        gc.collect()
        if "emptycache" in _DP_DIAG:
            # diagnostic: as torch.cuda.graph does before a capture (measured 0.3-0.6 ms/step SLOWER for the
            # segments, profiles/r6_graph_dp_world1.log)
            torch.cuda.empty_cache()
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        seg = SegmentedCapture(side, mode="global" if "globalseg" in _DP_DIAG else "relaxed")
        seg.expected_last = len(self.ddp.buckets)
        try:
            with torch.cuda.stream(side):
                seg.begin()
                self.model.train()
                self.optimizer.zero_grad()
                with self.ddp.capture_cuts(seg):
                    loss, _ = self.forward_loss(self._static_batch)
                    with deferred_sums(self._defer_sums):
                        loss.backward()
                rest = self.ddp.unlaunched_buckets()
                self.flat.gather_grads()             # buckets that never completed (a param without a gradient)
                self._static_loss = loss.detach()
                seg.end(extra_buckets=rest)
        except BaseException:
            seg.abort()
            raise
        torch.cuda.current_stream(self.device).wait_stream(side)
        torch.cuda.synchronize(self.device)
        self._segments = seg

    def drop_graph(self):
        """Leave the hipGraph step for good (capture failure, or a failed graph == eager check): every later step
        runs the eager hook-driven step.  Call it on every rank (it changes which collectives a step issues)."""
        self.graph = False
        self._graph = None
        self._segments = None
        self.flat.reattach_grads()

    def bucket_report(self):
        """Mean launch -> ready time (ms) per bucket over the timed graph-DP steps, and the buckets' sizes (MB)."""
        if not self.bucket_timing:
            return None
        acc = {}
        for step in self.bucket_timing:
            for b, l, d in step:
                acc.setdefault(b, []).append(l.elapsed_time(d))
        el = 4 if self.flat.grad.dtype == torch.float32 else 2
        return [{"bucket": b, "mb": round((self.ddp.buckets[b].end - self.ddp.buckets[b].start) * el / 2 ** 20, 2),
                 "launch_to_ready_ms": round(sum(v) / len(v), 3)} for b, v in sorted(acc.items())]

    # ------------------------------------------------------------------ graph == eager self-check
    def _snapshot(self) -> Dict:
        from ..ops import rng as _rng
        opt = self.optimizer
        with torch.no_grad():
            return dict(data=self.flat.data.clone(), m=opt.exp_avg.clone(), v=opt.exp_avg_sq.clone(),
                        dev=opt.dev_state.clone(), step=opt.step_count, dev_step=opt._dev_step, dev_lr=opt._dev_lr,
                        bufs=[b.detach().clone() for b in self.model.buffers()],
                        rng=(torch.cuda.get_rng_state(self.device) if self.device.type == "cuda" else None),
                        cpu_rng=torch.get_rng_state(),
                        ctr={d: t.clone() for d, t in _rng._COUNTERS.items()}, gstep=self.global_step)

    def _restore(self, s: Dict):
        from ..ops import rng as _rng
        opt = self.optimizer
        with torch.no_grad():
            self.flat.data.copy_(s["data"])
            opt.exp_avg.copy_(s["m"])
            opt.exp_avg_sq.copy_(s["v"])
            opt.dev_state.copy_(s["dev"])
            for b, c in zip(self.model.buffers(), s["bufs"]):
                b.copy_(c)
            for d, t in s["ctr"].items():
                _rng._COUNTERS[d].copy_(t)
        opt.step_count, opt._dev_step, opt._dev_lr = s["step"], s["dev_step"], s["dev_lr"]
        if s["rng"] is not None:
            torch.cuda.set_rng_state(s["rng"], self.device)
        torch.set_rng_state(s["cpu_rng"])
        self.global_step = s["gstep"]

    def graph_eager_check(self, batch: Dict) -> Optional[Dict]:
        """One captured-graph step and one eager step on ``batch`` from the SAME state (parameters, Adam moments, BN
        running statistics, RNG states, dropout counter); the reduced flat gradients, the updated parameters and the
        losses must be bitwise equal (every kernel is deterministic and the random draws replay identically).  The
        engine is left in the pre-check state.  None when no graph has been captured (nothing to compare)."""
        if not self.graph or (self._graph is None and self._segments is None):
            return None
        if not _same_shapes(self._static_batch, batch):
            return None
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        snap = self._snapshot()
        timing, self.comm_timing = self.comm_timing, None
        try:
            loss_g = self.train_step(batch).clone()
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            grad_g, data_g = self.flat.grad.clone(), self.flat.data.clone()
            self._restore(snap)
            loss_e = self._step_body(batch)
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            res = dict(grads=bool(torch.equal(grad_g, self.flat.grad)),
                       params=bool(torch.equal(data_g, self.flat.data)),
                       loss=bool(torch.equal(loss_g, loss_e)))
            if not res["grads"]:
                res["max_grad_diff"] = float((grad_g - self.flat.grad).abs().max())
        finally:
            self._restore(snap)
            self.comm_timing = timing
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
        res["equal"] = res["grads"] and res["params"] and res["loss"]
        return res

    @torch.no_grad()
    def eval_step(self, batch: Dict) -> torch.Tensor:
        self.model.eval()
        loss, _ = self.forward_loss(batch)
        return loss.detach()

    def epoch_end(self):
        self.scheduler.step()

    @property
    def lr(self) -> float:
        return self.optimizer.param_groups[0]["lr"]
