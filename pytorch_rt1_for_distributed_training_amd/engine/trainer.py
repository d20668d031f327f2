"""Epoch loop with Lightning-equivalent semantics (no Lightning dependency).

Mirrors what ``lightning.Trainer.fit`` + ``test`` do for the reference
(``distribute_train.py:192-247``): per-epoch ``DistributedSampler`` reshuffle,
``train_loss`` logged every ``log_every_n_steps`` and as an epoch mean
(``train_loss_step`` / ``train_loss_epoch``), a validation pass each epoch
(``eval_loss``), ``lr-Adam`` at epoch granularity (``LearningRateMonitor``),
MultiStepLR stepped per epoch, ``ModelCheckpoint`` on rank 0, resume from a
checkpoint (commented out in the reference, ``:240``, supported here), and a
final ``test`` pass (``test_loss``).

Differences: losses are accumulated on device and reduced across ranks only at
log points (the reference's ``sync_dist=True`` all-reduces a scalar every
step); ``eval_loss`` / ``test_loss`` are averaged over all ranks instead of
reporting rank 0's shard; a non-finite training loss aborts the run with the
step number (failure detection; the reference has none).
"""
from __future__ import annotations

import math
import os
import time
from typing import Dict, Iterable, Optional

import torch

from ..data.prefetch import DevicePrefetcher
from ..parallel import dist as pdist
from ..utils.checkpoint import ModelCheckpoint, build_checkpoint, load_checkpoint, load_model_state
from ..utils.logging import MultiLogger
from .step import TrainEngine


class NonFiniteLoss(RuntimeError):
    pass


class Trainer:
    def __init__(self, engine: TrainEngine, max_epochs: int = 100, log_every_n_steps: int = 500,
                 checkpoint: Optional[ModelCheckpoint] = None, logger: Optional[MultiLogger] = None,
                 limit_train_batches: Optional[int] = None, limit_val_batches: Optional[int] = None,
                 num_sanity_val_steps: int = 2, verbose: bool = True, batch_transform=None):
        self.engine = engine
        self.batch_transform = batch_transform   # device-side batch transform (GPU crop+resize of raw frames)
        self.max_epochs = max_epochs
        self.log_every = max(1, log_every_n_steps)
        self.ckpt = checkpoint
        self.logger = logger or MultiLogger([])
        self.limit_train = limit_train_batches
        self.limit_val = limit_val_batches
        self.sanity = num_sanity_val_steps
        self.verbose = verbose and pdist.context().is_main
        self.current_epoch = 0
        self.history: Dict[str, list] = {"train_loss_epoch": [], "eval_loss": [], "samples_per_sec": []}
        self.graph_checked = False
        self.graph_check = None

    # ------------------------------------------------------------------ helpers
    def _iter(self, loader, limit):
        pf = self.prefetcher = DevicePrefetcher(loader, self.engine.device, transform=self.batch_transform)
        it = iter(pf)
        try:
            for i, b in enumerate(it):
                if limit is not None and i >= limit:
                    break
                yield b
        finally:
            it.close()                       # stops the loader thread and fills pf.stats (input-path timing)

    def _mean_across(self, total: torch.Tensor, count: int) -> float:
        t = torch.stack([total.detach().double().reshape(()),
                         torch.tensor(float(count), dtype=torch.float64, device=total.device)])
        t = pdist.all_reduce_mean(t)
        return float(t[0] / t[1]) if float(t[1]) > 0 else float("nan")

    def _log(self, metrics, step=None):
        step = self.engine.global_step if step is None else step
        if pdist.context().is_main:
            self.logger.log(metrics, step, self.current_epoch)

    def _make_ckpt(self, callbacks):
        e = self.engine
        return build_checkpoint(e.model, e.optimizer, e.scheduler, epoch=self.current_epoch,
                                global_step=e.global_step, callbacks=callbacks)

    def _check_graph(self, batch):
        """Once, right after the hipGraph step is captured: one replayed step and one eager step on the same batch from
        the same state (TrainEngine.graph_eager_check, the engine is left untouched) must agree bitwise on every rank;
        otherwise training continues on the eager (hook-driven, bucketed) step.  This is what makes the segmented
        graph-DP step safe to use under RCCL by default."""
        e = self.engine
        self.graph_checked = True
        res = e.graph_eager_check(batch)
        if res is None:
            return
        ok = pdist.all_true(res["equal"])
        self.graph_check = dict(res, all_ranks_equal=ok)
        if self.verbose:
            print(f"[trainer] hipGraph step vs eager step on one batch: {'bitwise equal' if ok else 'DIFFERENT'} "
                  f"({res})", flush=True)
        if not ok:
            if self.verbose:
                print("[trainer] falling back to the eager step", flush=True)
            e.drop_graph()

    # ------------------------------------------------------------------ public
    def resume(self, path: str):
        ck = load_checkpoint(path, map_location="cpu")
        load_model_state(self.engine.model, ck)
        if ck.get("optimizer_states"):
            self.engine.optimizer.load_state_dict(ck["optimizer_states"][0])
        if ck.get("lr_schedulers"):
            self.engine.scheduler.load_state_dict(ck["lr_schedulers"][0])
        self.engine.global_step = int(ck.get("global_step", 0))
        self.current_epoch = int(ck.get("epoch", -1)) + 1
        if self.engine.ddp.enabled:
            self.engine.ddp.broadcast_parameters()

    def validate(self, loader, limit=None, name="eval_loss") -> float:
        total, n = None, 0
        for batch in self._iter(loader, limit):
            loss = self.engine.eval_step(batch)
            total = loss if total is None else total + loss
            n += 1
        if total is None:
            total = torch.zeros((), device=self.engine.device)
        return self._mean_across(total, n)

    def fit(self, train_loader: Iterable, val_loader: Optional[Iterable] = None):
        """Train on a high-priority HIP stream when batches are decoded on the device: the prefetch stream's decode
        kernels (data/resident.py, data/shards.py) then only take workgroup slots the step leaves free instead of
        competing with it for the CUs (the step is one graph launch that keeps the chip busy).
        ``RT1_TRAIN_STREAM=normal`` keeps the default stream instead (A/B: a high-priority queue in the process has a
        cost of its own, ~1 ms per bench step measured for an idle one, profiles/r6_graph_dp_world1.log)."""
        e = self.engine
        if (e.device.type == "cuda" and self.batch_transform is not None
                and os.environ.get("RT1_TRAIN_STREAM", "high") != "normal"):
            _, hi = torch.cuda.Stream.priority_range()
            s = torch.cuda.Stream(device=e.device, priority=hi)
            s.wait_stream(torch.cuda.current_stream(e.device))
            try:
                with torch.cuda.stream(s):
                    self._fit(train_loader, val_loader)
            finally:
                torch.cuda.current_stream(e.device).wait_stream(s)
            return
        self._fit(train_loader, val_loader)

    def _fit(self, train_loader: Iterable, val_loader: Optional[Iterable] = None):
        e = self.engine
        if val_loader is not None and self.sanity > 0 and self.current_epoch == 0:
            self.validate(val_loader, self.sanity)
        for epoch in range(self.current_epoch, self.max_epochs):
            self.current_epoch = epoch
            sampler = getattr(train_loader, "sampler", None)
            if hasattr(sampler, "set_epoch"):
                sampler.set_epoch(epoch)
            elif hasattr(train_loader, "set_epoch"):
                train_loader.set_epoch(epoch)
            self._log({"lr-Adam": e.lr})
            total, n, window, wn = None, 0, None, 0
            samples = 0
            t0 = time.perf_counter()
            for batch in self._iter(train_loader, self.limit_train):
                loss = e.train_step(batch)
                if e.graph and not self.graph_checked and (e._graph is not None or e._segments is not None):
                    self._check_graph(batch)
                total = loss if total is None else total + loss
                window = loss if window is None else window + loss
                n += 1
                wn += 1
                samples += int(batch["action_label"]["action"].shape[0]) * pdist.context().world_size
                if e.global_step % self.log_every == 0:
                    step_loss = self._mean_across(window, wn)
                    if not math.isfinite(step_loss):
                        raise NonFiniteLoss(f"non-finite train loss at step {e.global_step}: {step_loss}")
                    self._log({"train_loss_step": step_loss})
                    window, wn = None, 0
                    if self.verbose:
                        print(f"epoch {epoch} step {e.global_step} train_loss {step_loss:.6f} lr {e.lr:.2e}",
                              flush=True)
            if e.device.type == "cuda":
                torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            metrics = {"train_loss_epoch": self._mean_across(total, n) if total is not None else float("nan"),
                       "samples_per_sec": samples / dt if dt > 0 else 0.0}
            io = dict(getattr(getattr(self, "prefetcher", None), "stats", {}) or {})
            if io and n:
                io["step_ms"] = 1e3 * dt / n
                self.input_stats = io
                if self.verbose:
                    print(f"epoch {epoch} input path (per batch): " +
                          " ".join(f"{k} {v:.2f}" for k, v in io.items() if k != "batches"), flush=True)
            if not math.isfinite(metrics["train_loss_epoch"]) and n > 0:
                raise NonFiniteLoss(f"non-finite epoch loss at epoch {epoch}")
            if val_loader is not None:
                metrics["eval_loss"] = self.validate(val_loader, self.limit_val)
            self._log(metrics)
            for k in self.history:
                if k in metrics:
                    self.history[k].append(metrics[k])
            if self.verbose:
                print(f"epoch {epoch} " + " ".join(f"{k} {v:.6g}" for k, v in metrics.items()), flush=True)
            e.epoch_end()
            if self.ckpt is not None and pdist.context().is_main:
                self.ckpt.on_epoch_end(epoch, metrics, self._make_ckpt)
            self.logger.flush()
            pdist.barrier()
        self.current_epoch = self.max_epochs

    def test(self, loader, limit=None) -> float:
        loss = self.validate(loader, limit, "test_loss")
        self._log({"test_loss": loss})
        self.logger.flush()
        if self.verbose:
            print(f"test_loss {loss:.6g}", flush=True)
        return loss
