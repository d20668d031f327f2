"""Metric loggers with the reference's names and layout.

The reference logs ``train_loss`` (on_step + on_epoch -> ``train_loss_step`` /
``train_loss_epoch``), ``eval_loss``, ``test_loss`` and ``lr-Adam`` through
Lightning's ``CSVLogger`` (``log_dir/csv/exp_name/version_N/metrics.csv``) and
``TensorBoardLogger`` (``log_dir/tb/exp_name/version_N``) — ``distribute_train.py:
69,85,97,221,225-228``.  Same names, same directory convention here; the
framework additionally logs ``samples_per_sec`` and ``step_ms``.
"""
from __future__ import annotations

import csv
import os
from typing import Dict, List, Optional

from .tfevents import EventWriter


def _next_version(root: str) -> str:
    os.makedirs(root, exist_ok=True)
    vs = [int(d.split("_")[1]) for d in os.listdir(root) if d.startswith("version_") and d.split("_")[1].isdigit()]
    return os.path.join(root, f"version_{max(vs) + 1 if vs else 0}")


class CSVLogger:
    def __init__(self, save_dir: str, name: str):
        self.log_dir = _next_version(os.path.join(save_dir, name))
        os.makedirs(self.log_dir, exist_ok=True)
        self.path = os.path.join(self.log_dir, "metrics.csv")
        self.rows: List[Dict] = []
        self.keys: List[str] = ["epoch", "step"]

    def log(self, metrics: Dict[str, float], step: int, epoch: int):
        row = {"epoch": epoch, "step": step, **metrics}
        for k in row:
            if k not in self.keys:
                self.keys.append(k)
        self.rows.append(row)

    def flush(self):
        with open(self.path, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=self.keys)
            w.writeheader()
            for r in self.rows:
                w.writerow(r)


class TensorBoardLogger:
    def __init__(self, save_dir: str, name: str):
        self.log_dir = _next_version(os.path.join(save_dir, name))
        self.writer = EventWriter(self.log_dir)

    def log(self, metrics: Dict[str, float], step: int, epoch: int):
        for k, v in metrics.items():
            self.writer.add_scalar(k, float(v), step)

    def flush(self):
        self.writer.flush()


class MultiLogger:
    def __init__(self, loggers: Optional[List] = None, enabled: bool = True):
        self.loggers = loggers or []
        self.enabled = enabled

    def log(self, metrics: Dict[str, float], step: int, epoch: int):
        if self.enabled:
            for lg in self.loggers:
                lg.log(metrics, step, epoch)

    def flush(self):
        if self.enabled:
            for lg in self.loggers:
                lg.flush()
