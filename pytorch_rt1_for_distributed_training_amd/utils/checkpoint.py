"""Lightning-compatible RT-1 checkpoints.

The reference saves through Lightning's ``ModelCheckpoint`` (``distribute_train.py:214-220``):
a ``torch.save`` dict whose ``state_dict`` holds the policy under the ``model.``
prefix (the LightningModule attribute, ``:42``) in module-registration order —
806 entries for RT-1 — plus ``epoch``, ``global_step``,
``pytorch-lightning_version``, ``optimizer_states``, ``lr_schedulers``,
``callbacks``, ``loops``.  Files are named ``{epoch}-{eval_loss:.6f}-
{train_loss_epoch:.6f}.ckpt`` plus ``last.ckpt``; evaluation loads them with
``RT1_Lightning.load_from_checkpoint`` (``language_table/eval/main_rt1.py:75``).

This module writes exactly that layout from rank 0 (so reference tooling can
read our checkpoints and vice-versa) and reads with ``weights_only=True``
(nothing in a checkpoint file is ever executed).
"""
from __future__ import annotations

import os
import re
from typing import Any, Dict, Optional

import torch

PREFIX = "model."
LIGHTNING_VERSION = "2.3.0"


def lightning_state_dict(model: torch.nn.Module) -> Dict[str, torch.Tensor]:
    return {PREFIX + k: v.detach().cpu().clone() for k, v in model.state_dict().items()}


def build_checkpoint(model, optimizer=None, scheduler=None, epoch: int = 0, global_step: int = 0,
                     callbacks: Optional[Dict[str, Any]] = None, extra: Optional[Dict[str, Any]] = None) -> Dict:
    ck: Dict[str, Any] = {
        "epoch": int(epoch),
        "global_step": int(global_step),
        "pytorch-lightning_version": LIGHTNING_VERSION,
        "state_dict": lightning_state_dict(model),
        "loops": {"fit_loop": {"epoch_progress": {"current": {"completed": int(epoch)}}}},
        "callbacks": callbacks or {},
        "optimizer_states": [_cpu(optimizer.state_dict())] if optimizer is not None else [],
        "lr_schedulers": [scheduler.state_dict()] if scheduler is not None else [],
    }
    if extra:
        ck.update(extra)
    return ck


def _cpu(obj):
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_cpu(v) for v in obj)
    return obj


def save_checkpoint(path: str, ckpt: Dict):
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = path + ".tmp"
    torch.save(ckpt, tmp)
    os.replace(tmp, path)


def load_checkpoint(path: str, map_location="cpu") -> Dict:
    return torch.load(path, map_location=map_location, weights_only=True)


def load_model_state(model: torch.nn.Module, ckpt_or_path, strict: bool = True):
    ck = load_checkpoint(ckpt_or_path) if isinstance(ckpt_or_path, str) else ckpt_or_path
    sd = ck.get("state_dict", ck)
    sd = {k[len(PREFIX):] if k.startswith(PREFIX) else k: v for k, v in sd.items()}
    with torch.no_grad():
        return model.load_state_dict(sd, strict=strict)


def format_filename(template: str, metrics: Dict[str, float], epoch: int) -> str:
    """Lightning filename templating: ``{epoch}-{eval_loss:.6f}`` -> ``epoch=3-eval_loss=0.012345``."""
    def rep(m):
        name, fmt = m.group(1), m.group(2) or ""
        val = epoch if name == "epoch" else metrics.get(name, float("nan"))
        return f"{name}={format(val, fmt[1:]) if fmt else val}"
    return re.sub(r"\{([A-Za-z_][\w/]*)(:[^}]*)?\}", rep, template)


class ModelCheckpoint:
    """Keep-all + ``last.ckpt`` every N epochs (``distribute_train.py:214-220``)."""

    def __init__(self, dirpath: str, filename: str = "{epoch}-{eval_loss:.6f}-{train_loss_epoch:.6f}",
                 every_n_epochs: int = 1, save_last: bool = True):
        self.dirpath, self.filename, self.every = dirpath, filename, max(1, every_n_epochs)
        self.save_last = save_last
        self.best_model_path = ""
        self.last_model_path = ""

    def state(self) -> Dict:
        return {"dirpath": self.dirpath, "last_model_path": self.last_model_path}

    def on_epoch_end(self, epoch: int, metrics: Dict[str, float], make_ckpt) -> Optional[str]:
        if (epoch + 1) % self.every != 0:
            return None
        ck = make_ckpt({"ModelCheckpoint": self.state()})
        path = os.path.join(self.dirpath, format_filename(self.filename, metrics, epoch) + ".ckpt")
        save_checkpoint(path, ck)
        if self.save_last:
            self.last_model_path = os.path.join(self.dirpath, "last.ckpt")
            save_checkpoint(self.last_model_path, ck)
        return path
