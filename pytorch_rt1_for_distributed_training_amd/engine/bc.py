"""Behaviour-cloning trainer for the LAVA family, on the same DP runtime as RT-1.

Reference: ``language_table/train/bc.py:33-245`` (BCAgent: Adam(lr 1e-3, eps 1e-7), optional frozen keys,
per-example MSE between predicted and (normalised) actions, ``pmean`` of gradients and loss over the batch axis)
and ``train.py`` (step loop, periodic logging/checkpointing, restore-or-init).  Here the ``pmean`` is the
bucketed RCCL all-reduce of ``parallel.ddp`` with the 1/world average folded into the fused Adam kernel, and
checkpoints are plain ``torch.save`` dicts holding the parameters, the optimizer state, the step and the
normalisation statistics (restore-or-init via :meth:`BCTrainer.restore_or_init`).
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Sequence

import torch
import torch.nn as nn

from ..data.normalization import StdNormalizer
from ..parallel import dist as pdist
from ..parallel.ddp import DataParallel
from ..parallel.flat import FlatParameters
from .optim import FlatAdam


class BCTrainer:
    def __init__(self, model: nn.Module, stats: Dict, lr: float = 1e-3, eps: float = 1e-7,
                 freeze_keys: Sequence[str] = (), device=None, bucket_cap_mb: float = 32.0, augment=None,
                 pretrained_checkpoints: Sequence = ()):
        """``freeze_keys``: parameters whose name contains any key get no update -- the reference's
        ``optax.multi_transform({'adam', 'zero': set_to_zero})`` (``bc.py:119-140``); here they are left out of
        the flat optimizer buffer and the all-reduce entirely.  ``pretrained_checkpoints``: ``[(path,
        [(ckpt_prefix, model_prefix), ...]), ...]`` loaded before training with the reference's prefix-replacement
        rule (``bc.py:91-110``; e.g. a CLIP text tower into the language encoder)."""
        self.device = device or pdist.default_device()
        self.augment = augment            # data.augment.BCAugment: on-device crop/resize + photometric (J3)
        self.model = model.to(self.device)
        self.loaded_pretrained = []
        for path, replacements in pretrained_checkpoints:
            self.loaded_pretrained += load_pretrained(self.model, path, replacements)
        for name, p in self.model.named_parameters():
            if any(k in name for k in freeze_keys):
                p.requires_grad_(False)
        self.stats = stats
        a = stats["action"]
        self.action_norm = StdNormalizer(a["mean"], a["std"])
        trainable = [p for p in self.model.parameters() if p.requires_grad]
        self.flat = FlatParameters(list(reversed(trainable)), device=self.device)
        self.ddp = DataParallel(self.model, self.flat, bucket_cap_mb=bucket_cap_mb, broadcast_buffers=False)
        self.optimizer = FlatAdam(self.flat, lr=lr, eps=eps, all_params=list(self.model.parameters()))
        self.step = 0

    def loss(self, batch: Dict) -> torch.Tensor:
        obs, action = batch["observation"], batch["action"]
        if self.augment is not None:
            obs = dict(obs, rgb=self.augment(obs["rgb"], train=self.model.training))
        pred = self.model(obs)
        target = self.action_norm.normalize(action.to(pred.dtype))
        return torch.mean(torch.square(pred - target))

    def train_step(self, batch: Dict) -> torch.Tensor:
        self.model.train()
        self.ddp.prepare()
        self.optimizer.zero_grad()
        loss = self.loss(batch)
        loss.backward()
        self.ddp.finish()
        self.optimizer.step(grad_scale=self.ddp.grad_scale)
        self.step += 1
        return pdist.all_reduce_mean(loss.detach()) if self.ddp.enabled else loss.detach()

    @torch.no_grad()
    def predict(self, obs: Dict) -> torch.Tensor:
        self.model.eval()
        if self.augment is not None:
            obs = dict(obs, rgb=self.augment(obs["rgb"], train=False))
        return self.action_norm.denormalize(self.model(obs))

    # ------------------------------------------------------------------ checkpoints
    def state_dict(self) -> Dict:
        # statistics as JSON text so the checkpoint loads with torch.load(weights_only=True)
        return {"model": self.model.state_dict(), "optimizer": self.optimizer.state_dict(), "step": self.step,
                "stats": stats_to_json(self.stats)}

    def save(self, path: str):
        if pdist.context().is_main:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
            torch.save(self.state_dict(), path)

    def restore_or_init(self, path: Optional[str]) -> bool:
        if not path or not os.path.exists(path):
            return False
        ck = torch.load(path, map_location=self.device, weights_only=True)
        self.model.load_state_dict(ck["model"])
        self.optimizer.load_state_dict(ck["optimizer"])
        self.step = int(ck["step"])
        return True


def stats_to_json(stats: Dict) -> str:
    import json

    import numpy as np

    def conv(x):
        if isinstance(x, dict):
            return {k: conv(v) for k, v in x.items()}
        return np.asarray(x).tolist()
    return json.dumps(conv(stats))


def stats_from_json(text: str) -> Dict:
    import json

    import numpy as np

    def conv(x):
        if isinstance(x, dict):
            return {k: conv(v) for k, v in x.items()}
        return np.asarray(x, np.float32)
    return conv(json.loads(text))


def load_pretrained(model: nn.Module, path_or_state, replacements) -> list:
    """Copy tensors of a checkpoint into ``model``: every checkpoint key starting with ``ckpt_prefix`` is renamed
    by replacing that prefix with ``model_prefix`` and copied if the model has it (shape-checked).  Reads with
    ``torch.load(weights_only=True)``; a ``{"model": state_dict}`` wrapper is unwrapped.  Returns the
    (checkpoint key, model key) pairs that were loaded."""
    sd = path_or_state
    if isinstance(path_or_state, str):
        sd = torch.load(path_or_state, map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and isinstance(sd.get("model"), dict):
        sd = sd["model"]
    target = model.state_dict()
    loaded = []
    with torch.no_grad():
        for src, dst in replacements:
            for key, val in sd.items():
                if not key.startswith(src):
                    continue
                new = key.replace(src, dst)
                if new in target:
                    if tuple(target[new].shape) != tuple(val.shape):
                        raise ValueError(f"{key} -> {new}: shape {tuple(val.shape)} != {tuple(target[new].shape)}")
                    target[new].copy_(val.to(target[new].dtype))
                    loaded.append((key, new))
    return loaded
