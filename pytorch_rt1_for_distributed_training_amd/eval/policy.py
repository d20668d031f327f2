"""RT-1 closed-loop policy for evaluation rollouts.

Behaviour of the reference eval policy (``language_table/train/policy.py:32-112``,
``BCJaxPyPolicyRT1``): only the LAST frame of the history is fed (the history
itself lives in ``network_state``), the model runs in inference mode with a
rolling state, the predicted 2-d action is clipped to +-0.03, and the state is
zeroed at the start of every episode (``language_table/eval/main_rt1.py:158-160``).

Differences: device-agnostic (no hard-coded ``'cuda'``), no
``torch.cuda.empty_cache()`` per step (the reference frees the allocator cache
on every action), and a step is ``engine.infer.InferenceEngine``: the
fused HIP backend on GPU, one transformer pass instead of three, the rolling
state kept on the device, the whole step replayed from one hipGraph.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch

from ..config import RT1Config
from ..models import build_rt1
from ..utils.checkpoint import load_checkpoint, load_model_state


class RT1Policy:
    def __init__(self, model: torch.nn.Module, device=None, action_min: float = -0.03, action_max: float = 0.03,
                 action_mean: float = 0.0, action_std: float = 1.0, cfg: Optional[RT1Config] = None,
                 backend: str = "auto", graph: Optional[bool] = None):
        from ..engine.infer import InferenceEngine
        self.device = torch.device(device) if device is not None else next(model.parameters()).device
        self.engine = InferenceEngine(model, cfg, device=self.device, backend=backend, graph=graph)
        self.model = self.engine.model
        self.action_min, self.action_max = action_min, action_max
        self.action_mean, self.action_std = action_mean, action_std
        self.reset()

    @classmethod
    def from_checkpoint(cls, path: str, cfg: Optional[RT1Config] = None, device=None, backend: str = "auto",
                        **kw) -> "RT1Policy":
        cfg = cfg or RT1Config()
        model = build_rt1(cfg)
        load_model_state(model, load_checkpoint(path))
        return cls(model, device=device, cfg=cfg, backend=backend, **kw)

    @property
    def backend(self) -> str:
        return self.engine.backend

    @property
    def state(self) -> Dict[str, torch.Tensor]:
        """The rolling ``network_state`` (reference layout), living on the device."""
        e = self.engine
        return {"context_image_tokens": e.state_img, "action_tokens": e.state_act,
                "seq_idx": e.seq_idx.view(1).expand(e.b)}

    def reset(self):
        self.engine.reset()

    @torch.no_grad()
    def action(self, rgb, instruction_embedding) -> np.ndarray:
        """rgb: (H, W, 3) uint8 frame or (T, H, W, 3) history (last frame used);
        instruction_embedding: (512,) or (T, 512)."""
        rgb = np.asarray(rgb)
        if rgb.ndim == 4:
            rgb = rgb[-1]
        emb = np.asarray(instruction_embedding, dtype=np.float32)
        if emb.ndim == 2:
            emb = emb[-1]
        img = torch.from_numpy(np.ascontiguousarray(rgb)).permute(2, 0, 1)[None]
        if img.dtype != torch.uint8:
            img = (img.float().clamp(0, 1) * 255.0).round().to(torch.uint8)
        out = self.engine.step(img, torch.from_numpy(emb)[None])
        act = out["action"].float().cpu().numpy()[0]
        act = act * max(self.action_std, float(np.finfo(np.float32).eps)) + self.action_mean
        return np.clip(act, self.action_min, self.action_max)


class LavaPolicy:
    """Closed-loop LAVA policy: keeps the last ``sequence_length`` frames (first frame tiled at reset), predicts a
    normalised action, de-normalises it with the training statistics and clips it (reference eval: +-0.03)."""

    def __init__(self, model, stats, device=None, action_clip: float = 0.03):
        from ..data.normalization import StdNormalizer
        self.model = model
        self.device = torch.device(device) if device is not None else next(model.parameters()).device
        self.model.to(self.device).eval()
        self.norm = StdNormalizer(stats["action"]["mean"], stats["action"]["std"])
        self.T = model.cfg.sequence_length
        self.clip = action_clip
        self.frames = None

    def reset(self):
        self.frames = None

    @torch.no_grad()
    def action(self, rgb, instruction_embedding) -> np.ndarray:
        rgb = np.asarray(rgb)
        if rgb.ndim == 4:
            rgb = rgb[-1]
        emb = np.asarray(instruction_embedding, np.float32)
        if emb.ndim == 2:
            emb = emb[-1]
        if self.frames is None:
            self.frames = [rgb] * self.T
        else:
            self.frames = self.frames[1:] + [rgb]
        obs = {"rgb": torch.from_numpy(np.stack(self.frames))[None].to(self.device),
               "instruction_embedding": torch.from_numpy(np.repeat(emb[None], self.T, 0))[None].to(self.device)}
        a = self.norm.denormalize(self.model(obs)).float().cpu().numpy()[0]
        return np.clip(a, -self.clip, self.clip)
