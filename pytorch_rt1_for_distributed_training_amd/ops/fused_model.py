"""The ``hip`` backend of the RT-1 policy: routes hot paths to HIP kernels.

``TransformerNetwork`` calls ``model.fused.<hook>`` when a FusedRT1 is
installed.  Each hook uses the fused HIP implementation of its component and
keeps the eager module as the numerical oracle (``tests/test_kernels_gpu.py``).
"""
from __future__ import annotations

import torch

from ..models import preprocess


class FusedRT1:
    def __init__(self, model, cfg):
        self.cfg = cfg
        self.dtype = torch.bfloat16 if cfg.dtype == "bf16" else torch.float32
        self.fused_head = False
        if cfg.channels_last:
            model._image_tokenizer.to(memory_format=torch.channels_last)

    def _autocast(self):
        return torch.autocast("cuda", dtype=self.dtype, enabled=self.dtype != torch.float32)

    def tokenize_images(self, model, images, context, shift):
        b, t = images.shape[:2]
        frames = images.reshape(b * t, *images.shape[2:])
        frames = preprocess.convert_dtype_and_crop_images(frames, model._crop_ratio, shift)
        if self.cfg.channels_last:
            frames = frames.contiguous(memory_format=torch.channels_last)
        with self._autocast():
            return model._image_tokenizer(frames.reshape(b, t, *frames.shape[1:]), context)

    def transformer_hidden(self, model, tokens):
        with self._autocast():
            h, model._attention_scores = model._transformer.hidden(tokens, model._default_attention_mask)
        return h

    def action_loss(self, model, logits, targets, b, t):
        import torch.nn.functional as F
        ce = F.cross_entropy(logits.float().reshape(-1, logits.shape[-1]), targets.reshape(-1), reduction="none")
        num_items = float(b * t) * model._single_time_step_num_tokens
        return (ce.view(b, t, model._tokens_per_action) / num_items).mean(dim=-1)

    def action_logits(self, model, hidden, positions):
        with self._autocast():
            return model._transformer._output_tokens(hidden[:, positions])
