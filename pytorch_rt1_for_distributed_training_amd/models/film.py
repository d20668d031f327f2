"""FiLM conditioning (Perez et al. 2018) as used by RT-1.

Semantics follow ``film_efficientnet/film_conditioning_layer.py:23-51``:
``out = (1 + W_m c + b_m) * x + (W_a c + b_a)`` broadcast over H x W, with both
projections zero-initialised so a fresh layer is the identity.

MI355X note: the 27 FiLM layers of the encoder all project the same per-frame
text vector, so the fused path (``ops.film``) evaluates every gamma/beta with
ONE GEMM against the concatenated weights instead of 54 small Linear calls;
this module only owns the parameters and the eager formula.
"""
from __future__ import annotations

import torch
import torch.nn as nn


class FilmConditioning(nn.Module):
    def __init__(self, num_channels: int, text_vector_size: int = 512):
        super().__init__()
        self.num_channels = num_channels
        # attribute names are the checkpoint schema (``..._projection_{add,mult}.{weight,bias}``)
        self._projection_add = nn.Linear(text_vector_size, num_channels)
        self._projection_mult = nn.Linear(text_vector_size, num_channels)
        for p in self.parameters():
            nn.init.zeros_(p)

    def gamma_beta(self, conditioning: torch.Tensor):
        """(1 + gamma, beta), each (B, C)."""
        return 1.0 + self._projection_mult(conditioning), self._projection_add(conditioning)

    def forward(self, conv_filters: torch.Tensor, conditioning: torch.Tensor) -> torch.Tensor:
        # conv_filters: (B, C, H, W) (any memory format); conditioning: (B, D)
        scale, shift = self.gamma_beta(conditioning)
        return conv_filters * scale[:, :, None, None].to(conv_filters.dtype) + shift[:, :, None, None].to(conv_filters.dtype)
