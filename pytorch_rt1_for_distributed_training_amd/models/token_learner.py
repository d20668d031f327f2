"""TokenLearner (Ryoo et al. 2021) spatial pooling: H*W feature positions -> K tokens.

Spec: ``pytorch_robotics_transformer/tokenizers/token_learner.py:26-95``:
LayerNorm over channels -> 1x1 conv C->64 -> GELU(tanh) -> 1x1 conv 64->K ->
softmax over positions -> weighted sum of the (un-normalised) input features.

MI355X note: per frame the whole problem (120 positions x 512 ch bf16 =
120 KiB) fits in one CU's LDS, so the HIP path (``ops.token_learner``) runs
it as one workgroup per frame; the eager body here is its oracle.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class TokenLearnerModule(nn.Module):
    def __init__(self, inputs_channels: int, num_tokens: int, bottleneck_dim: int = 64, dropout_rate: float = 0.0):
        super().__init__()
        self.layerNorm = nn.LayerNorm(inputs_channels)
        self.conv1 = nn.Conv2d(inputs_channels, bottleneck_dim, 1)
        self.conv2 = nn.Conv2d(bottleneck_dim, num_tokens, 1)
        self.dropout_rate = dropout_rate
        self.num_tokens = num_tokens

    def forward_nhwc(self, feats: torch.Tensor) -> torch.Tensor:
        """feats: (N, P, C) with P = H*W positions -> (N, K, C)."""
        x = self.layerNorm(feats)
        x = F.gelu(F.linear(x, self.conv1.weight.flatten(1), self.conv1.bias), approximate="tanh")
        if self.dropout_rate > 0:
            x = F.dropout(x, self.dropout_rate, self.training)
        logits = F.linear(x, self.conv2.weight.flatten(1), self.conv2.bias)        # (N, P, K)
        if self.dropout_rate > 0:
            logits = F.dropout(logits, self.dropout_rate, self.training)
        weights = torch.softmax(logits.float(), dim=1).to(feats.dtype)              # softmax over positions
        return torch.bmm(weights.transpose(1, 2), feats)                           # (N, K, C)

    def forward(self, inputs: torch.Tensor) -> torch.Tensor:
        """inputs: (N, C, H, W) -> (N, K, C)."""
        n, c, h, w = inputs.shape
        return self.forward_nhwc(inputs.permute(0, 2, 3, 1).reshape(n, h * w, c))
