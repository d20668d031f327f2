"""RT-1 image tokenizer: FiLM-EfficientNet-B3 -> 1x1 conv -> FiLM -> TokenLearner.

Spec: ``film_efficientnet/pretrained_efficientnet_encoder.py:36-74`` (encoder
wrapper) and ``tokenizers/image_tokenizer.py:31-85`` (time folding, token
learner).  Attribute names (``_tokenizer.conv1x1``, ``_tokenizer.net``,
``_tokenizer.film_layer``, ``_token_learner``) are the checkpoint schema.

The forward takes the whole ``(b, t, 3, H, W)`` history at once and folds time
into the batch, so one launch of every backbone op covers ``b*t`` frames (768
frames per GPU at the BASELINE global batch of 1024 on 8 GPUs).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .efficientnet import FiLMEfficientNet, feature_map_size
from .film import FilmConditioning
from .token_learner import TokenLearnerModule


class EfficientNetEncoder(nn.Module):
    def __init__(self, token_embedding_size: int = 512, early_film: bool = True, pooling: bool = True,
                 width_coefficient: float = 1.2, depth_coefficient: float = 1.4, drop_connect_rate: float = 0.2,
                 text_vector_size: int = 512):
        super().__init__()
        self.net_out_channels = None
        net = FiLMEfficientNet(width_coefficient, depth_coefficient, drop_connect_rate,
                               include_film=early_film, text_vector_size=text_vector_size)
        # registration order = checkpoint key order: conv1x1, net, film_layer
        self.conv1x1 = nn.Conv2d(net.out_channels, token_embedding_size, 1, bias=False)
        self.net = net
        self.film_layer = FilmConditioning(token_embedding_size, text_vector_size)
        self.early_film = early_film
        self._pooling = pooling

    def forward(self, image: torch.Tensor, context: Optional[torch.Tensor]) -> torch.Tensor:
        feats = self.net(image, context) if self.early_film else self.net(image)
        feats = self.film_layer(F.conv2d(feats, self.conv1x1.weight.to(feats.dtype)), context)
        if self._pooling:
            return feats.mean(dim=(2, 3))
        return feats


class RT1ImageTokenizer(nn.Module):
    def __init__(self, embedding_output_dim: int = 512, use_token_learner: bool = True, num_tokens: int = 8,
                 height: int = 300, width: int = 300, **encoder_kw):
        super().__init__()
        self._tokenizer = EfficientNetEncoder(embedding_output_dim, early_film=True, pooling=False, **encoder_kw)
        self._use_token_learner = use_token_learner
        self._embedding_dim = embedding_output_dim
        fh, fw = feature_map_size(height, width, self._tokenizer.net.specs)
        self._feature_positions = fh * fw
        if use_token_learner:
            self._num_tokens = num_tokens
            self._token_learner = TokenLearnerModule(embedding_output_dim, num_tokens)

    @property
    def tokens_per_context_image(self) -> int:
        return self._num_tokens if self._use_token_learner else self._feature_positions

    def forward(self, image: torch.Tensor, context: Optional[torch.Tensor] = None) -> torch.Tensor:
        """image (b, t, 3, H, W), context (b, t, D) -> tokens (b, t, K, E)."""
        b, t = image.shape[:2]
        frames = image.reshape(b * t, *image.shape[2:])
        ctx = context.reshape(b * t, -1) if context is not None else None
        feats = self._tokenizer(frames, ctx)                       # (b*t, E, h, w)
        if self._use_token_learner:
            tokens = self._token_learner(feats)                    # (b*t, K, E)
            return tokens.reshape(b, t, tokens.shape[1], -1)
        n, e, h, w = feats.shape
        return feats.reshape(b, t, e, h * w).transpose(2, 3)
