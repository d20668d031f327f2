"""RT-1 model family: FiLM-EfficientNet-B3 tokenizer + TokenLearner + causal transformer."""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

from .. import spaces
from ..config import RT1Config
from .action_tokenizer import RT1ActionTokenizer
from .efficientnet import FiLMEfficientNet, MBConvBlock, block_specs, feature_map_size
from .film import FilmConditioning
from .image_tokenizer import EfficientNetEncoder, RT1ImageTokenizer
from .policy import TransformerNetwork
from .token_learner import TokenLearnerModule
from .transformer import Transformer, rt1_attention_mask

__all__ = ["RT1ActionTokenizer", "FiLMEfficientNet", "MBConvBlock", "FilmConditioning", "EfficientNetEncoder",
           "RT1ImageTokenizer", "TransformerNetwork", "TokenLearnerModule", "Transformer", "rt1_attention_mask",
           "observation_space", "action_space", "build_rt1", "load_pretrained_backbone", "block_specs", "feature_map_size"]


def observation_space(cfg: RT1Config) -> spaces.Dict:
    """``distribute_train.py:28-33``."""
    return spaces.Dict({
        "image": spaces.Box(0.0, 1.0, (3, cfg.height, cfg.width), np.float32),
        "natural_language_embedding": spaces.Box(-np.inf, np.inf, (cfg.text_embedding_size,), np.float32),
    })


def action_space(cfg: RT1Config) -> spaces.Dict:
    """``distribute_train.py:35-40`` (OrderedDict fixes the token order)."""
    return spaces.Dict(OrderedDict([
        ("terminate_episode", spaces.Discrete(cfg.terminate_classes)),
        ("action", spaces.Box(cfg.action_low, cfg.action_high, (cfg.action_dim,), np.float32)),
    ]))


def build_rt1(cfg: RT1Config, pretrained: str = None) -> TransformerNetwork:
    """The RT-1 policy exactly as ``RT1_Lightning.__init__`` builds it (``distribute_train.py:42-55``).

    ``pretrained`` (or ``cfg.pretrained``): path of a torchvision ``efficientnet_b3`` state dict (``.pth``,
    e.g. the reference's ``efficientnetb3_notop.pth``) mapped positionally onto the FiLM-free backbone, as the
    reference's default ``weights='imagenet'`` does (``film_efficientnet_encoder.py:376-425``,
    ``pretrained_efficientnet_encoder.py:52``).  The file is read with ``torch.load(weights_only=True)``: it
    executes nothing.  Without it the backbone is random-init (the reference's checkpoint blob is absent)."""
    model = TransformerNetwork(
        input_tensor_space=observation_space(cfg), output_tensor_space=action_space(cfg),
        vocab_size=cfg.vocab_size, token_embedding_size=cfg.token_embedding_size, num_layers=cfg.num_layers,
        layer_size=cfg.layer_size, num_heads=cfg.num_heads, feed_forward_size=cfg.feed_forward_size,
        dropout_rate=cfg.dropout_rate, time_sequence_length=cfg.seq_len, crop_size=236,
        use_token_learner=cfg.use_token_learner, width_coefficient=cfg.width_coefficient,
        depth_coefficient=cfg.depth_coefficient, drop_connect_rate=cfg.drop_connect_rate,
        crop_ratio=cfg.crop_ratio)
    path = pretrained or getattr(cfg, "pretrained", None)
    if path:
        load_pretrained_backbone(model, path)
    return model


def load_pretrained_backbone(model: TransformerNetwork, path_or_state) -> TransformerNetwork:
    """ImageNet init of the image tokenizer's EfficientNet-B3 from a torchvision state dict (path or dict)."""
    import torch
    from .efficientnet import load_torchvision_b3_state_dict
    sd = path_or_state
    if isinstance(path_or_state, str):
        sd = torch.load(path_or_state, map_location="cpu", weights_only=True)
        if isinstance(sd, dict) and "state_dict" in sd and isinstance(sd["state_dict"], dict):
            sd = sd["state_dict"]
    load_torchvision_b3_state_dict(model._image_tokenizer._tokenizer.net, sd)
    return model
