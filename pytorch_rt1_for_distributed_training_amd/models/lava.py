"""LAVA (Language-Attends-to-Vision-to-Act) behaviour-cloning policy -- the second model family.

Behavioural spec: ``language_table/train/networks/{lava,dense_resnet}.py`` and the
``language_table_sim_local`` config (sequence 4, d_model 128, 2 heads, 4 pixel-language layers, 2 temporal
layers, pyramid levels (2, 3, 4), conv-maxpool image encoder, dense-resnet head 1024 x 2 blocks, MSE BC):

  rgb (B, T, H, W, 3) -> conv3x3+ReLU+maxpool x4 (+1 maxpool) feature pyramid
  -> per chosen level: Dense -> d_model, * sqrt(d_model), + 2-D sin/cos positions -> one "visual sentence"
  -> language query (512-d instruction embedding -> Dense -> d_model, * sqrt(d_model)) attends to the visual
     sentence through pre-norm cross-attention layers (residual on the language path only, ReLU FFN)
  -> LayerNorm -> temporal pre-norm transformer over the T steps (+ 1-D sin/cos positions), mean over time, LN
  -> dense resnet -> action (2).
Dense layers use N(0, 0.05) kernel and bias init as in the reference.  The language encoder is the
``clip_in_obs`` variant: a precomputed 512-d embedding per step (here from any text encoder, e.g.
``sim.HashedTextEncoder``) -- the frozen CLIP text tower and its checkpoint are not available offline.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclass
class LavaConfig:
    sequence_length: int = 4
    d_model: int = 128
    num_heads: int = 2
    num_layers: int = 4                       # pixel-language layers
    temporal_layers: int = 2
    pyramid_fuse_layers: Tuple[int, ...] = (2, 3, 4)
    dense_resnet_width: int = 1024
    dense_resnet_blocks: int = 2
    action_size: int = 2
    lang_dim: int = 512
    height: int = 180
    width: int = 320
    dropout: float = 0.1


def _dense(i: int, o: int) -> nn.Linear:
    lin = nn.Linear(i, o)
    nn.init.normal_(lin.weight, std=0.05)
    nn.init.normal_(lin.bias, std=0.05)
    return lin


def _flax_conv(cin: int, cout: int, k: int) -> nn.Conv2d:
    """3x3 SAME conv with Flax ``nn.Conv``'s default init (``pixel.py:56``): truncated LeCun-normal weights
    (variance 1 / fan_in, truncated at 2 sigma) and a zero bias."""
    conv = nn.Conv2d(cin, cout, k, padding=k // 2)
    std = math.sqrt(1.0 / (cin * k * k)) / 0.87962566103423978
    nn.init.trunc_normal_(conv.weight, std=std, a=-2 * std, b=2 * std)
    nn.init.zeros_(conv.bias)
    return conv


def sincos_1d(length: int, d: int) -> torch.Tensor:
    pe = np.zeros((length, d), np.float32)
    pos = np.arange(length)[:, None]
    div = np.exp(np.arange(0, d, 2) * -(np.log(1.0e4) / d))
    pe[:, 0::2] = np.sin(pos * div)
    pe[:, 1::2] = np.cos(pos * div)
    return torch.from_numpy(pe)


def sincos_2d(d: int, h: int, w: int) -> torch.Tensor:
    """(h*w, d): first half of the channels encodes the column, second half the row (sin/cos interleaved)."""
    if d % 4:
        raise ValueError("2-D sin/cos positions need d_model % 4 == 0")
    half = d // 2
    div = np.exp(np.arange(0.0, half, 2) * -(np.log(10000.0) / half))
    pe = np.zeros((d, h, w), np.float32)
    px = np.arange(w)[:, None] * div                                     # (w, half/2)
    py = np.arange(h)[:, None] * div
    pe[0:half:2] = np.sin(px).T[:, None, :]
    pe[1:half:2] = np.cos(px).T[:, None, :]
    pe[half::2] = np.sin(py).T[:, :, None]
    pe[half + 1::2] = np.cos(py).T[:, :, None]
    return torch.from_numpy(pe.reshape(d, h * w).T.copy())


class ConvMaxpoolEncoder(nn.Module):
    """Feature pyramid: 4 x (conv3x3 SAME + ReLU + maxpool2), then one more maxpool (5 levels).  The convs take
    Flax ``nn.Conv``'s default init like the reference's (``language_table/train/networks/lava.py:43``)."""

    def __init__(self, channels: Sequence[int] = (32, 64, 128, 256)):
        super().__init__()
        convs, cin = [], 3
        for c in channels:
            convs.append(_flax_conv(cin, c, 3))
            cin = c
        self.convs = nn.ModuleList(convs)
        self.channels = list(channels) + [channels[-1]]

    def forward(self, x):                                                # x (N, 3, H, W)
        levels = []
        for conv in self.convs:
            x = F.max_pool2d(F.relu(conv(x)), 2)
            levels.append(x)
        levels.append(F.max_pool2d(x, 2))
        return levels


class CrossLayer(nn.Module):
    """Pre-norm language(query) -> pixels(key/value) attention with a residual on the language path."""

    def __init__(self, d: int, heads: int, dff: int, dropout: float):
        super().__init__()
        self.ln_pix, self.ln_lang, self.ln_ffn = nn.LayerNorm(d), nn.LayerNorm(d), nn.LayerNorm(d)
        self.attn = nn.MultiheadAttention(d, heads, batch_first=True)
        self.ff1, self.ff2 = _dense(d, dff), _dense(dff, dff)
        self.drop = nn.Dropout(dropout)

    def forward(self, pix, lang):
        p, q = self.ln_pix(pix), self.ln_lang(lang)
        x3 = lang + self.drop(self.attn(q, p, p, need_weights=False)[0])
        return x3 + self.drop(self.ff2(F.relu(self.ff1(self.ln_ffn(x3)))))


class SelfLayer(nn.Module):
    def __init__(self, d: int, heads: int, dff: int, dropout: float):
        super().__init__()
        self.ln1, self.ln2 = nn.LayerNorm(d), nn.LayerNorm(d)
        self.attn = nn.MultiheadAttention(d, heads, batch_first=True)
        self.ff1, self.ff2 = _dense(d, dff), _dense(dff, dff)
        self.drop = nn.Dropout(dropout)

    def forward(self, x):
        h = self.ln1(x)
        x3 = x + self.drop(self.attn(h, h, h, need_weights=False)[0])
        return x3 + self.drop(self.ff2(F.relu(self.ff1(self.ln2(x3)))))


class DenseResnet(nn.Module):
    def __init__(self, din: int, width: int, blocks: int):
        super().__init__()
        self.inp = _dense(din, width)
        self.blocks = nn.ModuleList(nn.Sequential(nn.ReLU(), _dense(width, width // 4), nn.ReLU(),
                                                  _dense(width // 4, width // 4), nn.ReLU(),
                                                  _dense(width // 4, width)) for _ in range(blocks))

    def forward(self, x):
        x = self.inp(x)
        for b in self.blocks:
            x = x + b(x)
        return x


class SequenceLAVMSE(nn.Module):
    """obs {rgb (B,T,H,W,3) in [0,1] or uint8, instruction_embedding (B,T,512)} -> action (B, action_size)."""

    def __init__(self, cfg: LavaConfig = LavaConfig()):
        super().__init__()
        self.cfg = cfg
        d = cfg.d_model
        self.image_encoder = ConvMaxpoolEncoder()
        self.visual_proj = nn.ModuleDict({str(i): _dense(self.image_encoder.channels[i], d)
                                          for i in cfg.pyramid_fuse_layers})
        self.lang_proj = _dense(cfg.lang_dim, d)
        self.cross = nn.ModuleList(CrossLayer(d, 2, d, cfg.dropout) for _ in range(cfg.num_layers))
        self.fuse_norm = nn.LayerNorm(d)
        self.temporal_in = _dense(d, d)
        self.temporal = nn.ModuleList(SelfLayer(d, cfg.num_heads, d, cfg.dropout)
                                      for _ in range(cfg.temporal_layers))
        self.temporal_norm = nn.LayerNorm(d)
        self.head = DenseResnet(d, cfg.dense_resnet_width, cfg.dense_resnet_blocks)
        self.action_projection = _dense(cfg.dense_resnet_width, cfg.action_size)
        self.drop = nn.Dropout(cfg.dropout)
        self.register_buffer("pos_t", sincos_1d(cfg.sequence_length, d), persistent=False)
        self._pos2d = {}

    def _pos(self, h: int, w: int, device) -> torch.Tensor:
        key = (h, w, str(device))
        if key not in self._pos2d:
            self._pos2d[key] = sincos_2d(self.cfg.d_model, h, w).to(device)
        return self._pos2d[key]

    def encode(self, rgb: torch.Tensor, lang: torch.Tensor) -> torch.Tensor:
        b, t = rgb.shape[:2]
        x = rgb.reshape(b * t, *rgb.shape[2:])
        if x.dtype == torch.uint8:
            x = x.float() / 255.0
        x = x.permute(0, 3, 1, 2).contiguous()                         # NHWC -> NCHW
        levels = self.image_encoder(x)
        d = self.cfg.d_model
        sent = []
        for i in self.cfg.pyramid_fuse_layers:
            f = levels[i]                                               # (N, C, h, w)
            h, w = f.shape[-2:]
            v = self.visual_proj[str(i)](f.flatten(2).transpose(1, 2)) * math.sqrt(d)
            sent.append(v + self._pos(h, w, v.device))
        pixels = self.drop(torch.cat(sent, dim=1))                      # (N, sum hw, d)
        q = self.drop(self.lang_proj(lang.reshape(b * t, -1).float()) * math.sqrt(d))[:, None]
        for layer in self.cross:
            q = layer(pixels, q)
        z = self.fuse_norm(q[:, 0]).reshape(b, t, d)
        z = self.temporal_in(z) * math.sqrt(d) + self.pos_t[:t]
        z = self.drop(z)
        for layer in self.temporal:
            z = layer(z)
        return self.temporal_norm(z.mean(dim=1))

    def forward(self, obs) -> torch.Tensor:
        return self.action_projection(self.head(self.encode(obs["rgb"], obs["instruction_embedding"])))


# ---------------------------------------------------------------------------------------------------------------
# PixelLangMSE: the simple pixel-language BC network (reference language_table/train/networks/pixel.py:25-111)
class LanguageFusion(nn.Module):
    """Multiplicative language fusion: Dense(lang -> C) tiled over H x W, times the feature map."""

    def __init__(self, lang_dim: int, channels: int):
        super().__init__()
        self.proj = _dense(lang_dim, channels)

    def forward(self, lang, image):                                      # lang (B, D), image (B, C, H, W)
        return image * self.proj(lang)[:, :, None, None]


class ConvMaxpoolLanguageEncoder(nn.Module):
    """4 x [conv3x3 SAME (+bias) -> language fusion from the 2nd conv on -> ReLU -> maxpool 2 VALID], spatial
    mean, a final multiplicative language gate, ReLU, LayerNorm (``pixel.py:47-80``, ``fuse_from = 2``)."""

    def __init__(self, in_ch: int, lang_dim: int = 512, channels: Sequence[int] = (32, 64, 128, 256),
                 fuse_from: int = 2):
        super().__init__()
        convs, fuses, cin = [], [], in_ch
        for i, c in enumerate(channels):
            convs.append(_flax_conv(cin, c, 3))
            fuses.append(LanguageFusion(lang_dim, c) if fuse_from <= i + 1 else None)
            cin = c
        self.convs = nn.ModuleList(convs)
        self.fuses = nn.ModuleList(f if f is not None else nn.Identity() for f in fuses)
        self._fuse = [f is not None for f in fuses]
        self.lang_gate = _dense(lang_dim, channels[-1]) if fuse_from <= len(channels) + 1 else None
        self.norm = nn.LayerNorm(channels[-1], eps=1e-6)

    def forward(self, x, lang):                                          # x (B, C, H, W)
        for conv, fuse, on in zip(self.convs, self.fuses, self._fuse):
            x = conv(x)
            if on:
                x = fuse(lang, x)
            x = F.max_pool2d(F.relu(x), 2)
        x = x.mean(dim=(2, 3))
        if self.lang_gate is not None:
            x = x * self.lang_gate(lang)
        return self.norm(F.relu(x))


class PixelLangMSE(nn.Module):
    """obs {rgb (B, N, W, H, C) in [0,1] or uint8, clip_embedding / instruction_embedding (B, N, 512)}
    -> action (B, action_size).

    The N frames are stacked channel-wise with the reference's raw reshape ``(b, n, w, h, c) -> (b, w, h, c*n)``
    (a reinterpretation of memory, not a transpose -- kept as is), the last step's language embedding conditions
    the encoder, then the dense resnet and an N(0, 0.05)-initialised action projection (``pixel.py:84-111``)."""

    def __init__(self, action_size: int = 2, dense_resnet_width: int = 1024, dense_resnet_num_blocks: int = 2,
                 sequence_length: int = 4, lang_dim: int = 512):
        super().__init__()
        self.encoder = ConvMaxpoolLanguageEncoder(3 * sequence_length, lang_dim)
        self.dense_resnet = DenseResnet(256, dense_resnet_width, dense_resnet_num_blocks)
        self.action_projection = _dense(dense_resnet_width, action_size)

    def forward(self, obs) -> torch.Tensor:
        rgb = obs["rgb"]
        if rgb.dtype == torch.uint8:
            rgb = rgb.float() / 255.0
        b, n, w, h, c = rgb.shape
        rgb = rgb.contiguous().reshape(b, w, h, c * n)                  # reference's channel stacking
        lang = obs.get("clip_embedding", obs.get("instruction_embedding"))[:, -1]
        x = self.encoder(rgb.permute(0, 3, 1, 2), lang.float())
        return self.action_projection(self.dense_resnet(x))
