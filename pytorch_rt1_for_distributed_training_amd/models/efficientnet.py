"""FiLM-conditioned EfficientNet-B3 backbone (RT-1 image encoder body).

Behavioural spec: ``pytorch_robotics_transformer/film_efficientnet/
film_efficientnet_encoder.py`` (block table ``:36-99``, ``round_filters`` /
``round_repeats`` ``:123-140``, ``SeModule`` ``:142-161``, ``MBConvBlock``
``:164-244``, ``EfficientNet`` ``:246-373``, B3 factory ``:429-442``).

Module/attribute names are kept identical to the reference because they ARE
the checkpoint format (``...net.blocks.{i}.block.{j}.{0,1}.*``,
``...net.films.{i}._projection_*``); the implementation is
independent.  Differences by design:

* no torchvision dependency (``ConvBNAct`` / ``StochasticDepth`` are local);
* the forward is memory-format agnostic and runs channels-last on MI355X, where
  every 1x1 conv is a plain GEMM over ``N*H*W`` rows and the depthwise conv
  vectorises over channels;
* ``MBConvBlock.forward`` dispatches to the fused HIP implementation
  (``ops.mbconv``) when the model backend is ``hip``; the eager body below is
  the numerical oracle for it.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .film import FilmConditioning

# EfficientNet-B0 stage table (Tan & Le 2019, Table 1):
# (kernel, repeats, in_ch, out_ch, expand_ratio, stride)
_B0_STAGES = (
    (3, 1, 32, 16, 1, 1),
    (3, 2, 16, 24, 6, 2),
    (5, 2, 24, 40, 6, 2),
    (3, 3, 40, 80, 6, 2),
    (5, 3, 80, 112, 6, 1),
    (5, 4, 112, 192, 6, 2),
    (3, 1, 192, 320, 6, 1),
)
SE_RATIO = 0.25


def round_filters(filters: float, divisor: int, width_coefficient: float) -> int:
    """Scale a channel count by the width multiplier, snapping to ``divisor``
    (round-half-up at divisor/2) and never losing more than 10%."""
    scaled = filters * width_coefficient
    snapped = max(divisor, int(scaled + divisor / 2) // divisor * divisor)
    if snapped < 0.9 * scaled:
        snapped += divisor
    return int(snapped)


def round_repeats(repeats: int, depth_coefficient: float) -> int:
    return int(math.ceil(depth_coefficient * repeats))


@dataclass(frozen=True)
class BlockSpec:
    index: int
    kernel: int
    in_ch: int
    out_ch: int
    expand_ratio: int
    stride: int
    drop_rate: float

    @property
    def expand_ch(self) -> int:
        return self.in_ch * self.expand_ratio

    @property
    def se_ch(self) -> int:
        # NB: the reference sizes the squeeze by the *block input* width
        # (``film_efficientnet_encoder.py:146``), not the expanded width.
        return max(1, int(self.in_ch * SE_RATIO))

    @property
    def has_skip(self) -> bool:
        return self.stride == 1 and self.in_ch == self.out_ch


def block_specs(width_coefficient: float = 1.2, depth_coefficient: float = 1.4,
                drop_connect_rate: float = 0.2, divisor: int = 8) -> List[BlockSpec]:
    total = sum(round_repeats(r, depth_coefficient) for (_, r, *_rest) in _B0_STAGES)
    specs: List[BlockSpec] = []
    for (k, reps, cin, cout, e, s) in _B0_STAGES:
        cin = round_filters(cin, divisor, width_coefficient)
        cout = round_filters(cout, divisor, width_coefficient)
        for j in range(round_repeats(reps, depth_coefficient)):
            b = len(specs)
            specs.append(BlockSpec(b, k, cin if j == 0 else cout, cout, e, s if j == 0 else 1,
                                   drop_connect_rate * b / float(total)))
    return specs


def conv_out_size(n: int, k: int, s: int) -> int:
    p = (k - 1) // 2
    return (n + 2 * p - k) // s + 1


def feature_map_size(height: int, width: int, specs: Optional[List[BlockSpec]] = None):
    """Spatial size of the backbone output for an input of height x width."""
    specs = specs or block_specs()
    h, w = conv_out_size(height, 3, 2), conv_out_size(width, 3, 2)
    for sp in specs:
        h, w = conv_out_size(h, sp.kernel, sp.stride), conv_out_size(w, sp.kernel, sp.stride)
    return h, w


class ConvBNAct(nn.Sequential):
    """conv(bias=False) -> BatchNorm2d -> optional SiLU.  Indices 0/1/2 match
    torchvision's ``Conv2dNormActivation`` so state-dict keys line up."""

    def __init__(self, cin: int, cout: int, kernel: int, stride: int = 1, groups: int = 1, act: bool = True):
        mods = [nn.Conv2d(cin, cout, kernel, stride, (kernel - 1) // 2, groups=groups, bias=False),
                nn.BatchNorm2d(cout)]
        if act:
            mods.append(nn.SiLU())
        super().__init__(*mods)

    @property
    def conv(self) -> nn.Conv2d:
        return self[0]

    @property
    def bn(self) -> nn.BatchNorm2d:
        return self[1]

    @property
    def has_act(self) -> bool:
        return len(self) > 2


class StochasticDepth(nn.Module):
    """Per-sample ("row") drop-path: ``x * Bernoulli(1-p) / (1-p)`` in training."""

    def __init__(self, p: float):
        super().__init__()
        self.p = float(p)

    def keep_mask(self, n: int, device, dtype=torch.float32) -> torch.Tensor:
        keep = 1.0 - self.p
        return torch.empty(n, device=device, dtype=dtype).bernoulli_(keep).div_(keep)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not self.training or self.p == 0.0:
            return x
        return x * self.keep_mask(x.shape[0], x.device, x.dtype).view(-1, 1, 1, 1)


class SqueezeExcite(nn.Module):
    def __init__(self, expand_ch: int, se_ch: int):
        super().__init__()
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc1 = nn.Conv2d(expand_ch, se_ch, 1)
        self.silu0 = nn.SiLU()
        self.fc2 = nn.Conv2d(se_ch, expand_ch, 1)
        self.act = nn.Sigmoid()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        s = x.mean(dim=(2, 3), keepdim=True)
        s = torch.sigmoid(self.fc2(F.silu(self.fc1(s))))
        return x * s


class MBConvBlock(nn.Module):
    """Inverted-residual block: [expand 1x1] -> depthwise kxk -> SE -> project 1x1,
    with drop-path + identity skip when shape-preserving."""

    def __init__(self, spec: BlockSpec):
        super().__init__()
        self.spec = spec
        layers: List[nn.Module] = []
        if spec.expand_ratio != 1:
            layers.append(ConvBNAct(spec.in_ch, spec.expand_ch, 1))
        layers.append(ConvBNAct(spec.expand_ch, spec.expand_ch, spec.kernel, spec.stride, groups=spec.expand_ch))
        layers.append(SqueezeExcite(spec.expand_ch, spec.se_ch))
        layers.append(ConvBNAct(spec.expand_ch, spec.out_ch, 1, act=False))
        self.block = nn.Sequential(*layers)
        if spec.drop_rate > 0:
            self.dropout = StochasticDepth(spec.drop_rate)

    # convenience views used by the fused path
    @property
    def expand(self) -> Optional[ConvBNAct]:
        return self.block[0] if self.spec.expand_ratio != 1 else None

    @property
    def depthwise(self) -> ConvBNAct:
        return self.block[1 if self.spec.expand_ratio != 1 else 0]

    @property
    def se(self) -> SqueezeExcite:
        return self.block[-2]

    @property
    def project(self) -> ConvBNAct:
        return self.block[-1]

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        y = self.block(x)
        if self.spec.has_skip:
            if self.spec.drop_rate > 0:
                y = self.dropout(y)
            y = x + y
        return y


class FiLMEfficientNet(nn.Module):
    """EfficientNet body (no classification top unless ``include_top``) with a
    FiLM layer after every MBConv block."""

    def __init__(self, width_coefficient: float = 1.2, depth_coefficient: float = 1.4,
                 drop_connect_rate: float = 0.2, include_film: bool = True, text_vector_size: int = 512,
                 include_top: bool = False, classes: int = 1000, dropout_rate: float = 0.3, divisor: int = 8):
        super().__init__()
        self.include_film = include_film
        self.include_top = include_top
        self.specs = block_specs(width_coefficient, depth_coefficient, drop_connect_rate, divisor)
        stem_ch = round_filters(32, divisor, width_coefficient)
        self.convNormAct0 = ConvBNAct(3, stem_ch, 3, 2)
        self.blocks = nn.ModuleList(MBConvBlock(s) for s in self.specs)
        if include_film:
            self.films = nn.ModuleList(FilmConditioning(s.out_ch, text_vector_size) for s in self.specs)
        top_ch = round_filters(1280, divisor, width_coefficient)
        self.convNormAct1 = ConvBNAct(self.specs[-1].out_ch, top_ch, 1)
        self.out_channels = top_ch
        if include_top:
            self.glovalAvePool = nn.AdaptiveAvgPool2d(1)
            self.dropout = nn.Dropout(dropout_rate) if dropout_rate > 0 else nn.Identity()
            self.fc = nn.Linear(top_ch, classes)

    def forward(self, x: torch.Tensor, context: Optional[torch.Tensor] = None) -> torch.Tensor:
        x = self.convNormAct0(x)
        if self.include_film:
            for blk, film in zip(self.blocks, self.films):
                x = film(blk(x), context)
        else:
            for blk in self.blocks:
                x = blk(x)
        x = self.convNormAct1(x)
        if self.include_top:
            x = torch.flatten(self.glovalAvePool(x), 1)
            x = self.fc(self.dropout(x))
        return x


def load_torchvision_b3_state_dict(model: FiLMEfficientNet, official_state_dict) -> FiLMEfficientNet:
    """Map a torchvision ``efficientnet_b3`` state dict onto a FiLM-free
    backbone *positionally*, like ``load_official_pytorch_param``
    (``film_efficientnet_encoder.py:411-425``).  FiLM layers keep their
    zero init.  Load the file with ``torch.load(..., weights_only=True)``."""
    target = model.state_dict()
    keys = [k for k in target if not k.startswith("films.")]
    src = list(official_state_dict.values())
    if len(src) < len(keys):
        raise ValueError(f"official state dict has {len(src)} tensors, backbone needs {len(keys)}")
    for k, v in zip(keys, src):
        if target[k].shape != v.shape:
            raise ValueError(f"shape mismatch for {k}: {tuple(target[k].shape)} vs {tuple(v.shape)}")
        target[k] = v
    model.load_state_dict(target)
    return model
