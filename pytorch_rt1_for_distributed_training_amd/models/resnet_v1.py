"""ResNet V1 (He et al. 2015) -- the image trunk option of the Language-Table BC stack.

Behavioural spec: ``/root/reference/language_table/train/networks/resnet_v1.py:37-259`` (Flax).  Kept from it:

* no conv biases; BatchNorm after every conv (Flax momentum 0.9 == torch momentum 0.1, eps 1e-5);
* the basic block zero-initialises its second BN scale (Fixup-style), the bottleneck block does NOT zero its
  third BN (the reference comments about it but calls the plain norm); the classifier head is zero-initialised;
* TensorFlow ``SAME`` padding: strided convs and the stem max-pool pad asymmetrically (more on the bottom/right),
  which differs from PyTorch's symmetric ``padding=k//2`` by one pixel on strided layers;
* conv kernels use Flax's default LeCun-normal (truncated) init;
* ``MultiscaleResNet`` returns the stem conv output, the pooled stem and every stage output (6 maps).

Inputs are NHWC like the reference (``x (B, H, W, C)``); the trunk runs channels-last NCHW tensors internally.
Parameter counts equal the reference's (``resnet_v1_test.py:24-40``: ResNet50 = 25,557,032 at 1000 classes).
"""
from __future__ import annotations

import functools
import math
from typing import List, Sequence, Type

import torch
import torch.nn as nn
import torch.nn.functional as F


def _same_pad(x: torch.Tensor, k: int, s: int, value: float = 0.0) -> torch.Tensor:
    """TensorFlow SAME padding for a k x k window with stride s (extra pixel on the bottom / right)."""
    h, w = x.shape[-2:]

    def amount(n):
        out = -(-n // s)
        return max((out - 1) * s + k - n, 0)

    ph, pw = amount(h), amount(w)
    if ph == 0 and pw == 0:
        return x
    return F.pad(x, (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2), value=value)


class SameConv(nn.Conv2d):
    def __init__(self, cin: int, cout: int, k: int, stride: int = 1):
        super().__init__(cin, cout, k, stride=stride, padding=0, bias=False)
        fan_in = cin * k * k
        std = math.sqrt(1.0 / fan_in) / 0.87962566103423978      # lecun_normal (truncated at 2 sigma)
        nn.init.trunc_normal_(self.weight, std=std, a=-2 * std, b=2 * std)

    def forward(self, x):
        return super().forward(_same_pad(x, self.kernel_size[0], self.stride[0]))


def _bn(c: int, zero: bool = False) -> nn.BatchNorm2d:
    bn = nn.BatchNorm2d(c, eps=1e-5, momentum=0.1)
    if zero:
        nn.init.zeros_(bn.weight)
    return bn


class ResNetBlock(nn.Module):
    """Basic block (ResNet-18/34): two 3x3 convs; projection when the shape changes."""
    expansion = 1

    def __init__(self, cin: int, filters: int, stride: int = 1):
        super().__init__()
        self.conv1, self.bn1 = SameConv(cin, filters, 3, stride), _bn(filters)
        self.conv2, self.bn2 = SameConv(filters, filters, 3), _bn(filters, zero=True)
        self.proj = None
        if stride != 1 or cin != filters:
            self.proj = nn.Sequential(SameConv(cin, filters, 1, stride), _bn(filters))

    def forward(self, x):
        r = x if self.proj is None else self.proj(x)
        y = F.relu(self.bn1(self.conv1(x)))
        y = self.bn2(self.conv2(y))
        return F.relu(r + y)


class BottleneckResNetBlock(nn.Module):
    """Bottleneck block (ResNet-50+): 1x1 -> 3x3 (strided) -> 1x1 (4x filters)."""
    expansion = 4

    def __init__(self, cin: int, filters: int, stride: int = 1):
        super().__init__()
        out = 4 * filters
        self.conv1, self.bn1 = SameConv(cin, filters, 1), _bn(filters)
        self.conv2, self.bn2 = SameConv(filters, filters, 3, stride), _bn(filters)
        self.conv3, self.bn3 = SameConv(filters, out, 1), _bn(out)
        self.proj = None
        if stride != 1 or cin != out:
            self.proj = nn.Sequential(SameConv(cin, out, 1, stride), _bn(out))

    def forward(self, x):
        r = x if self.proj is None else self.proj(x)
        y = F.relu(self.bn1(self.conv1(x)))
        y = F.relu(self.bn2(self.conv2(y)))
        y = self.bn3(self.conv3(y))
        return F.relu(r + y)


class _Trunk(nn.Module):
    def __init__(self, block_cls: Type[nn.Module], stage_sizes: Sequence[int], width_factor: int = 1,
                 in_ch: int = 3):
        super().__init__()
        width = 64 * width_factor
        self.init_conv = SameConv(in_ch, width, 7, 2)
        self.init_bn = _bn(width)
        stages, cin = [], width
        for i, n in enumerate(stage_sizes):
            filters = width * 2 ** i
            blocks = []
            for j in range(n):
                blocks.append(block_cls(cin, filters, (1 if i == 0 or j > 0 else 2)))
                cin = filters * block_cls.expansion
            stages.append(nn.Sequential(*blocks))
        self.stages = nn.ModuleList(stages)
        self.out_channels = cin

    def _stem(self, x) -> List[torch.Tensor]:
        c = self.init_conv(x)
        y = F.relu(self.init_bn(c))
        y = F.max_pool2d(_same_pad(y, 3, 2, value=float("-inf")), 3, 2)
        return [c, y]


class ResNet(_Trunk):
    """``ResNet(num_classes, block_cls, stage_sizes, width_factor)``; forward(x NHWC) -> logits."""

    def __init__(self, num_classes: int, block_cls: Type[nn.Module], stage_sizes: Sequence[int],
                 width_factor: int = 1, in_ch: int = 3):
        super().__init__(block_cls, stage_sizes, width_factor, in_ch)
        self.head = nn.Linear(self.out_channels, num_classes)
        nn.init.zeros_(self.head.weight)
        nn.init.zeros_(self.head.bias)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = x.permute(0, 3, 1, 2)
        y = self._stem(x)[-1]
        for st in self.stages:
            y = st(y)
        return self.head(y.mean(dim=(2, 3)))


class MultiscaleResNet(_Trunk):
    """Feature pyramid: [stem conv, pooled stem, stage1, ..., stageN] as NHWC maps (reference ``:197-259``)."""

    def forward(self, x: torch.Tensor) -> List[torch.Tensor]:
        x = x.permute(0, 3, 1, 2)
        outs = self._stem(x)
        y = outs[-1]
        for st in self.stages:
            y = st(y)
            outs.append(y)
        return [o.permute(0, 2, 3, 1) for o in outs]


ResNet18 = functools.partial(ResNet, stage_sizes=(2, 2, 2, 2), block_cls=ResNetBlock)
ResNet34 = functools.partial(ResNet, stage_sizes=(3, 4, 6, 3), block_cls=ResNetBlock)
ResNet50 = functools.partial(ResNet, stage_sizes=(3, 4, 6, 3), block_cls=BottleneckResNetBlock)
ResNet101 = functools.partial(ResNet, stage_sizes=(3, 4, 23, 3), block_cls=BottleneckResNetBlock)
ResNet152 = functools.partial(ResNet, stage_sizes=(3, 8, 36, 3), block_cls=BottleneckResNetBlock)
ResNet200 = functools.partial(ResNet, stage_sizes=(3, 24, 36, 3), block_cls=BottleneckResNetBlock)


def count_parameters(m: nn.Module) -> int:
    """Trainable parameters (Flax ``params``; BN running statistics are ``batch_stats``, not counted)."""
    return sum(p.numel() for p in m.parameters())
