"""On-device image augmentation of the behaviour-cloning pipeline.

Behavioural spec: ``language_table/train/input_pipeline_rlds.py:325-387`` (``DecodeAndRandomResizedCrop``: one
random crop of ``factor x`` the frame size per window, then a bilinear resize to (180, 320), values /255) and
``:390-457`` (``PhotometricDistortions``: brightness +-0.1, saturation x[0.8, 1.2], hue +-0.03 turns, contrast
x[0.8, 1.2], in that order, one draw per window, clipped to [0, 1]).

The reference runs these per example on the tf.data CPU workers.  Here they are batched tensor ops on the GPU
after the host->device copy (uint8 crosses PCIe, 4x fewer bytes than float): one gather-free crop per sample via
``F.grid_sample`` over the whole [B*T] stack, and the colour ops as fused elementwise math over [B, T, 3, H, W]
(HSV round trip only for the hue term).  Draws come from a ``torch.Generator`` so a run is reproducible.
"""
from __future__ import annotations

import dataclasses
from typing import Optional, Tuple

import torch
import torch.nn.functional as F


def _to_float_cf(rgb: torch.Tensor) -> torch.Tensor:
    """[B, T, H, W, 3] uint8 / float -> [B, T, 3, H, W] float32 in [0, 1]."""
    x = rgb.permute(0, 1, 4, 2, 3)
    return x.float() / 255.0 if rgb.dtype == torch.uint8 else x.float()


def random_resized_crop(rgb: torch.Tensor, factor: Optional[float], size: Tuple[int, int],
                        generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """[B, T, H, W, 3] -> [B, T, 3, h, w] float: an axis-aligned crop of (factor*H, factor*W) at a random
    integer offset (shared by the T frames of a window), bilinearly resized to ``size``."""
    x = _to_float_cf(rgb)
    B, T, C, H, W = x.shape
    if factor is None or factor >= 1.0:
        ch, cw = float(H), float(W)
        oy = torch.zeros(B, device=x.device)
        ox = torch.zeros(B, device=x.device)
    else:
        ch, cw = H * factor, W * factor
        # integer offsets in [0, H - ch), like tf.random.stateless_uniform(maxval=int(H - ch))
        oy = torch.floor(torch.rand(B, generator=generator, device=generator.device if generator else "cpu")
                         * max(int(H - ch), 1)).to(x.device)
        ox = torch.floor(torch.rand(B, generator=generator, device=generator.device if generator else "cpu")
                         * max(int(W - cw), 1)).to(x.device)
    h, w = size
    # output pixel centres (half-pixel convention) -> input coordinates of the crop -> [-1, 1] grid
    ys = (torch.arange(h, device=x.device, dtype=torch.float32) + 0.5) * (ch / h)
    xs = (torch.arange(w, device=x.device, dtype=torch.float32) + 0.5) * (cw / w)
    gy = ((oy[:, None] + ys[None, :]) / H) * 2 - 1                        # [B, h]
    gx = ((ox[:, None] + xs[None, :]) / W) * 2 - 1                        # [B, w]
    grid = torch.stack(torch.broadcast_tensors(gx[:, None, :], gy[:, :, None]), dim=-1)   # [B, h, w, 2]
    grid = grid[:, None].expand(B, T, h, w, 2).reshape(B * T, h, w, 2)
    out = F.grid_sample(x.reshape(B * T, C, H, W), grid, mode="bilinear", padding_mode="border",
                        align_corners=False)
    return out.view(B, T, C, h, w)


def _rgb_to_hsv(x: torch.Tensor):
    r, g, b = x.unbind(-3)
    mx, _ = x.max(-3)
    mn, _ = x.min(-3)
    d = mx - mn
    s = torch.where(mx > 0, d / mx.clamp_min(1e-12), torch.zeros_like(mx))
    dd = d.clamp_min(1e-12)
    h = torch.where(mx == r, ((g - b) / dd) % 6, torch.where(mx == g, (b - r) / dd + 2, (r - g) / dd + 4)) / 6
    h = torch.where(d > 0, h, torch.zeros_like(h))
    return h, s, mx


def _hsv_to_rgb(h, s, v):
    h6 = (h % 1.0) * 6
    k = torch.stack([(5 + h6) % 6, (3 + h6) % 6, (1 + h6) % 6], dim=-3)
    return v.unsqueeze(-3) - v.unsqueeze(-3) * s.unsqueeze(-3) * (torch.minimum(k, 4 - k).clamp(0, 1))


@dataclasses.dataclass
class PhotometricDistortions:
    brightness_max_delta: float = 0.1
    contrast_lower: float = 0.8
    contrast_upper: float = 1.2
    hue_max_delta: float = 0.03
    saturation_lower: float = 0.8
    saturation_upper: float = 1.2

    def __call__(self, x: torch.Tensor, generator: Optional[torch.Generator] = None) -> torch.Tensor:
        """x [B, T, 3, H, W] in [0, 1] -> same; one draw of each factor per window (b)."""
        B = x.shape[0]
        dev = generator.device if generator is not None else "cpu"

        def u(lo, hi):
            return (torch.rand(B, generator=generator, device=dev) * (hi - lo) + lo).to(x.device).view(B, 1, 1, 1, 1)

        if self.brightness_max_delta:
            x = (x + u(-self.brightness_max_delta, self.brightness_max_delta)).clamp(0, 1)
        sat = (self.saturation_lower, self.saturation_upper) != (1.0, 1.0)
        if sat or self.hue_max_delta:
            h, s, v = _rgb_to_hsv(x)
            if sat:
                s = (s * u(self.saturation_lower, self.saturation_upper).squeeze(2)).clamp(0, 1)
                x = _hsv_to_rgb(h, s, v).clamp(0, 1)
            if self.hue_max_delta:
                if sat:
                    h, s, v = _rgb_to_hsv(x)
                h = h + u(-self.hue_max_delta, self.hue_max_delta).squeeze(2)
                x = _hsv_to_rgb(h, s, v).clamp(0, 1)
        if (self.contrast_lower, self.contrast_upper) != (1.0, 1.0):
            mean = x.mean(dim=(-2, -1), keepdim=True)              # per frame, per channel (tf.adjust_contrast)
            x = ((x - mean) * u(self.contrast_lower, self.contrast_upper) + mean).clamp(0, 1)
        return x


@dataclasses.dataclass
class BCAugment:
    """crop + resize + photometric distortions for a BC batch; returns rgb as [B, T, H, W, 3] float in [0, 1]
    (the layout the LAVA encoder takes)."""
    random_crop_factor: Optional[float] = 0.95
    resize_size: Tuple[int, int] = (180, 320)
    photometric: Optional[PhotometricDistortions] = dataclasses.field(default_factory=PhotometricDistortions)
    seed: int = 0

    def __post_init__(self):
        self._gen = None

    def __call__(self, rgb: torch.Tensor, train: bool = True) -> torch.Tensor:
        if self._gen is None:
            self._gen = torch.Generator(device="cpu")
            self._gen.manual_seed(self.seed)
        if not train:
            # eval: the deterministic central crop of the same factor (the env wrapper's CentralCrop)
            x = central_crop(rgb, self.random_crop_factor, self.resize_size)
        else:
            x = random_resized_crop(rgb, self.random_crop_factor, self.resize_size, self._gen)
            if self.photometric is not None:
                x = self.photometric(x, self._gen)
        return x.permute(0, 1, 3, 4, 2).contiguous()


def central_crop(rgb: torch.Tensor, factor: Optional[float], size: Tuple[int, int]) -> torch.Tensor:
    x = _to_float_cf(rgb)
    B, T, C, H, W = x.shape
    f = 1.0 if factor is None else min(factor, 1.0)
    ch, cw = int(H * f), int(W * f)
    oy, ox = (H - ch) // 2, (W - cw) // 2
    x = x[..., oy:oy + ch, ox:ox + cw].reshape(B * T, C, ch, cw)
    return F.interpolate(x, size=size, mode="bilinear", align_corners=False).view(B, T, C, *size)
