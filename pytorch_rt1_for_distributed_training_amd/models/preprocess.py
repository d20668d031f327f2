"""Random-shift augmentation applied to RT-1 input frames.

Spec: ``film_efficientnet/preprocessors.py:37-56`` — uint8 -> [0,1] float,
zero-pad by ``int(0.07 H)`` / ``int(0.07 W)`` and crop an H x W window at ONE
random offset shared by the whole batch.  It runs at inference too
(``transformer_network.py:444-446``).

The shift is equivalent to a translated read with zero fill outside the
image, which is how the HIP stem consumes it (no padded copy is ever
materialised); ``random_shift`` returns the offsets so callers can pass them to
that fused path or keep them in device memory for graph replay.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn.functional as F


def shift_pads(height: int, width: int, ratio: float = 0.07) -> Tuple[int, int]:
    return int(height * ratio), int(width * ratio)


def random_shift(height: int, width: int, ratio: float = 0.07, generator: Optional[torch.Generator] = None):
    """Draw (dy, dx) in [-pad, +pad]: the crop origin minus the pad."""
    ud, lr = shift_pads(height, width, ratio)
    sh = int(torch.randint(0, 2 * ud + 1, (), generator=generator))
    sw = int(torch.randint(0, 2 * lr + 1, (), generator=generator))
    return sh - ud, sw - lr


def shift_images(images: torch.Tensor, dy: int, dx: int) -> torch.Tensor:
    """out[..., y, x] = images[..., y + dy, x + dx] (zero outside)."""
    h, w = images.shape[-2:]
    if dy == 0 and dx == 0:
        return images
    padded = F.pad(images, (max(-dx, 0), max(dx, 0), max(-dy, 0), max(dy, 0)))
    y0, x0 = max(dy, 0), max(dx, 0)
    return padded[..., y0:y0 + h, x0:x0 + w]


def convert_dtype_and_crop_images(images: torch.Tensor, ratio: float = 0.07, shift=None,
                                  generator: Optional[torch.Generator] = None) -> torch.Tensor:
    if images.dtype == torch.uint8:
        images = images.float() / 255.0
    elif not images.is_floating_point():
        images = images.float()
    h, w = images.shape[-2:]
    if shift is None:
        shift = random_shift(h, w, ratio, generator)
    return shift_images(images, *shift)
