"""HIP/CDNA4 kernels for RT-1 (Python side).

``_ext`` loads the in-tree extension built from ``csrc/`` (gfx950).  On a GPU
box the extension is REQUIRED for the ``hip`` backend: ``load()`` raises with
the build command instead of silently falling back to eager PyTorch.
"""
from __future__ import annotations

from ._ext import available, load  # noqa: F401


def install(model, cfg):
    """Route the model's hot paths through the fused HIP implementation."""
    from .fused_model import FusedRT1
    model.fused = FusedRT1(model, cfg)
    return model
