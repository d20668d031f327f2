"""MI355X-native RT-1 (Robotics Transformer 1) training framework.

Layers (bottom-up): ``csrc`` HIP/CDNA4 kernels + C++ runtime -> ``ops`` (Python
bindings, autograd functions) -> ``models`` (RT-1 modules, checkpoint-schema
compatible with the reference) -> ``parallel`` (RCCL data parallel) ->
``engine`` (train step, optimizer, graphs) -> ``data`` / ``utils`` / ``eval``.
"""
__version__ = "0.1.0"

from .config import RT1Config, preset  # noqa: F401
from . import spaces  # noqa: F401
