"""Loader for the in-tree HIP extension ``_rt1_hip`` (built by ``build.py``)."""
from __future__ import annotations

import importlib
import importlib.util
import os
import sys

_MOD = None
_ERR = None
HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)


def load():
    """Import the compiled extension; raise loudly if it is missing."""
    global _MOD, _ERR
    if _MOD is not None:
        return _MOD
    try:
        import torch  # noqa: F401  (loads libamdhip64 / libtorch_hip first)
        alt = os.environ.get("RT1_HIP_SO")   # A/B kernel variant built by `build.py --variant NAME`
        if alt:
            name = "pytorch_rt1_for_distributed_training_amd._rt1_hip"
            spec = importlib.util.spec_from_file_location(name, alt)
            _MOD = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(_MOD)
            sys.modules[name] = _MOD
            return _MOD
        _MOD = importlib.import_module("pytorch_rt1_for_distributed_training_amd._rt1_hip")
    except ImportError as e:
        _ERR = e
        raise ImportError(
            "HIP extension _rt1_hip is not built. Run `python build.py` (hipcc --offload-arch=gfx950) "
            f"in the repo root. Original error: {e}") from e
    return _MOD


def available() -> bool:
    try:
        load()
        return True
    except ImportError:
        return False
