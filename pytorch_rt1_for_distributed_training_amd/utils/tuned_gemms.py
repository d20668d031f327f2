"""hipBLASLt solution choices for the library GEMMs the step still issues (PyTorch TunableOp results tuned on MI355X).

The encoder's skinny / tall 1x1 convs run on the hand-written MFMA kernels; what stays on hipBLASLt (transformer
projections, the SE MLP, the wide-N products of blocks 18-25, conv1x1) uses the library's default heuristic per shape.
``tools/gpu/tunableop.sh`` times every candidate solution of those shapes once on an MI355X and writes
``tuning/tunableop_results<device>.csv``; with the env set below PyTorch dispatches each GEMM to the recorded
solution and never tunes at run time (0.6 ms/step, ``profiles/r2_tunableop_ab.log``).  The file carries validator lines
(PyTorch, HIP, hipBLASLt, rocBLAS versions, gfx arch): on a mismatching install PyTorch ignores it and the defaults
apply.  ``RT1_TUNED_GEMMS=0`` turns it off.  Call before the first GEMM (before ``import torch`` to be safe).
"""
from __future__ import annotations

import os

_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tuning")


def enable_tuned_gemms() -> bool:
    if os.environ.get("RT1_TUNED_GEMMS", "1") == "0" or "PYTORCH_TUNABLEOP_ENABLED" in os.environ:
        return False
    if not os.path.exists(os.path.join(_DIR, "tunableop_results0.csv")):
        return False
    os.environ["PYTORCH_TUNABLEOP_ENABLED"] = "1"
    os.environ["PYTORCH_TUNABLEOP_TUNING"] = "0"            # read-only: dispatch to the recorded solutions
    os.environ["PYTORCH_TUNABLEOP_FILENAME"] = os.path.join(_DIR, "tunableop_results.csv")   # + device ordinal
    return True
