"""Same-box A/B switches of the fused training path, in one place.

Every default below is the measured winner; the comment at the switch's use site names the log that decided it.
``RT1_AB`` overrides any of them for an A/B run without a rebuild::

    RT1_AB=dw_fused=0,xmode=all python bench.py --steps 20

(``tools/gpu/ab_env.sh`` with ``AB_ENV=<name>``, ``tools/parity_ablation.py``).  An unknown name raises, so a typo
cannot silently measure the default twice.  Kernel tuning constants live in the HIP sources as ``constexpr`` values
(an A/B of one is a ``build.py --variant`` build); the only other ``RT1_*`` environment variables are runtime and
debugging knobs (``RT1_SYNC_CHECK``, ``RT1_BLOCK_TIMING``, ``RT1_SE_DEBUG``, ``RT1_TUNED_GEMMS``, ...), listed in
README.md.
"""
from __future__ import annotations

import os
from typing import Dict

DEFAULTS: Dict[str, str] = {
    # backbone (ops/backbone.py)
    "pw_tall": "1",        # tall-skinny MFMA kernel for wide-K narrow-N 1x1 convs (0: hipBLASLt)
    "g256": "1",           # top / block-25 expand on gemm256.hip with the BN-statistics epilogue
    "wgrad_mfma": "1",     # streaming MFMA weight-gradient kernel on the mid-resolution shapes
    "wgrad_deep": "1",     # ... and on the two deep shapes of _WGRAD_TILE
    "dw_fused": "1",       # fused depthwise backward
    "dw_s2_fused": "1",    # ... for the stride-2 blocks too
    "dw_variant": "1",     # 1: the unified single-pass stride-1 kernel, 0: the two-pass one
    "dw_res": "1",         # residual gradient in the unified depthwise backward's store (block 1)
    "pw_pro": "1",         # project-conv operand prologue silu(bn2(y2)) * gate inside the GEMM
    "proj_bwd": "1",       # project-conv backward from (dy3, y2) per frame (projbwd.hip)
    "se_fused": "1",       # fused SE MLP kernels (se.hip)
    "stem_in_block0": "1", # stem BN + SiLU applied inside block 0
    "stem_bn_bwd": "1",    # stem BN backward folded into the stem weight-gradient staging
    "pw_bwd_z": "1",       # y-free (dz-mode) expand backward
    "pw_z_wide": "1",      # ... for the wide expand convs
    "z_gemm": "1",         # dz-mode dgrad on gemm.hip: 1 blocks 19-24 (r5 re-check: +0.15 % over 2), 2 blocks 19-25, 0 off
    "xmode": "1",          # y1-free expand blocks: 1 block 2, all every supported block, 0 none
    "gram_bn": "1",        # BN1 of the wide expand convs from Gram moments of the block input
    "gemm_proj": "1",      # deep project convs on gemm.hip with prologue and BN3-statistics epilogue
    "gemm_proj_dgrad": "1",  # ... and their data gradients
    "tall_res": "1",       # residual gradient in the wide dz-mode dgrad's epilogue
    "gram_sx": "1",        # x's column sums from the Gram-matrix wgrad pass (ops/backbone.py gram_moments)
    # transformer (ops/attention.py)
    "tf_wgrad": "1",       # transformer weight gradients on the MFMA wgrad kernel
    "tf_gemm": "1",        # transformer projections of ops/attention.py _TF_GEMM_CFG on gemm.hip's small tiles
    "tf_fuse_ln": "1",     # next LayerNorm formed in the residual kernel, LN2 backward emits the bf16 operand
    # data parallel (parallel/flat.py)
    "multi_copy": "1",     # one-launch gradient gather into the flat bucket
}


def _parse(spec: str) -> Dict[str, str]:
    out: Dict[str, str] = {}
    for item in filter(None, (s.strip() for s in spec.split(","))):
        name, sep, value = item.partition("=")
        name = name.strip()
        if not sep or name not in DEFAULTS:
            raise ValueError(f"RT1_AB: unknown or malformed switch {item!r}; known: {', '.join(sorted(DEFAULTS))}")
        out[name] = value.strip()
    return out


_OVERRIDES = _parse(os.environ.get("RT1_AB", ""))


def get(name: str) -> str:
    """Current value of switch ``name`` (the default unless ``RT1_AB`` overrides it)."""
    if name not in DEFAULTS:
        raise KeyError(name)
    return _OVERRIDES.get(name, DEFAULTS[name])


def on(name: str) -> bool:
    return get(name) != "0"


def overrides() -> Dict[str, str]:
    """The switches this process runs off their defaults (recorded in bench / trainer metadata)."""
    return dict(_OVERRIDES)
