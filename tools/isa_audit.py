#!/usr/bin/env python3
"""Audit the gfx950 machine code of the built kernels for instruction forms this project does not ship.

Rules:
  * (csrc/kernels/common.h NO_PACKED_FP32) no packed fp32 VALU op (v_pk_fma/mul/add_f32) whose low lane reads a HIGH
    source element (a non-default ``op_sel:[...]``).  Such an instruction in se_wsum_part dropped its low-lane product
    for 16 lanes when two processes shared the GPU (profiles/r4_se_dp_rootcause.md).
  * (csrc/kernels/imgproc.hip clip8_opaque) no ``v_ashr_pk_u8_i32``: the compiler fused two clamps + byte packs into
    it and then OR-ed the upper bytes into a destination whose high half still held an old value (byte 2 of every
    packed word was corrupted).

Works on the objects ``build.py`` leaves in build/hip (no GPU needed): the .hip_fatbin section of each object is
unbundled to its gfx950 code object and disassembled with the ROCm LLVM tools.

  python tools/isa_audit.py            # prints offending (object, kernel, instruction) and exits 1 if any
"""
from __future__ import annotations

import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "build", "hip")
LLVM = "/opt/rocm/lib/llvm/bin"
ARCH = os.environ.get("RT1_OFFLOAD_ARCH", "gfx950")
_PK_OPSEL = re.compile(r"\bv_pk_(fma|mul|add)_f32\b.*\bop_sel:\[|\bv_ashr_pk_u8_i32\b")
_FUNC = re.compile(r"^[0-9a-f]+ <(.+)>:$")


def tools_available() -> bool:
    return all(os.path.exists(os.path.join(LLVM, t)) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-objdump"))


def disassemble(obj: str, tmp: str) -> str:
    """gfx950 disassembly of one host object's embedded device code ('' if it has none)."""
    base = os.path.join(tmp, os.path.basename(obj))
    fat, co = base + ".fatbin", base + ".co"
    r = subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", obj, os.devnull],
                       capture_output=True, text=True)
    if r.returncode != 0 or not os.path.exists(fat):
        return ""
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fat}",
                    f"--targets=hipv4-amdgcn-amd-amdhsa--{ARCH}", f"--output={co}"], check=True,
                   capture_output=True)
    return subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "-C", co], check=True, capture_output=True,
                          text=True).stdout


def current_objects():
    """build/hip objects whose kernel source still exists (a removed kernel's stale object is not shipped)."""
    src = os.path.join(ROOT, "pytorch_rt1_for_distributed_training_amd", "csrc")
    return [o for o in sorted(glob.glob(os.path.join(BUILD, "*.o")))
            if os.path.exists(os.path.join(src, "kernels", os.path.basename(o)[:-2]))
            or os.path.exists(os.path.join(src, os.path.basename(o)[:-2]))]


def audit(objs=None):
    """[(object, kernel, instruction)] of every forbidden instruction in ``objs`` (default: build/hip/*.o)."""
    objs = current_objects() if objs is None else objs
    bad = []
    with tempfile.TemporaryDirectory() as tmp:
        for obj in objs:
            fn = "?"
            for line in disassemble(obj, tmp).splitlines():
                m = _FUNC.match(line.strip())
                if m:
                    fn = m.group(1)
                elif _PK_OPSEL.search(line):
                    bad.append((os.path.basename(obj), fn, line.split("//")[0].strip()))
    return bad


def main():
    objs = current_objects()
    if not objs:
        raise SystemExit(f"no objects under {BUILD}: run `python build.py` first")
    bad = audit(objs)
    for obj, fn, ins in bad:
        print(f"{obj}: {fn[:100]}: {ins}")
    print(f"{len(objs)} objects, {len(bad)} forbidden instructions")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
