#!/usr/bin/env python3
"""VGPR / SGPR / scratch / LDS per kernel of a built object (build/hip/<unit>.o), from the code object's metadata
notes -- the register budget check for a kernel edit, no GPU needed.

    python tools/kernel_resources.py build/hip/dwconv.hip.o [name-filter]
"""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_audit  # noqa: E402

LLVM = "/opt/rocm/lib/llvm/bin"


def code_object(obj: str, tmp: str) -> str:
    base = os.path.join(tmp, os.path.basename(obj))
    fat, co = base + ".fatbin", base + ".co"
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", obj, os.devnull],
                   check=True, capture_output=True)
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fat}",
                    f"--targets=hipv4-amdgcn-amd-amdhsa--{isa_audit.ARCH}", f"--output={co}"], check=True,
                   capture_output=True)
    return co


def resources(obj: str):
    with tempfile.TemporaryDirectory() as tmp:
        co = code_object(obj, tmp)
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True, capture_output=True,
                               text=True).stdout
        names = subprocess.run(["c++filt"], input="\n".join(
            re.findall(r"\.name:\s+(\S+)", notes)), capture_output=True, text=True).stdout.splitlines()
    out = []
    blocks = re.split(r"\n\s+- \.agpr_count", notes)[1:]
    for blk, nm in zip(blocks, names):
        get = lambda k: int(re.search(rf"\.{k}:\s+(\d+)", blk).group(1)) if re.search(rf"\.{k}:\s+(\d+)", blk) else -1
        out.append((nm, get("vgpr_count"), get("sgpr_count"), get("private_segment_fixed_size"),
                    get("group_segment_fixed_size"), get("vgpr_spill_count")))
    return out


if __name__ == "__main__":
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    for nm, v, sg, scr, lds, spill in resources(sys.argv[1]):
        if flt in nm:
            print(f"vgpr {v:4d} sgpr {sg:3d} scratch {scr:5d} spill {spill:3d} lds {lds:6d}  {nm[:150]}")
