#!/usr/bin/env python3
"""Build the in-tree HIP extension ``_rt1_hip`` for gfx950 (MI355X).

No torch cpp_extension / hipify: every ``csrc/kernels/*.hip`` is a plain HIP
translation unit compiled by ``hipcc --offload-arch=gfx950`` (no torch headers,
seconds per file); ``csrc/bindings.cpp`` is the only unit that includes torch;
the objects are linked with ``hipcc -shared`` against the torch libraries that
are already loaded in-process.  Incremental: an object is rebuilt only when its
source or a header changed.  The ``.so`` lands inside the package so it travels
with the repo snapshot to the GPU box.

    python build.py            # build (parallel, incremental)
    python build.py --clean    # remove objects and the .so first
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "pytorch_rt1_for_distributed_training_amd")
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(ROOT, "build", "hip")
ARCH = os.environ.get("RT1_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG, "_rt1_hip" + suffix)


def _torch_paths():
    import torch
    from torch.utils.cpp_extension import include_paths, library_paths
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return include_paths(), library_paths(), abi


def _newer(src_list, out) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in src_list)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("command failed:\n" + " ".join(cmd) + "\n" + r.stdout + r.stderr)
    return r


def build(verbose: bool = False, jobs: int = 8, clean: bool = False, defines=(), out: str = None,
          build_dir: str = None) -> str:
    """Compile + link.  ``defines`` / ``out`` / ``build_dir`` build an A/B kernel variant (e.g. ``-D RT1_DW_TIMING=2``)
    into its own object dir and .so, loadable with ``RT1_HIP_SO=<path>`` (ops/_ext.py)."""
    BUILD_DIR = build_dir or BUILD
    if clean and os.path.isdir(BUILD_DIR):
        shutil.rmtree(BUILD_DIR)
    os.makedirs(BUILD_DIR, exist_ok=True)
    dflags = [f"-D{d}" for d in defines]
    headers = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    kernels = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    common = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", CSRC,
              "-Wno-unused-result", "-Wno-unused-command-line-argument"] + dflags
    jobs_list = []
    objs = []
    for src in kernels:
        obj = os.path.join(BUILD_DIR, os.path.basename(src) + ".o")
        objs.append(obj)
        if _newer([src] + headers, obj):
            jobs_list.append([HIPCC] + common + ["-munsafe-fp-atomics", "-c", src, "-o", obj])
    inc, libs, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    host_srcs = sorted(glob.glob(os.path.join(CSRC, "*.cpp")))     # bindings.cpp, comm.cpp: torch-facing host code
    for src in host_srcs:
        obj = os.path.join(BUILD_DIR, os.path.basename(src) + ".o")
        objs.append(obj)
        if not _newer([src] + headers, obj):
            continue
        cmd = [HIPCC, "-O2", "-std=c++17", "-fPIC", "-x", "c++", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
               f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=_rt1_hip", "-DTORCH_API_INCLUDE_EXTENSION_H",
               "-I", CSRC, "-I", py_inc, "-I", "/opt/rocm/include", "-Wno-unused-result",
               "-Wno-deprecated-declarations"]
        for i in inc:
            cmd += ["-isystem", i]
        jobs_list.append(cmd + ["-c", src, "-o", obj])
    if jobs_list:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            futs = {ex.submit(_run, c): c for c in jobs_list}
            for f in cf.as_completed(futs):
                f.result()
                if verbose:
                    print("built", futs[f][-1], flush=True)
    out = out or ext_path()
    if jobs_list or not os.path.exists(out):
        link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out] + objs
        for lp in libs:
            link += ["-L", lp, f"-Wl,-rpath,{lp}"]
        # librccl: resolves to the RCCL torch already loaded (same SONAME), so one RCCL per process
        link += ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python", "-lrccl"]
        _run(link)
        if verbose:
            print("linked", out, flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("-q", "--quiet", action="store_true")
    ap.add_argument("-D", "--define", action="append", default=[], help="extra -D for the kernel units (variant)")
    ap.add_argument("--variant", default=None, help="variant name: objects in build/<name>, .so in build/<name>/")
    a = ap.parse_args()
    out = bdir = None
    if a.variant:
        bdir = os.path.join(ROOT, "build", a.variant)
        out = os.path.join(bdir, os.path.basename(ext_path()))
    print(build(verbose=not a.quiet, jobs=a.jobs, clean=a.clean, defines=a.define, out=out, build_dir=bdir))


if __name__ == "__main__":
    main()
