#!/usr/bin/env python3
"""Per-step kernel time by category from a rocprofv3 --stats kernel_stats.csv (tools/gpu/prof.sh output).

usage: python tools/prof_categories.py gpurun_out/prof_<tag>/run_kernel_stats.csv [--steps 5]
       python tools/prof_categories.py --trace gpurun_out/mct   (tools/gpu/memcpy_trace.sh output)

The stats mode divides whole-run totals by the step count, so one-off kernels of the model build, the probe step and
warmup (parameter init, flat-buffer packing: ~1300 ``__amd_rocclr_copyBuffer`` dispatches) are spread over the steps.
The trace mode counts only kernels that start after a step's input H2D copy (the > 1 ms memory copy of the uint8
frame batch marks each step) and skips the first ``--skip`` steps.
"""
import argparse
import collections
import csv
import glob
import gzip
import os


def category(k: str) -> str:
    if k.startswith("Cijk") or k.startswith("Custom_Cijk"):
        return "hipBLASLt GEMM"
    if "dw_" in k:
        return "depthwise"
    if "proj_bwd" in k:
        return "project bwd (projbwd.hip)"
    if any(s in k for s in ("bn_", "block_tail", "frame_pool", "tail_bwd", "se_", "add_scaled")):
        return "BN/SE glue"
    if "pw_" in k or "wgrad" in k or "gemm_kernel" in k or "xgram" in k:
        return "pointwise MFMA"
    if "copyBuffer" in k:
        return "copyBuffer blits"
    if "stem" in k:
        return "stem"
    if any(s in k for s in ("attn", "tf_", "resid", "drop_bwd", "ln_")):
        return "transformer"
    if "tl_" in k or "head_" in k or "embed" in k:
        return "tokenlearner/head/embed"
    if "colsum" in k or "reduce_kernel" in k:
        return "reductions"
    if "adam" in k:
        return "optimizer"
    return "other"


def _open(path):
    return gzip.open(path, "rt") if path.endswith(".gz") else open(path)


def from_trace(d: str, skip: int):
    mc = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv*"), recursive=True)
    marks = sorted(int(r["Start_Timestamp"]) for f in mc for r in csv.DictReader(_open(f))
                   if int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) > 1_000_000)
    if len(marks) <= skip:
        raise SystemExit(f"only {len(marks)} step markers in {d}")
    t0, steps = marks[skip], len(marks) - skip
    tot, calls = collections.Counter(), collections.Counter()
    for f in kt:
        for r in csv.DictReader(_open(f)):
            t = int(r["Start_Timestamp"])
            if t < t0:
                continue
            c = category(r["Kernel_Name"])
            tot[c] += (int(r["End_Timestamp"]) - t) / 1e6 / steps
            calls[c] += 1 / steps
    return tot, calls, steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="?")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--trace", help="rocprofv3 output dir with kernel + memory-copy traces")
    ap.add_argument("--skip", type=int, default=2, help="trace mode: steps to skip (probe + first warmup)")
    a = ap.parse_args()
    tot = collections.Counter()
    calls = collections.Counter()
    if a.trace:
        tot, calls, n = from_trace(a.trace, a.skip)
        print(f"# {n} steps from the kernel trace")
    else:
        for r in csv.DictReader(open(a.csv)):
            c = category(r["Name"])
            tot[c] += float(r["TotalDurationNs"]) / 1e6 / a.steps
            calls[c] += int(r["Calls"]) / a.steps
    print(f"{'category':26s} {'ms/step':>8s} {'launches/step':>14s}")
    for c, t in tot.most_common():
        print(f"{c:26s} {t:8.2f} {calls[c]:14.0f}")
    print(f"{'total':26s} {sum(tot.values()):8.2f} {sum(calls.values()):14.0f}")


if __name__ == "__main__":
    main()
