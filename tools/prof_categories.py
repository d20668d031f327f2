#!/usr/bin/env python3
"""Per-step kernel time by category from a rocprofv3 --stats kernel_stats.csv (tools/gpu/prof.sh output).

usage: python tools/prof_categories.py gpurun_out/prof_<tag>/run_kernel_stats.csv [--steps 5]
"""
import argparse
import collections
import csv


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
        return "input H2D blits (copyBuffer)"
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    tot = collections.Counter()
    calls = collections.Counter()
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
