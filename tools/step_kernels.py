#!/usr/bin/env python3
"""Ordered kernel list of ONE step from a rocprofv3 kernel + memory-copy trace (tools/gpu/trace_now.sh output).

Steps are delimited like tools/prof_categories.py --trace does: each step starts at its > 1 ms input H2D copy.  Prints
index, start offset (us from the step start), duration (us), grid / workgroup size and the kernel name, so a kernel can
be mapped to its call site by position (forward blocks 0..25, top, transformer, head, backward in reverse).

usage: python tools/step_kernels.py gpurun_out/trN [--step -2] [--match dw_] [--width 90]
"""
import argparse
import csv
import glob
import gzip
import os


def _rows(path):
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rt") as f:
        yield from csv.DictReader(f)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--step", type=int, default=-2, help="step index (python-style; -2 = the one before the last)")
    ap.add_argument("--match", default="", help="only kernels whose name contains this")
    ap.add_argument("--width", type=int, default=90)
    a = ap.parse_args()
    kt = glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv*"), recursive=True)
    mc = glob.glob(os.path.join(a.trace_dir, "**", "*memory_copy_trace.csv*"), recursive=True)
    if not kt or not mc:
        raise SystemExit("need a kernel trace and a memory-copy trace under " + a.trace_dir)
    starts = sorted(int(r["Start_Timestamp"]) for r in _rows(mc[0])
                    if int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) > 1_000_000)
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                  r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["Workgroup_Size_X"]) for r in _rows(kt[0])))
    bounds = starts + [float("inf")]
    s = a.step if a.step >= 0 else len(starts) + a.step
    t0, t1 = bounds[s], bounds[s + 1]
    tot = 0.0
    n = 0
    for i, (b, e, name, gx, gy, gz, wg) in enumerate(k for k in ks if t0 <= k[0] < t1):
        if a.match and a.match not in name:
            continue
        d = (e - b) / 1e3
        tot += d
        n += 1
        print(f"{i:5d} {(b - t0) / 1e3:10.1f} {d:9.1f}  {gx:>8}x{gy:<4}x{gz:<3} wg{wg:<5} {name[:a.width]}")
    print(f"# {n} kernels, {tot / 1e3:.3f} ms (step {s} of {len(starts)})")


if __name__ == "__main__":
    main()
