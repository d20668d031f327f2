#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--memory-copy-trace`` csv directory: copies by direction and size bucket, plus the
__amd_rocclr_copyBuffer kernel dispatch count from the kernel trace of the same run (tools/gpu/memcpy_trace.sh)."""
import collections
import csv
import glob
import os
import sys


def main(d):
    mc = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    by = collections.Counter()
    byb = collections.Counter()
    for f in mc:
        for r in csv.DictReader(open(f)):
            kind = r.get("Direction") or r.get("Operation") or r.get("Kind") or "?"
            size = int(r.get("Bytes") or r.get("Size") or 0)
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            bucket = 1 << max(0, size - 1).bit_length() if size else 0
            by[(kind, bucket)] += 1
            byb[kind] += dur
    print("memory copies (direction, size bucket <= bytes): count")
    for (k, b), c in sorted(by.items()):
        print(f"  {k:24s} {b:>12d}  {c}")
    print("total us by direction:", {k: round(v, 1) for k, v in byb.items()})
    # the per-step input copy (the 207 MB uint8 frame batch, > 1 ms) marks the start of each step
    marks = sorted(int(r["Start_Timestamp"]) for f in mc for r in csv.DictReader(open(f))
                   if int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) > 1_000_000)
    n = n_steps = 0
    names = collections.Counter()
    for f in kt:
        for r in csv.DictReader(open(f)):
            t = int(r["Start_Timestamp"])
            if "copyBuffer" in r.get("Kernel_Name", ""):
                n += 1
                if marks and t >= marks[0]:
                    n_steps += 1
            if marks and t >= marks[0]:
                names["all kernels in steps"] += 1
    print("copyBuffer kernel dispatches: %d in the whole run, %d after the first step's input copy "
          "(%d step input copies; %s)" % (n, n_steps, len(marks), dict(names)))


if __name__ == "__main__":
    main(sys.argv[1])
