#!/usr/bin/env python3
"""One step's kernel sequence from a rocprofv3 kernel trace (csv or csv.gz): start offset, duration, grid, VGPRs and
the short kernel name, in launch order.  Steps are delimited by the fused Adam launch.

    python tools/step_sequence.py gpurun_out/trN/run_kernel_trace.csv.gz [--step -2] > /tmp/step_seq.txt
"""
import argparse
import csv
import gzip
import re


def short(name: str) -> str:
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    depth, out = 0, []
    for ch in name:                      # drop the argument list, keep template arguments
        if ch == "(" and depth == 0 and out and out[-1] not in " <,":
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return re.sub(r"\s+", " ", "".join(out))[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step", type=int, default=-2, help="which step (python index over Adam-delimited steps)")
    a = ap.parse_args()
    op = gzip.open if a.trace.endswith(".gz") else open
    rows = sorted(csv.DictReader(op(a.trace, "rt")), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "flat_adam" in r["Kernel_Name"]]
    bounds = list(zip([-1] + ends[:-1], ends))
    lo, hi = bounds[a.step]
    step = rows[lo + 1:hi + 1]
    t0 = int(step[0]["Start_Timestamp"])
    tot = 0.0
    for r in step:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += d
        print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} {d:8.1f} {r['Grid_Size_X']:>8}x{r['Grid_Size_Y']:>4} "
              f"{r['VGPR_Count']:>4} {short(r['Kernel_Name'])}")
    print(f"# {len(step)} kernels, {tot / 1e3:.2f} ms of kernels, span {(int(step[-1]['End_Timestamp']) - t0) / 1e3:.2f} ms")


if __name__ == "__main__":
    main()
