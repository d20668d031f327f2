#!/usr/bin/env python3
"""Kernel busy time vs wall time of hipGraph-replayed steps from a rocprofv3 --kernel-trace CSV.

  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gt -o run -- python3 bench.py --steps 5 --warmup 3
  python tools/graph_timeline.py gpurun_out/gt --last 5

Steps are split at the gaps between consecutive bench steps (the largest idle gaps); for each step: wall time from the
first kernel start to the last kernel end, the summed kernel durations, the idle time between kernels and the number
of gaps above 1 / 5 us.
"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("d")
    ap.add_argument("--last", type=int, default=5)
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.d, "**", "*kernel_trace.csv"), recursive=True)[0]
    ks = []
    for r in csv.DictReader(open(f)):
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ks.sort()
    # step boundaries: the (steps) largest gaps
    gaps = [(ks[i + 1][0] - ks[i][1], i) for i in range(len(ks) - 1)]
    big = sorted(sorted(gaps, reverse=True)[:a.last + 3], key=lambda g: g[1])
    cuts = [g[1] + 1 for g in big]
    segs, prev = [], 0
    for c in cuts + [len(ks)]:
        segs.append(ks[prev:c])
        prev = c
    segs = [s for s in segs if len(s) > 500][-a.last:]
    for s in segs:
        wall = (s[-1][1] - s[0][0]) / 1e6
        busy = 0
        end = s[0][0]
        idle, n1, n5 = 0, 0, 0
        for st, en, _ in s:
            if st > end:
                g = st - end
                idle += g
                n1 += g > 1000
                n5 += g > 5000
            busy += en - max(st, end) if en > end else 0
            end = max(end, en)
        print(f"kernels {len(s):5d}  wall {wall:7.2f} ms  busy {busy / 1e6:7.2f} ms  idle {idle / 1e6:6.2f} ms  "
              f"gaps>1us {n1}  gaps>5us {n5}")


if __name__ == "__main__":
    main()
