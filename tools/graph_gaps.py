#!/usr/bin/env python3
"""Idle time between kernels in a rocprofv3 kernel trace: per replayed step, the span from first kernel start to last
kernel end vs the sum of kernel durations (gaps = launch/dependency bubbles), plus the kernels with the largest
count per step.

usage: python tools/graph_gaps.py <kernel_trace.csv> [--steps K]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=3, help="trailing steps to analyse (split at the largest gaps)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    # split steps at the (steps-1) largest idle gaps among the trailing part of the trace
    gaps = [(ks[i + 1][0] - ks[i][1], i) for i in range(len(ks) - 1)]
    cut = sorted(i for _, i in sorted(gaps, reverse=True)[: a.steps])
    segs = []
    prev = cut[0] + 1
    for c in cut[1:] + [len(ks) - 1]:
        segs.append(ks[prev: c + 1])
        prev = c + 1
    for s in segs[-a.steps:]:
        span = (s[-1][1] - s[0][0]) / 1e6
        busy = sum(e - b for b, e, _ in s) / 1e6
        # union of intervals (concurrent kernels)
        u, cur_b, cur_e = 0, None, None
        for b, e, _ in s:
            if cur_e is None or b > cur_e:
                if cur_e is not None:
                    u += cur_e - cur_b
                cur_b, cur_e = b, e
            else:
                cur_e = max(cur_e, e)
        u += cur_e - cur_b
        print(f"step: {len(s)} kernels, span {span:.2f} ms, kernel-busy (union) {u / 1e6:.2f} ms, "
              f"sum of durations {busy:.2f} ms, idle {span - u / 1e6:.2f} ms")
    s = segs[-1]
    cnt = collections.Counter(n.split("(")[0].replace("void ", "")[:70] for _, _, n in s)
    small = collections.Counter()
    for b, e, n in s:
        if e - b < 10000:
            small[n.split("(")[0].replace("void ", "")[:70]] += 1
    print("kernels < 10 us in the last step:", sum(small.values()))
    for n, c in small.most_common(25):
        print(f"  {c:5d}  {n}")


if __name__ == "__main__":
    main()
