#!/usr/bin/env python3
"""Per-kernel ms/step difference between two rocprofv3 --stats runs (tools/gpu/prof_ab.sh output).

usage: python tools/prof_diff.py gpurun_out/prof_X0 gpurun_out/prof_X1 [--steps 5] [--top 20]
"""
import argparse
import csv


def load(d, steps):
    out = {}
    for r in csv.DictReader(open(f"{d}/run_kernel_stats.csv")):
        k = r["Name"][:100]
        c, t = out.get(k, (0, 0.0))
        out[k] = (c + int(r["Calls"]), t + float(r["TotalDurationNs"]) / 1e6 / steps)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--top", type=int, default=20)
    o = ap.parse_args()
    a, b = load(o.a, o.steps), load(o.b, o.steps)
    print(f"total ms/step: {sum(v[1] for v in a.values()):.3f} -> {sum(v[1] for v in b.values()):.3f}")
    keys = sorted(set(a) | set(b), key=lambda k: -abs(b.get(k, (0, 0))[1] - a.get(k, (0, 0))[1]))
    print(f"{'a ms':>8s} {'b ms':>8s} {'a n':>5s} {'b n':>5s}  kernel")
    for k in keys[:o.top]:
        (na, ta), (nb, tb) = a.get(k, (0, 0.0)), b.get(k, (0, 0.0))
        print(f"{ta:8.3f} {tb:8.3f} {na:5d} {nb:5d}  {k}")


if __name__ == "__main__":
    main()
