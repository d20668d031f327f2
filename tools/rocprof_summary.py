#!/usr/bin/env python3
"""Summarise rocprofv3 kernel stats / kernel trace CSVs into a markdown table.

usage: python tools/rocprof_summary.py <rocprof output dir> [--top 40] [--out profiles/x.md] [--title ...]
"""
import argparse
import csv
import glob
import os
import sys


def find(d, pattern):
    return sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--out", default=None)
    ap.add_argument("--title", default="rocprofv3 kernel summary")
    a = ap.parse_args()
    rows = []
    stats = find(a.dir, "*kernel_stats.csv")
    if stats:
        with open(stats[0]) as f:
            for r in csv.DictReader(f):
                rows.append((r.get("Name") or r.get("KernelName"), int(float(r["Calls"])), float(r["TotalDurationNs"]),
                             float(r.get("Percentage", 0))))
    else:
        traces = find(a.dir, "*kernel_trace.csv")
        if not traces:
            sys.exit(f"no kernel stats/trace csv under {a.dir}")
        agg = {}
        for tr in traces:
            with open(tr) as f:
                for r in csv.DictReader(f):
                    n = r.get("Kernel_Name") or r.get("KernelName")
                    d = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
                    c, t = agg.get(n, (0, 0.0))
                    agg[n] = (c + 1, t + d)
        tot = sum(t for _, t in agg.values())
        rows = [(n, c, t, 100.0 * t / tot) for n, (c, t) in agg.items()]
    rows.sort(key=lambda r: -r[2])
    total = sum(r[2] for r in rows)
    lines = [f"# {a.title}", "", f"source: `{a.dir}`  total kernel time: {total / 1e6:.2f} ms over "
             f"{sum(r[1] for r in rows)} dispatches", "",
             "| # | kernel | calls | total ms | % | avg us |", "|---|---|---|---|---|---|"]
    for i, (n, c, t, pct) in enumerate(rows[:a.top]):
        short = (n[:110] + "...") if len(n) > 113 else n
        lines.append(f"| {i + 1} | `{short}` | {c} | {t / 1e6:.3f} | {100.0 * t / total:.1f} | {t / max(c, 1) / 1e3:.1f} |")
    text = "\n".join(lines) + "\n"
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        open(a.out, "w").write(text)
    print(text)


if __name__ == "__main__":
    main()
