#!/usr/bin/env python3
"""HBM bytes per kernel of ONE eager step from the rocprofv3 FETCH_SIZE / WRITE_SIZE passes of tools/gpu/pmc_bytes.sh
(reads = FETCH_SIZE x --fetch_scale, default 2: the counter reports half of a wide coalesced read on gfx950).

The step is the span after the second-to-last fused-Adam dispatch up to the last one; per kernel name: launches, PMC-
serialised time, GB moved (FETCH_SIZE + WRITE_SIZE, KB units), achieved TB/s and the time at 5 TB/s.

  python tools/pmc_step_bytes.py gpurun_out/<tag>_f gpurun_out/<tag>_w [--top 40]
"""
import argparse
import collections
import csv
import glob
import os
import re


def load(d, counter):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] == counter:
                    rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"]),
                                 int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows.sort()
    return rows


def last_step(rows):
    adam = [i for i, r in enumerate(rows) if "flat_adam" in r[1]]
    if len(adam) < 2:
        raise SystemExit("need two fused-Adam dispatches in the trace")
    return rows[adam[-2] + 1: adam[-1] + 1]


def short(n):
    return re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", "").replace("void ", ""))[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--fetch_scale", type=float, default=2.0,
                    help="FETCH_SIZE multiplier: on gfx950 it counts half the bytes of 16-B-per-lane coalesced reads "
                         "(profiles/r6_pmc_calibration.md); 1.0 reproduces the raw counter")
    a = ap.parse_args()
    f = last_step(load(a.fetch_dir, "FETCH_SIZE"))
    w = last_step(load(a.write_dir, "WRITE_SIZE"))
    if len(f) != len(w) or any(x[1] != y[1] for x, y in zip(f, w)):
        raise SystemExit(f"the two passes' steps differ ({len(f)} vs {len(w)} dispatches)")
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for (_, n, fb, dt), (_, _, wb, _) in zip(f, w):
        e = agg[short(n)]
        e[0] += 1
        e[1] += dt / 1e6
        e[2] += (a.fetch_scale * fb + wb) * 1024 / 1e9
    tms = sum(v[1] for v in agg.values())
    tgb = sum(v[2] for v in agg.values())
    print(f"step kernels {len(f)}, sum dur {tms:.2f} ms, bytes {tgb:.2f} GB ({tgb / tms:.2f} TB/s averaged)")
    print(f"{'kernel':72s} {'n':>4s} {'ms':>7s} {'GB':>7s} {'TB/s':>6s} {'ms@5TB/s':>9s}")
    for k, (n, ms, gb) in sorted(agg.items(), key=lambda x: -x[1][1])[:a.top]:
        print(f"{k:72s} {n:4d} {ms:7.3f} {gb:7.3f} {gb / ms if ms else 0:6.2f} {gb / 5.0:9.3f}")


if __name__ == "__main__":
    main()
