#!/usr/bin/env python3
"""SQ counters per kernel of ONE eager step from the rocprofv3 --pmc passes of tools/gpu/pmc_sq_step.sh.

The step is the span after the second-to-last fused-Adam dispatch up to the last one (as tools/pmc_step_bytes.py).
Per kernel name (dispatches of one name summed): launches, PMC-serialised time, waves, VALU / LDS / VMEM instructions
per wave, wait fractions (SQ_WAIT_ANY / SQ_WAVE_CYCLES: a wave waiting on anything; SQ_WAIT_INST_ANY: waiting for an
instruction's dependency), VALU-active share of the busy cycles, LDS bank-conflict cycles per LDS-active cycle and
the achieved waves per SIMD (SQ_WAVE_CYCLES / (busy cycles x SIMDs), SQ counts quad-cycles per wave).

  python tools/pmc_step_sq.py gpurun_out/<tag>_a gpurun_out/<tag>_b [--match dw_] [--top 60]
"""
import argparse
import collections
import csv
import glob
import os
import re


def load(d):
    """{dispatch_id: (kernel, dur_ns, {counter: value})} of one pass directory."""
    rows = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                i = int(r["Dispatch_Id"])
                e = rows.setdefault(i, [r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), {}])
                e[2][r["Counter_Name"]] = e[2].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return rows


def last_step(rows):
    ids = sorted(rows)
    adam = [k for k, i in enumerate(ids) if "flat_adam" in rows[i][0]]
    if len(adam) < 2:
        raise SystemExit("need two fused-Adam dispatches in the trace")
    return [rows[i] for i in ids[adam[-2] + 1: adam[-1] + 1]]


def short(n):
    return re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", "").replace("void ", ""))[:64]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default="")
    ap.add_argument("--top", type=int, default=60)
    a = ap.parse_args()
    steps = [last_step(load(d)) for d in a.dirs]
    n0 = len(steps[0])
    for s in steps[1:]:
        if len(s) != n0 or any(x[0] != y[0] for x, y in zip(steps[0], s)):
            raise SystemExit("the passes' steps differ")
    agg = collections.defaultdict(lambda: [0, 0.0, collections.Counter()])
    for k in range(n0):
        name = short(steps[0][k][0])
        e = agg[name]
        e[0] += 1
        e[1] += steps[0][k][1] / 1e6
        for s in steps:
            e[2].update(s[k][2])
    tot = sum(v[1] for v in agg.values())
    print(f"step kernels {n0}, PMC-serialised sum {tot:.2f} ms")
    hdr = (f"{'kernel':64s} {'n':>3s} {'ms':>6s} {'waves':>7s} {'valu/w':>7s} {'lds/w':>6s} {'vmrd/w':>6s} "
           f"{'vmwr/w':>6s} {'salu/w':>6s} {'wait':>5s} {'wdep':>5s} {'valu%':>5s} {'ldsCf':>5s} {'w/SIMD':>6s}")
    print(hdr)
    for name, (n, ms, c) in sorted(agg.items(), key=lambda x: -x[1][1])[:a.top]:
        if a.match and a.match not in name:
            continue
        w = c.get("SQ_WAVES", 0.0) or 1.0
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        busy = c.get("SQ_BUSY_CYCLES", 0.0) or 1.0
        print(f"{name:64s} {n:3d} {ms:6.3f} {int(w):7d} {c.get('SQ_INSTS_VALU', 0) / w:7.0f} "
              f"{c.get('SQ_INSTS_LDS', 0) / w:6.0f} {c.get('SQ_INSTS_VMEM_RD', 0) / w:6.1f} "
              f"{c.get('SQ_INSTS_VMEM_WR', 0) / w:6.1f} {c.get('SQ_INSTS_SALU', 0) / w:6.0f} "
              f"{c.get('SQ_WAIT_ANY', 0) / wc:5.2f} {c.get('SQ_WAIT_INST_ANY', 0) / wc:5.2f} "
              f"{c.get('SQ_ACTIVE_INST_VALU', 0) / busy:5.2f} "
              f"{c.get('SQ_LDS_BANK_CONFLICT', 0) / max(c.get('SQ_ACTIVE_INST_LDS', 0), 1):5.2f} "
              f"{wc / busy:6.2f}")


if __name__ == "__main__":
    main()
