#!/usr/bin/env python3
"""Average rocprofv3 --pmc counter CSVs per kernel (dispatches of one kernel averaged), one row per kernel.

usage: python tools/pmc_summary.py <pmc dir> [<pmc dir> ...]
"""
import collections
import csv
import glob
import os
import re
import sys


def main():
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    name = r.get("Kernel_Name") or r.get("KernelName")
                    short = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", "").replace("void ", ""))
                    cn = r.get("Counter_Name")
                    agg[short][cn].append(float(r.get("Counter_Value", 0)))
    cols = sorted({c for k in agg.values() for c in k})
    print("kernel\t" + "\t".join(cols))
    for k, cs in sorted(agg.items()):
        vals = [sum(cs[c]) / len(cs[c]) if cs.get(c) else float("nan") for c in cols]
        print(k[:70].replace("\t", " ") + "\t" + "\t".join(f"{v:.4g}" for v in vals))
    # derived per-kernel view (per-wave instruction mix, stall fractions)
    print()
    for k, cs in sorted(agg.items()):
        f = {c: (sum(v) / len(v)) for c, v in cs.items()}
        w = f.get("SQ_WAVES", 0)
        if not w or "SQ_WAVE_CYCLES" not in f:
            continue
        busy = max(f.get("SQ_BUSY_CYCLES", 1), 1)
        print(f"{k[:60]:60s} waves={int(w):7d} busy={int(busy):9d} valu/w={f.get('SQ_INSTS_VALU', 0) / w:8.0f} "
              f"lds/w={f.get('SQ_INSTS_LDS', 0) / w:6.0f} vmrd/w={f.get('SQ_INSTS_VMEM_RD', 0) / w:6.1f} "
              f"salu/w={f.get('SQ_INSTS_SALU', 0) / w:6.0f} "
              f"wait_inst={f.get('SQ_WAIT_INST_ANY', 0) / f['SQ_WAVE_CYCLES']:.2f} "
              f"wait_any={f.get('SQ_WAIT_ANY', 0) / f['SQ_WAVE_CYCLES']:.2f} "
              f"valu_act/busy={f.get('SQ_ACTIVE_INST_VALU', 0) / busy:.2f} "
              f"ldsconf/ldsact={f.get('SQ_LDS_BANK_CONFLICT', 0) / max(f.get('SQ_ACTIVE_INST_LDS', 1), 1):.2f}")


if __name__ == "__main__":
    main()
