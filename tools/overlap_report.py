#!/usr/bin/env python3
"""Comm/compute overlap in a rocprofv3 trace of one rank (``--kernel-trace --memory-copy-trace``, csv output).

For each of the last ``--steps`` training steps (delimited by the fused Adam kernel ``flat_adam``) it lists the
gradient-bucket transfers -- device->host copies of the gloo rehearsal, or RCCL kernels (``ncclKernel`` /
``ncclDevKernel``) on a real multi-GPU run -- and how much of each one ran while a compute kernel of the same
step was executing on the device.  Used for ``profiles/r2_dp_overlap*.md``.

  python tools/overlap_report.py gpurun_out/dp3_trace_r0 --steps 2
"""
from __future__ import annotations

import argparse
import csv
import glob
import os


def _rows(path):
    with open(path, newline="") as f:
        yield from csv.DictReader(f)


def load(d):
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    mt = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)
    kernels = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Stream_Id", ""))
               for p in kt for r in _rows(p)]
    copies = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"], r.get("Stream_Id", ""))
              for p in mt for r in _rows(p)]
    kernels.sort()
    copies.sort()
    return kernels, copies


def merge(intervals):
    out = []
    for s, e in sorted(intervals):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def overlap(a0, a1, merged):
    tot = 0
    for s, e in merged:
        if e <= a0:
            continue
        if s >= a1:
            break
        tot += min(a1, e) - max(a0, s)
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    kernels, copies = load(a.trace_dir)
    adam = [k for k in kernels if "flat_adam" in k[2]]
    if len(adam) < a.steps + 1:
        raise SystemExit(f"need >= {a.steps + 1} Adam kernels, found {len(adam)}")
    lines = [f"# comm / compute overlap: `{a.trace_dir}`", ""]
    for si in range(len(adam) - a.steps, len(adam)):
        t0, t1 = adam[si - 1][1], adam[si][0]
        win = [k for k in kernels if t0 <= k[0] < t1]
        main_stream = max(set(k[3] for k in win), key=lambda sid: sum(1 for k in win if k[3] == sid))
        # transfers: RCCL kernels, or the blit kernels gloo's pinned copies run on its own streams
        comm_k = [k for k in win if "nccl" in k[2].lower() or ("copyBuffer" in k[2] and k[3] != main_stream)]
        compute = [(k[0], k[1]) for k in win if k[3] == main_stream and "nccl" not in k[2].lower()]
        merged = merge(compute)
        xfer = [(c[0], c[1], c[2]) for c in copies if t0 <= c[0] < t1 and "DEVICE_TO_HOST" in c[2]]
        xfer += [(k[0], k[1], ("RCCL " if "nccl" in k[2].lower() else f"copy (stream {k[3]}) ") + k[2][:32])
                 for k in comm_k]
        xfer.sort()
        busy = sum(e - s for s, e in merged)
        lines.append(f"## step window {si}: {(t1 - t0) / 1e6:.2f} ms, compute busy {busy / 1e6:.2f} ms, "
                     f"{len(xfer)} gradient transfers")
        lines.append("")
        lines.append("| # | transfer | start (ms into step) | duration (us) | overlapped with compute (us) |")
        lines.append("|---|---|---|---|---|")
        ov_tot = dur_tot = 0
        for i, (s, e, kind) in enumerate(xfer):
            ov = overlap(s, e, merged)
            ov_tot += ov
            dur_tot += e - s
            lines.append(f"| {i} | {kind} | {(s - t0) / 1e6:.2f} | {(e - s) / 1e3:.1f} | {ov / 1e3:.1f} |")
        last_compute_end = merged[-1][1] if merged else t0
        before_end = sum(1 for s, e, _ in xfer if s < last_compute_end)
        lines.append("")
        lines.append(f"{before_end}/{len(xfer)} transfers start before the step's last compute kernel ends; "
                     f"{ov_tot / 1e3:.1f} of {dur_tot / 1e3:.1f} us of transfer time overlaps compute.")
        lines.append("")
    text = "\n".join(lines)
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
