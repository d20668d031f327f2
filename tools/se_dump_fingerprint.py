#!/usr/bin/env python3
"""Fingerprint the fused-SE dw1 mismatches dumped by RT1_SE_DEBUG=1 RT1_SE_DUMP=<dir> (ops/backbone.py
_se_debug_check): for each dump, the differing (row j, column c) positions, which of the two outputs is wrong against
an fp64 recomputation, and whether wrong - right equals minus ONE frame's term dh[n, j] * pool[n, c] / HW.  CPU only.

  python tools/se_dump_fingerprint.py gpurun_out/sedump
"""
import glob
import os
import sys

import torch


def main():
    for path in sorted(glob.glob(os.path.join(sys.argv[1], "*.pt"))):
        d = torch.load(path, weights_only=True)
        a, b = d["first"], d["rerun"]
        red, gate, h, pool, inv_hw = d["args"][:5]
        f2 = d["args"][6]
        dz = red[0].double() * gate.double() * (1 - gate.double())
        x = h.double()
        sg = torch.sigmoid(x)
        dh = (dz @ f2.double()) * (sg * (1 + x * (1 - sg)))
        ref = (dh.t() @ pool.double()) * inv_hw
        wrong, right, which = (a, b, "first") if (a.double() - ref).abs().max() > (b.double() - ref).abs().max() \
            else (b, a, "rerun")
        bad = (a != b).nonzero().tolist()
        print(f"{os.path.basename(path)}: dw1 {tuple(a.shape)}, {len(bad)} positions differ, wrong output = {which}")
        for j in sorted({p[0] for p in bad}):
            cols = [c for r, c in bad if r == j]
            frames = set()
            for c in cols:
                delta = (wrong[j, c].double() - right[j, c].double()) / inv_hw
                terms = dh[:, j] * pool[:, c].double()
                n = int((terms + delta).abs().argmin())
                rel = float((terms[n] + delta).abs() / terms[n].abs().clamp_min(1e-30))
                frames.add((n, rel < 1e-4))
            mods = sorted({c % 4 for c in cols})
            print(f"  row j={j} (j % 2 = {j % 2}): {len(cols)} columns, c % 4 in {mods}, channel tiles "
                  f"{sorted({c // 64 for c in cols})}; wrong = right - term(n) for (n, exact): {sorted(frames)}")


if __name__ == "__main__":
    main()
