#!/usr/bin/env python3
"""pw_z_prep (Mk = We^T diag(k2) We, r0, Wt of the y-free wide expand backward) and pw_z_finish (dWe) at the step's
shapes, this build vs another build of the extension (--ab <.so>), interleaved launches, outputs compared.

  python tools/bench_zprep.py [--ab build/head/<so>]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ab", default="")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from pytorch_rt1_for_distributed_training_amd import ops
    from bench_dw_replay import _time, load_other
    ext = ops.load()
    other = load_other(a.ab) if a.ab else None
    tot = [0.0, 0.0]
    # (CE, CIN) of the wide expand blocks on the y-free path: 9-12, 13, 14-17, 19-23, 24 (per step)
    for (CE, CIN, n) in [(576, 96, 5), (816, 136, 5), (1392, 232, 6)]:
        We = (torch.randn(CE, CIN, device="cuda") * CIN ** -0.5).to(torch.bfloat16)
        consts = torch.randn(5 * CE, device="cuda")
        S = torch.randn(CE, CIN, device="cuda")
        G = torch.randn(CIN, CIN, device="cuda")
        sx = torch.randn(CIN, device="cuda")
        for name, args in (("pw_z_prep", (We, consts)), ("pw_z_finish", (S, G, sx, We, consts))):
            fns = [getattr(ext, name)] + ([getattr(other, name)] if other else [])
            us = _time(fns, args, {}, a.iters)
            line = f"{name:12s} CE {CE:5d} CIN {CIN:4d} (x{n}/step): {us[0]:7.1f} us"
            if other:
                oa, ob = fns[0](*args), fns[1](*args)
                if isinstance(oa, torch.Tensor):
                    oa, ob = [oa], [ob]
                d = [float((x.float() - y.float()).norm() / (y.float().norm() + 1e-12)) for x, y in zip(oa, ob)]
                line += f" | other {us[1]:7.1f} us; out rel diff " + " ".join(f"{v:.1e}" for v in d)
            for k, u in enumerate(us):
                tot[k] += n * u
            print(line, flush=True)
    print(f"per step: {tot[0] / 1e3:.3f} ms" + (f" vs other {tot[1] / 1e3:.3f} ms" if other else ""))


if __name__ == "__main__":
    main()
