"""Debug: repeat the fused SE forward/backward 200x under GPU contention (a second stream of big GEMMs and the other
process of a pair) and report any run that differs bitwise from the first."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pytorch_rt1_for_distributed_training_amd import ops  # noqa: E402

ext = ops.load()
torch.manual_seed(0)
N, C, S, HW = int(os.environ.get("SE_N", "24")), int(os.environ.get("SE_C", "576")), int(os.environ.get("SE_S", "24")), 64
pool = torch.randn(N, C, device="cuda") * 10
f1w, f1b = torch.randn(S, C, device="cuda") * 0.05, torch.randn(S, device="cuda") * 0.1
f2w, f2b = torch.randn(C, S, device="cuda") * 0.05, torch.randn(C, device="cuda") * 0.1
red = torch.randn(5, N, C, device="cuda")
side = torch.cuda.Stream()
a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)


def run():
    pl, h, gate = ext.se_fwd(pool.clone(), 1.0 / HW, f1w, f1b, f2w, f2b)
    return [h, gate] + list(ext.se_bwd(red.clone(), gate, h, pl, 1.0 / HW, f1w, f2w, float(N * HW)))


names = ["h", "gate", "df2w", "df2b", "df1w", "df1b", "rb", "db2", "dg2", "mdz2", "mdzx2"]
ref = run()
torch.cuda.synchronize()
bad = 0
for it in range(200):
    with torch.cuda.stream(side):
        for _ in range(3):
            a = (a @ a).clamp_(-1, 1)
    out = run()
    torch.cuda.synchronize()
    for n, x, y in zip(names, ref, out):
        if not torch.equal(x, y):
            bad += 1
            print(f"iter {it}: {n} differs, maxdiff {float((x - y).abs().max()):.3e}", flush=True)
print(f"done: {bad} mismatches (N={N} C={C} S={S})")
