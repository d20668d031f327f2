"""Debug: replay se_bwd on inputs dumped by RT1_SE_DEBUG + RT1_SE_DUMP (ops/backbone.py _se_debug_check) in one
process, 200 times, and report how many distinct dw1 results appear and whether they equal the dumped first / rerun
outputs."""
import glob
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_rt1_for_distributed_training_amd import ops  # noqa: E402

ext = ops.load()
for path in sorted(glob.glob(os.path.join(sys.argv[1], "*.pt")))[:6]:
    d = torch.load(path, weights_only=True)
    args = [a.cuda() if torch.is_tensor(a) else a for a in d["args"]]
    first, rerun = d["first"].cuda(), d["rerun"].cuda()
    distinct, eq_first, eq_rerun = [], 0, 0
    for _ in range(200):
        r = ext.se_bwd(*args)[2]
        eq_first += int(torch.equal(r, first))
        eq_rerun += int(torch.equal(r, rerun))
        if not any(torch.equal(r, x) for x in distinct):
            distinct.append(r)
    print(f"{os.path.basename(path)}: shapes red {tuple(args[0].shape)} h {tuple(args[2].shape)}; 200 replays: "
          f"{len(distinct)} distinct, {eq_first} == first, {eq_rerun} == rerun", flush=True)
