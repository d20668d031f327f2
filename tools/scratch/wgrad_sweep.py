"""Sweep the split-K factor of the encoder's weight-gradient GEMMs (ops/backbone.py wgrad) per layer shape."""
import sys, os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pytorch_rt1_for_distributed_training_amd.ops import backbone as bb

BF = torch.bfloat16


def wgrad_s(dy, x, S):
    M = dy.shape[0]
    if S == 1:
        return torch.mm(dy.t(), x, out_dtype=torch.float32)
    rows = M // S
    M1 = rows * S
    part = torch.bmm(dy[:M1].view(S, rows, dy.shape[1]).transpose(1, 2), x[:M1].view(S, rows, x.shape[1]),
                     out_dtype=torch.float32)
    out = part.sum(0)
    if M1 < M:
        out += torch.mm(dy[M1:].t(), x[M1:], out_dtype=torch.float32)
    return out


def t(fn, it=8):
    for _ in range(2):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(it)]
    for a, b in ev:
        a.record(); fn(); b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
    return ts[len(ts) // 2]


shapes = [(17280000, 24, 40), (17280000, 24, 24), (4320000, 32, 144), (4320000, 32, 192), (1108992, 48, 192),
          (277248, 576, 96), (277248, 96, 576), (277248, 816, 136), (277248, 136, 816), (76800, 1392, 232),
          (76800, 232, 1392), (76800, 2304, 384), (76800, 384, 2304), (1108992, 288, 48), (1108992, 48, 288),
          (277248, 96, 288)]
for M, Co, Ci in shapes:
    dy = torch.randn(M, Co, device="cuda").to(BF)
    x = torch.randn(M, Ci, device="cuda").to(BF)
    roof = M * (Co + Ci) * 2 / 5.5e12 * 1e6
    cur = t(lambda: bb.wgrad(dy, x))
    if len(sys.argv) > 1 and M < 4000000:
        continue
    res = {S: t(lambda S=S: wgrad_s(dy, x, S)) for S in (8, 16, 32, 64, 128, 256, 512, 1024, 2048)
           if M // S >= 256}
    best = min(res, key=res.get)
    print(f"M={M:8d} Co={Co:5d} Ci={Ci:5d} roof {roof:6.1f}us  current {cur:7.1f}  " +
          " ".join(f"S{S}:{v:6.1f}" for S, v in res.items()) + f"  best S={best}", flush=True)
