"""Grid-cap sweep of the y-free expand backward (pwbwd.hip pw_bwd_z) at 768 frames, 300x300."""
import torch, sys, os
sys.path.insert(0, os.getcwd())
from pytorch_rt1_for_distributed_training_amd.ops import load
ext = load()
BF = torch.bfloat16
def timeit(fn, iters=10):
    for _ in range(3): fn()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record(); b.synchronize(); ts.append(a.elapsed_time(b) * 1e3)
    return sorted(ts)[len(ts) // 2]
shapes = [("blk2", 768*150*150, 144, 24, 22500, False), ("blk3", 768*75*75, 192, 32, 5625, True),
          ("blk5", 768*75*75, 192, 32, 5625, False), ("blk6", 768*38*38, 288, 48, 1444, True),
          ("blk8", 768*38*38, 288, 48, 1444, False)]
for name, M, CE, CIN, HW, res in shapes:
    dz = torch.randn(M, CE, device="cuda").to(BF)
    x = torch.randn(M, CIN, device="cuda").to(BF); We = torch.randn(CE, CIN, device="cuda").to(BF)
    consts = torch.rand(5, CE, device="cuda")
    dout = torch.randn(M, CIN, device="cuda").to(BF) if res else None
    fm = torch.rand(M // HW, CIN, device="cuda") if res else None
    row = []
    for mb in (256, 512, 1024, 2048, 3072, 4096, 6144, 8192):
        t = timeit(lambda: ext.pw_bwd_z(dz, x, We, consts, dout, fm, HW, mb))
        row.append(f"{mb}:{t:7.1f}")
    gb = M * (CE + 2 * CIN + (CIN if res else 0)) * 2 / 1e9
    print(name, f"{gb:.2f} GB", " ".join(row), flush=True)
    del dz, x
    torch.cuda.empty_cache()
