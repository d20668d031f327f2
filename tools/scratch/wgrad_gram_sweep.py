"""G = x^T x (the wide dz-mode expand backward) on the wgrad kernel variants vs split-K bmm, at 768 x 19 x 19 rows."""
import torch, sys, os
sys.path.insert(0, os.getcwd())
from pytorch_rt1_for_distributed_training_amd.ops import load, backbone
ext = load()
def timeit(fn, iters=10):
    for _ in range(3): fn()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record(); b.synchronize(); ts.append(a.elapsed_time(b) * 1e3)
    return sorted(ts)[len(ts) // 2]
M = 768 * 361
for C in (96, 136):
    x = torch.randn(M, C, device="cuda").to(torch.bfloat16)
    row = [f"C={C}"]
    for v in range(6):
        row.append(f"v{v}:{timeit(lambda: ext.wgrad(x, x, variant=v)):7.1f}")
    row.append(f"auto:{timeit(lambda: ext.wgrad(x, x, variant=-1)):7.1f}")
    row.append(f"bmm:{timeit(lambda: backbone.wgrad_bmm(x, x)):7.1f}")
    row.append(f"colsum:{timeit(lambda: ext.colsum(x)):6.1f}")
    print(" ".join(row), flush=True)
