"""pwtall.hip vs hipBLASLt on the tall-skinny encoder shapes (forward project convs and expand/top dgrads)."""
import torch

from pytorch_rt1_for_distributed_training_amd import ops

BF = torch.bfloat16
ext = ops.load()


def t(fn, it=20):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(it)]
    for a, b in ev:
        a.record(); fn(); b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
    return ts[len(ts) // 2]


tot_mm = tot_tall = 0.0
for M, K, N in [(277248, 576, 96), (277248, 816, 136), (76800, 816, 136), (76800, 1392, 232), (19200, 1392, 232),
                (19200, 2304, 384), (76800, 2304, 384), (19200, 1536, 384), (277248, 288, 96), (76800, 576, 96)]:
    a = torch.randn(M, K, device="cuda").to(BF)
    w = torch.randn(N, K, device="cuda").to(BF)
    roof = M * (K + N) * 2 / 5.5e12 * 1e6
    mm = t(lambda: torch.mm(a, w.t()))
    tall = t(lambda: ext.pw_tall(a, w)[0])
    err = ((ext.pw_tall(a, w)[0].float() - a.float() @ w.float().t()).norm() / (a.float() @ w.float().t()).norm()).item()
    tot_mm += mm
    tot_tall += tall
    print(f"M={M:7d} K={K:5d} N={N:4d} roof(5.5TB/s) {roof:6.1f}us  hipblaslt {mm:6.1f}us  pw_tall {tall:6.1f}us "
          f"({mm / tall:4.2f}x, {roof / tall * 100:5.1f}% roof) err {err:.1e}", flush=True)
    del a, w
print(f"total hipblaslt {tot_mm:.0f}us pw_tall {tot_tall:.0f}us", flush=True)
