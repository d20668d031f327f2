"""Forward / dgrad 1x1-conv GEMM formulations on hipBLASLt for the tall-skinny encoder shapes."""
import torch

BF = torch.bfloat16


def t(fn, it=10):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(it)]
    for a, b in ev:
        a.record(); fn(); b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
    return ts[len(ts) // 2]


for M, K, N in [(277248, 576, 96), (277248, 816, 136), (76800, 1392, 232), (76800, 2304, 384), (277248, 288, 96),
                (76800, 816, 232), (277248, 96, 576), (277248, 136, 816), (76800, 232, 1392), (76800, 384, 2304)]:
    a = torch.randn(M, K, device="cuda").to(BF)
    w = torch.randn(N, K, device="cuda").to(BF)
    wt = w.t().contiguous()
    roof = M * (K + N) * 2 / 5.5e12 * 1e6
    res = {"mm_NT": t(lambda: torch.mm(a, w.t())), "mm_NN": t(lambda: torch.mm(a, wt))}
    for S in (2, 4, 8, 16):
        if M % S == 0:
            res[f"bmm{S}"] = t(lambda S=S: torch.bmm(a.view(S, M // S, K), w.t().unsqueeze(0).expand(S, K, N)))
    best = min(res, key=res.get)
    print(f"M={M:7d} K={K:5d} N={N:5d} roof {roof:6.1f}us " + " ".join(f"{k}:{v:6.1f}" for k, v in res.items()) +
          f"  best {best}", flush=True)
