"""Probe: fp8 (OCP e4m3fn) GEMM support on this ROCm/torch build (torch._scaled_mm -> hipBLASLt)."""
import time

import torch

print(torch.__version__, torch.cuda.get_device_name(0), torch.cuda.get_device_capability(0))
M, K, N = 5760 * 16, 1536, 512
a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
for dt in (torch.float8_e4m3fn, torch.float8_e4m3fnuz):
    try:
        sa = (a.abs().amax().float() / torch.finfo(dt).max).clamp(min=1e-12)
        sb = (b.abs().amax().float() / torch.finfo(dt).max).clamp(min=1e-12)
        a8 = (a.float() / sa).to(dt)
        b8 = (b.float() / sb).to(dt)
        out = torch._scaled_mm(a8, b8.t(), scale_a=sa, scale_b=sb, out_dtype=torch.bfloat16)
        ref = a.float() @ b.float().t()
        err = float((out.float() - ref).norm() / ref.norm())
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            torch._scaled_mm(a8, b8.t(), scale_a=sa, scale_b=sb, out_dtype=torch.bfloat16)
        torch.cuda.synchronize()
        t8 = (time.perf_counter() - t0) / 20
        t0 = time.perf_counter()
        for _ in range(20):
            a @ b.t()
        torch.cuda.synchronize()
        t16 = (time.perf_counter() - t0) / 20
        print(f"{dt}: ok rel_err={err:.4f} fp8 {2*M*N*K/t8/1e12:.1f} TF/s  bf16 {2*M*N*K/t16/1e12:.1f} TF/s")
    except Exception as e:  # noqa: BLE001
        print(f"{dt}: FAILED {type(e).__name__}: {str(e)[:200]}")
