"""Is torch's fp32 GEMM exact fp32 on this ROCm build?  Relative error vs fp64 for the SE shapes."""
import torch
torch.manual_seed(0)
for (M, K, N) in [(768, 40, 10), (768, 2304, 96), (768, 96, 2304), (40, 768, 10)]:
    a = torch.randn(M, K, device="cuda", dtype=torch.float64)
    b = torch.randn(K, N, device="cuda", dtype=torch.float64)
    ref = a @ b
    for name, f in (("mm", lambda: a.float() @ b.float()), ("addmm", lambda: torch.addmm(torch.zeros(N, device="cuda"), a.float(), b.float(), alpha=0.5) * 2),
                    ("mm_t", lambda: (b.float().t().contiguous() @ a.float().t().contiguous()).t())):
        out = f().double()
        err = ((out - ref).norm() / ref.norm()).item()
        print(f"{name:6s} M{M} K{K} N{N}: rel err {err:.2e}  (fp32 eps 6e-8, bf16 4e-3, tf32 5e-4)")
print("allow_tf32", torch.backends.cuda.matmul.allow_tf32, torch.get_float32_matmul_precision())
