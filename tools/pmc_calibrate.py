#!/usr/bin/env python3
"""Known-byte kernels for calibrating rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 (tools/gpu/pmc_calibrate.sh):
each op below moves a byte count fixed by its shapes, run 3 times; compare the counters' per-dispatch values with
the expected bytes printed here.

  python tools/pmc_calibrate.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from pytorch_rt1_for_distributed_training_amd import ops
    ext = ops.load()
    n = 1 << 29                                            # 1 GiB of bf16
    x = torch.randn(n, device="cuda").to(torch.bfloat16)
    y = torch.empty_like(x)
    M, C = n // 256, 256                                   # [M, 256] channels-last rows, the same 1 GiB
    sc, sh = torch.rand(C, device="cuda"), torch.rand(C, device="cuda")
    torch.cuda.synchronize()
    for _ in range(3):
        y.copy_(x)                                         # torch copy: reads 1 GiB, writes 1 GiB
    for _ in range(3):
        ext.bn_apply(x.view(M, C), sc, sh, 1, None, 0)     # bn_apply_flat (SiLU): reads 1 GiB, writes 1 GiB
    for _ in range(3):
        torch.sum(x.view(-1, 4096).float(), dim=1)         # (casts: read 1 GiB, write 2 GiB fp32; then a read 2 GiB)
    torch.cuda.synchronize()
    print(f"expected per dispatch: copy read {n * 2 / 1e9:.3f} GB write {n * 2 / 1e9:.3f} GB; "
          f"bn_apply read {n * 2 / 1e9:.3f} GB write {n * 2 / 1e9:.3f} GB")


if __name__ == "__main__":
    main()
