"""Stem kernels at the bench shape (768 uint8 frames of 300x300): forward and weight gradient, HIP events."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pytorch_rt1_for_distributed_training_amd.ops import load  # noqa: E402

ext = load()
N, H, W = 768, 300, 300
img = torch.randint(0, 256, (N, 3, H, W), device="cuda", dtype=torch.uint8)
shift = torch.tensor([3, -5], dtype=torch.int32, device="cuda")
w = torch.randn(40, 27, device="cuda") * 0.3
dy = torch.randn(N, 150, 150, 40, device="cuda").to(torch.bfloat16)


def t(fn, it=10):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3


for mb in (1024, 2048, 4096):
    print(f"max_blocks {mb}: stem_fwd {t(lambda: ext.stem_fwd(img, shift, w, mb)):8.1f} us   "
          f"stem_bwd_weight {t(lambda: ext.stem_bwd_weight(img, shift, dy, mb)):8.1f} us", flush=True)
