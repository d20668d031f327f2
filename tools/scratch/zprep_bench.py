"""pw_z_prep (Mk / r0 kernel + Wt transpose kernel) at the wide-block shapes, under rocprofv3 --stats."""
import torch, sys, os
sys.path.insert(0, os.getcwd())
from pytorch_rt1_for_distributed_training_amd.ops import load
ext = load()
for CE, CIN in ((576, 96), (816, 136)):
    We = torch.randn(CE, CIN, device="cuda").to(torch.bfloat16)
    consts = torch.rand(5, CE, device="cuda")
    for _ in range(20):
        ext.pw_z_prep(We, consts)
    torch.cuda.synchronize()
print("ok")
