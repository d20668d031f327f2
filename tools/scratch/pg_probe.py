"""Does a torch ProcessGroupNCCL (RCCL) world=1 run exit cleanly on this box?"""
import os
import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29511")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
t = torch.ones(8, device="cuda")
dist.all_reduce(t)
torch.cuda.synchronize()
print("all_reduce ok", t.sum().item(), flush=True)
dist.destroy_process_group()
print("destroyed pg", flush=True)
