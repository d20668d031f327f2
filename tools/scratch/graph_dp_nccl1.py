"""hipGraph DP step next to a live RCCL communicator, on one GPU: a 1-rank nccl process group (its watchdog
thread running), DataParallel forced on so the engine takes the graph-DP path (captured forward+backward, RCCL
all-reduce of the flat gradient + Adam after each replay).  Compares against the eager single-GPU step."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import pytorch_rt1_for_distributed_training_amd as rt1  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.data.synthetic import make_batch  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.models import build_rt1  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29541")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
t = torch.ones(4, device="cuda")
dist.all_reduce(t)                                  # creates the communicator (and the watchdog's work)
torch.cuda.synchronize()
cfg = rt1.RT1Config(height=128, width=128, seq_len=6, backend="hip", dropout_rate=0.0, drop_connect_rate=0.0,
                    crop_ratio=0.0)


def run(graph, force_dp):
    torch.manual_seed(0)
    eng = TrainEngine(build_rt1(cfg), cfg, order_probe=False, bucket_cap_mb=4.0, graph=graph)
    if force_dp:
        eng.ddp.enabled = True                      # world 1: every collective is a real 1-rank RCCL call
    g = torch.Generator().manual_seed(7)
    losses = [float(eng.train_step(make_batch(4, 6, 128, 128, device="cuda", generator=g))) for _ in range(5)]
    torch.cuda.synchronize()
    return eng, losses


eng, losses = run(True, True)
assert eng.graph and eng._graph is not None, "capture failed next to the RCCL communicator"
ref, ref_losses = run(False, False)
d = float((eng.flat.data - ref.flat.data).abs().max())
print(f"graph-DP(RCCL world 1) losses {losses}\neager losses           {ref_losses}\nmax |param diff| {d:.3e}",
      flush=True)
rel = max(abs(a - b) / abs(b) for a, b in zip(losses, ref_losses))
dist.destroy_process_group()
sys.exit(0 if rel < 1e-3 else 1)
