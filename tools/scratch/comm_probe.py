"""Step-by-step probe of the native RCCL communicator (prints before every call)."""
import sys
import torch

def say(*a):
    print(*a, flush=True)

from pytorch_rt1_for_distributed_training_amd.ops import load
ext = load()
say("rccl version", ext.comm.rccl_version())
torch.cuda.init()
say("device", torch.cuda.current_device())
uid = ext.comm.unique_id()
say("uid", len(uid))
c = ext.comm.Communicator(uid, 1, 0, 0)
say("communicator ok")
t = torch.arange(16, device="cuda", dtype=torch.float32)
w = c.all_reduce_(t, "sum")
say("all_reduce issued")
w.wait()
torch.cuda.synchronize()
say("all_reduce done", t[:4].tolist())
w2 = c.broadcast_(t, 0)
w2.synchronize()
say("broadcast done")
w3 = c.all_reduce_coalesced_([t, t.clone()], "sum")
w3.synchronize()
say("coalesced done")
import os, time
mode = os.environ.get("PROBE_MODE", "destroy")
if mode == "destroy":
    c.destroy()
    say("destroyed")
    time.sleep(3)
    say("slept 3s after destroy")
elif mode == "leak":
    say("leaking communicator")
    time.sleep(3)
    say("slept 3s")
if os.environ.get("PROBE_HARD_EXIT"):
    os._exit(0)
