#!/usr/bin/env python3
"""Which hip-backend path sets the precision of a gradient tensor?  Whole-model step (the setup of
tests/test_parity_gpu.py::test_full_model_step_hip_bf16_vs_torch_fp32) repeated with kernel-path switches, each in a
fresh process (the switches are read at import), printing the cosine vs fp32 of the watched tensors for the hip backend
and for torch's own bf16 autocast in the same process.

  python tools/parity_ablation.py                          # all variants
  python tools/parity_ablation.py --one proj_bwd=0      # one variant (ops/switches.py names), this process
"""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WATCH = ["_image_tokenizer._tokenizer.net.blocks.0.block.1.fc1.weight",
         "_image_tokenizer._tokenizer.net.blocks.2.block.2.fc1.weight",
         "_image_tokenizer._tokenizer.net.blocks.0.block.1.fc2.weight",
         "_image_tokenizer._tokenizer.net.blocks.0.block.0.0.weight",
         "_image_tokenizer._tokenizer.net.blocks.0.block.2.0.weight"]
VARIANTS = ["", "proj_bwd=0", "stem_in_block0=0", "dw_fused=0", "pw_pro=0", "se_fused=0",
            "proj_bwd=0,pw_pro=0,dw_fused=0,stem_in_block0=0"]


def run_one(seed: int):
    import torch
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, ROOT)
    import test_parity_gpu as T
    from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine
    from pytorch_rt1_for_distributed_training_amd.models import build_rt1
    eh, et = T._engines()
    cb = et.cfg.replace(dtype="bf16")
    mb = build_rt1(cb)
    mb.load_state_dict(et.model.state_dict())
    eb = TrainEngine(mb, cb, order_probe=False, device=torch.device("cuda"))
    batch = T._batch(eh.cfg, seed=seed)
    eh._batch = et._batch = eb._batch = batch
    for e in (eh, et, eb):
        e.model.train()
    _, gh = T._grads(eh)
    _, gt = T._grads(et)
    _, gb = T._grads(eb)
    cos = lambda a, b: float(torch.dot(a.flatten(), b.flatten()) / (a.norm() * b.norm() + 1e-30))
    out = []
    for n in WATCH:
        out.append(f"{n.split('net.')[-1]}: hip {cos(gh[n], gt[n]):.4f} torch-bf16 {cos(gb[n], gt[n]):.4f}")
    allc = sorted(cos(gh[n], gt[n]) for n in gt if float(gt[n].norm()) > 0)
    print(" | ".join(out) + f" | hip median {allc[len(allc) // 2]:.4f}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--one", default=None)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--variants", nargs="*", default=None, help="subset of variants ('' = default)")
    a = ap.parse_args()
    if a.one is not None:
        run_one(a.seed)
        return
    for v in (VARIANTS if a.variants is None else a.variants):
        env = dict(os.environ, PYTHONPATH=ROOT, RT1_AB=v)      # ops/switches.py overrides
        print(f"== {v or 'default'}", flush=True)
        r = subprocess.run([sys.executable, __file__, "--one", v, "--seed", str(a.seed)], env=env, timeout=600)
        if r.returncode:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
