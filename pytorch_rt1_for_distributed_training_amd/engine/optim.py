"""Adam / AdamW over the flat parameter buffer.

The reference uses ``torch.optim.Adam(lr)`` (beta=(0.9,0.999), eps=1e-8,
weight_decay=0) stepped per batch and ``MultiStepLR(milestones, 0.1)`` stepped
per epoch (``distribute_train.py:99-110``).  ``FlatAdam`` is numerically the
same update but owns flat fp32 moment buffers aligned with
``parallel.FlatParameters`` so one fused HIP kernel (``ops.adam``) updates all
35.2M trainable parameters per step; it also folds the data-parallel 1/world
gradient average into that pass.  AdamW is the same kernel with decoupled
decay (``weight_decay > 0``); the default 0 keeps parity with the reference.

It subclasses ``torch.optim.Optimizer`` so torch LR schedulers drive
``param_groups[0]['lr']`` and ``state_dict()`` is emitted in torch-Adam layout
(per-parameter ``step``/``exp_avg``/``exp_avg_sq``) for Lightning-format
checkpoints.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import torch

from ..parallel.flat import FlatParameters


class FlatAdam(torch.optim.Optimizer):
    def __init__(self, flat: FlatParameters, lr: float = 5e-4, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, all_params: Optional[Sequence[torch.nn.Parameter]] = None,
                 use_kernel: Optional[bool] = None):
        self.flat = flat
        params = list(all_params) if all_params is not None else list(flat.params)
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False,
                                      maximize=False, foreach=None, capturable=False, differentiable=False,
                                      fused=None, decoupled_weight_decay=weight_decay > 0))
        self.exp_avg = torch.zeros_like(flat.data)
        self.exp_avg_sq = torch.zeros_like(flat.data)
        self.step_count = 0
        # device-resident step counter + lr so a captured graph replays correctly
        self.dev_state = torch.zeros(2, dtype=torch.float32, device=flat.data.device)
        self._dev_lr = None
        self._dev_step = None
        self._kernel = None
        if use_kernel is None:
            use_kernel = flat.data.is_cuda
        if use_kernel:
            from ..ops import adam as adam_ops
            self._kernel = adam_ops

    @torch.no_grad()
    def step(self, closure=None, grad_scale: float = 1.0):
        loss = closure() if closure is not None else None
        g = self.param_groups[0]
        lr, (b1, b2), eps, wd = g["lr"], g["betas"], g["eps"], g["weight_decay"]
        self.step_count += 1
        t = self.step_count
        self.flat.gather_grads()
        if self._kernel is not None:
            # {step, lr} live on the device and the step is advanced by a device op, so the eager step and a
            # captured hipGraph replay run the identical kernel (the host writes dev_state only when it is
            # out of date, e.g. after an lr-scheduler step -- never inside a capture)
            if not torch.cuda.is_current_stream_capturing() and (self._dev_step != t - 1 or self._dev_lr != lr):
                self.write_device_state(t - 1, lr)
            self.dev_state[0:1].add_(1.0)
            self._dev_step = t
            self._kernel.flat_adam_dev_step(self.flat.data, self.flat.grad, self.exp_avg, self.exp_avg_sq,
                                            self.dev_state, beta1=b1, beta2=b2, eps=eps, weight_decay=wd,
                                            grad_scale=grad_scale)
            return loss
        grad = self.flat.grad
        if grad_scale != 1.0:
            grad = grad * grad_scale
        p = self.flat.data
        if wd:
            p.mul_(1.0 - lr * wd)
        self.exp_avg.lerp_(grad, 1.0 - b1)
        self.exp_avg_sq.mul_(b2).addcmul_(grad, grad, value=1.0 - b2)
        bc1 = 1.0 - b1 ** t
        bc2 = 1.0 - b2 ** t
        denom = (self.exp_avg_sq.sqrt() / math.sqrt(bc2)).add_(eps)
        p.addcdiv_(self.exp_avg, denom, value=-lr / bc1)
        return loss

    def write_device_state(self, step: int, lr: float):
        """Host -> device write of {step, lr} (a small H2D copy; outside any capture)."""
        self.dev_state.copy_(torch.tensor([float(step), float(lr)]))
        self._dev_step = int(step)
        self._dev_lr = float(lr)

    def sync_device_state(self):
        self.write_device_state(self.step_count, self.param_groups[0]["lr"])

    def zero_grad(self, set_to_none: bool = True):
        self.flat.zero_grad(set_to_none)

    # -------------------------------------------------------------- torch-Adam layout (de)serialisation
    def state_dict(self) -> Dict:
        groups = []
        index: Dict[int, int] = {}
        for g in self.param_groups:
            ids = []
            for p in g["params"]:
                index.setdefault(id(p), len(index))
                ids.append(index[id(p)])
            d = {k: v for k, v in g.items() if k != "params"}
            d["params"] = ids
            groups.append(d)
        state = {}
        if self.step_count > 0:
            for p, o in zip(self.flat.params, self.flat.offsets):
                n = p.numel()
                state[index[id(p)]] = {"step": torch.tensor(float(self.step_count)),
                                       "exp_avg": self.exp_avg[o:o + n].view_as(p).detach().clone(),
                                       "exp_avg_sq": self.exp_avg_sq[o:o + n].view_as(p).detach().clone()}
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, sd: Dict):
        groups = sd["param_groups"]
        for g, sg in zip(self.param_groups, groups):
            for k, v in sg.items():
                if k != "params":
                    g[k] = v
        pos = {}
        for g in self.param_groups:
            for p in g["params"]:
                pos.setdefault(id(p), len(pos))
        steps = []
        with torch.no_grad():
            for p, o in zip(self.flat.params, self.flat.offsets):
                st = sd["state"].get(pos[id(p)], sd["state"].get(str(pos[id(p)])))
                if st is None:
                    continue
                n = p.numel()
                self.exp_avg[o:o + n].copy_(st["exp_avg"].reshape(-1))
                self.exp_avg_sq[o:o + n].copy_(st["exp_avg_sq"].reshape(-1))
                steps.append(int(float(st["step"])))
        self.step_count = max(steps) if steps else 0


def multistep_lr(optimizer: torch.optim.Optimizer, milestones: List[int], gamma: float = 0.1):
    return torch.optim.lr_scheduler.MultiStepLR(optimizer, milestones, gamma=gamma, last_epoch=-1)
