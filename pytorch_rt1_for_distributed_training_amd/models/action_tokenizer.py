"""Action <-> token conversion for RT-1.

Spec: ``tokenizers/action_tokenizer.py:68-159``.  Discrete actions are already
tokens; Box actions are clamped to [low, high], normalised to [0, 1], scaled by
``vocab_size - 1`` and *truncated* (not rounded) to an integer bucket.
Detokenize inverts the scaling; a discrete token is reset to 0 when it is
``> n`` (the reference's off-by-one check, kept for behavioural parity —
SURVEY §2.10 item 6).

Device-agnostic: ``low``/``high`` live on whatever device the action is on (the
reference hard-codes ``.to('cuda')``).
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch

from .. import spaces


class RT1ActionTokenizer:
    def __init__(self, action_space: spaces.Dict, vocab_size: int):
        self._action_space = action_space
        self._vocab_size = int(vocab_size)
        self._action_order = list(action_space.keys())
        n = 0
        for k in self._action_order:
            sp = action_space[k]
            if isinstance(sp, spaces.Discrete):
                n += 1
            elif isinstance(sp, spaces.Box):
                if len(sp.shape) != 1:
                    raise ValueError(f"Only action shapes with single dimension supported, got {sp.shape}")
                n += sp.shape[0]
            else:
                raise ValueError("action spaces must be Discrete or Box")
        self._tokens_per_action = n
        self._bounds_cache: Dict = {}

    @property
    def tokens_per_action(self) -> int:
        return self._tokens_per_action

    @property
    def action_order(self):
        return list(self._action_order)

    def _bounds(self, key, device, dtype):
        ck = (key, device, dtype)
        if ck not in self._bounds_cache:
            sp = self._action_space[key]
            self._bounds_cache[ck] = (torch.as_tensor(sp.low, dtype=dtype, device=device),
                                      torch.as_tensor(sp.high, dtype=dtype, device=device))
        return self._bounds_cache[ck]

    def flat_spec(self):
        """(keys, dims, low, high) of the concatenated tokens: dims[i] = Box width or 0 for a Discrete component, low /
        high one float per token (0 / 1 for Discrete) -- the layout of the fused HIP tokenizer (ops action_tokenize)."""
        if getattr(self, "_flat_spec", None) is None:
            keys, dims, low, high = [], [], [], []
            for k in self._action_order:
                sp = self._action_space[k]
                keys.append(k)
                if isinstance(sp, spaces.Discrete):
                    dims.append(0)
                    low.append(0.0)
                    high.append(1.0)
                else:
                    dims.append(int(sp.shape[0]))
                    low += [float(v) for v in np.asarray(sp.low, dtype=np.float32).reshape(-1)]
                    high += [float(v) for v in np.asarray(sp.high, dtype=np.float32).reshape(-1)]
            self._flat_spec = (keys, dims, low, high)
        return self._flat_spec

    def tokenize(self, action: Dict[str, torch.Tensor]) -> torch.Tensor:
        out = []
        for k in self._action_order:
            a = torch.as_tensor(action[k])
            sp = self._action_space[k]
            if isinstance(sp, spaces.Discrete):
                # host-side range check only for host tensors: on the GPU it would be a device->host sync
                # every step (and is illegal inside a captured hipGraph)
                if not a.is_cuda and not bool(torch.all(a < self._vocab_size)):
                    raise ValueError("Discrete action should be smaller than vocab size.")
                out.append(a.to(torch.int64).unsqueeze(-1))
            else:
                a = a.to(torch.float32)
                low, high = self._bounds(k, a.device, a.dtype)
                a = torch.minimum(torch.maximum(a, low), high)
                tok = (a - low) / (high - low) * (self._vocab_size - 1)
                out.append(tok.to(torch.int32).to(torch.int64))
        return torch.cat(out, dim=-1)

    def detokenize(self, action_tokens: torch.Tensor) -> Dict[str, torch.Tensor]:
        action = {}
        idx = 0
        for k in self._action_order:
            sp = self._action_space[k]
            if isinstance(sp, spaces.Discrete):
                t = action_tokens[..., idx]
                action[k] = torch.where(t > sp.n, torch.zeros_like(t), t)
                idx += 1
            else:
                d = sp.shape[0]
                t = action_tokens[..., idx:idx + d].to(torch.float32) / (self._vocab_size - 1)
                low, high = self._bounds(k, t.device, torch.float32)   # cached: no H2D copy per call / in a graph
                action[k] = t * (high - low) + low
                idx += d
        return action
