"""Closed-loop RT-1 inference on MI355X: the HIP backend, a device-resident rolling state, one hipGraph per step.

The reference runs inference as three full transformer passes per policy step on a host-managed state
(``/root/reference/pytorch_robotics_transformer/transformer_network.py:230-292``) and calls
``torch.cuda.empty_cache()`` after every action (``language_table/train/policy.py:57-100``).  Here a policy step is

    tokenize the new frame (fused FiLM-EfficientNet + TokenLearner, eval-mode BN)  ->  roll the image-token
    window when it is full and write the new tokens at ``min(seq_idx, T-1)``  ->  ONE transformer pass over the
    T*L window  ->  logits at the 3 action positions of the current step  ->  argmax  ->  detokenize

with every index (roll, insert slot, gather positions) computed on the device from a device ``seq_idx``, so the
whole step has static shapes, no host synchronisation and is captured once as a hipGraph; a step is then one
H2D copy of the frame + one graph replay + one D2H copy of the action.  The single pass is exact: action-token
inputs are zero vectors (``transformer_network.py:383``), so the three reference passes produce identical logits
(SURVEY K23).

On caching K/V across steps: RT-1 adds a learned ABSOLUTE position embedding to every token and, once the window
is full (step >= T), rolls the whole window left by one step each call (``:289-290, 467-468``): every token moves
to a new position, its layer-0 input changes, and so do its keys and values in every layer.  Cached K/V are
therefore only valid during the first T-1 steps of an episode; this engine keeps the exact single pass (66 tokens
are a few microseconds of MFMA work) and spends its effort on removing launch overhead instead.
"""
from __future__ import annotations

import time
from typing import Dict, Optional

import numpy as np
import torch

from ..config import RT1Config
from ..parallel.flat import FlatParameters


class InferenceEngine:
    def __init__(self, model: torch.nn.Module, cfg: Optional[RT1Config] = None, device=None, batch_size: int = 1,
                 graph: Optional[bool] = None, backend: str = "auto"):
        if cfg is None:
            _, H0, W0 = model._input_tensor_space["image"].shape
            cfg = RT1Config(height=int(H0), width=int(W0), seq_len=model._time_sequence_length)
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        self.model = model.to(self.device).eval()
        self.cfg = cfg
        self.b = int(batch_size)
        cuda = self.device.type == "cuda"
        if backend == "auto":
            from ..ops import available
            backend = "hip" if (cuda and available()) else "torch"
        self.backend = backend
        if backend == "hip":
            if not cuda:
                raise ValueError("the hip backend needs a GPU")
            from ..ops import install
            install(self.model, cfg)
            # bf16 weight shadow over one flat buffer (one cast kernel per step instead of one per GEMM)
            trainable = [p for p in self.model.parameters()]
            self._flat = FlatParameters(trainable, device=self.device)
            self.model.fused.attach_flat(self._flat)
        m = self.model
        self.T, self.L = m._time_sequence_length, m.tokens_per_step
        self.K, self.A = m._tokens_per_context_image, m._tokens_per_action
        E = m._token_embedding_size
        H, W = cfg.height, cfg.width
        dev = self.device
        # static, device-resident inputs and state
        self.image = torch.zeros(self.b, 3, H, W, dtype=torch.uint8, device=dev)
        self.context = torch.zeros(self.b, cfg.text_embedding_size, device=dev)
        self.state_img = torch.zeros(self.b, self.T, self.K, E, device=dev)
        self.state_act = torch.zeros(self.b, self.T, self.A, dtype=torch.long, device=dev)
        self.seq_idx = torch.zeros((), dtype=torch.long, device=dev)
        self._ar_T = torch.arange(self.T, device=dev)
        self._ar_A = torch.arange(self.A, device=dev)
        self.graph = (graph if graph is not None else True) and backend == "hip"
        self._g = None
        self._out = None
        self.last_logits = None

    # ---------------------------------------------------------------- the step (device ops only)
    def _body(self):
        m = self.model
        T, L, K, A = self.T, self.L, self.K, self.A
        new = m.tokenize_images(self.image[:, None], self.context[:, None])            # (b, 1, K, E)
        full = (self.seq_idx == T).long()
        order = (self._ar_T + full) % T                                                # roll left by one when full
        simg = self.state_img.index_select(1, order)
        sact = self.state_act.index_select(1, order)
        ts = torch.clamp(self.seq_idx, max=T - 1).view(1)
        simg.index_copy_(1, ts, new.to(simg.dtype))
        hidden = m.transformer_hidden(m.assemble_tokens(simg.to(new.dtype)))
        pos = (K - 1) + ts * L + self._ar_A                                            # predicting positions
        logits = m.action_logits(hidden, pos)                                          # (b, A, V)
        tokens = logits.argmax(dim=-1)
        sact.index_copy_(1, ts, tokens.view(self.b, 1, A))
        self.state_img.copy_(simg)
        self.state_act.copy_(sact)
        self.seq_idx.copy_(torch.clamp(self.seq_idx + 1, max=T))
        act = m._action_tokenizer.detokenize(tokens)
        return {"tokens": tokens, "logits": logits.float(), **{k: v.float() for k, v in act.items()}}

    def reset(self):
        self.state_img.zero_()
        self.state_act.zero_()
        self.seq_idx.zero_()

    def _capture(self):
        torch.cuda.synchronize(self.device)
        saved = (self.state_img.clone(), self.state_act.clone(), self.seq_idx.clone())
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s), torch.no_grad():
            self._body()                                       # warm-up (lazy init, cached bounds / positions)
        torch.cuda.current_stream(self.device).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(g):
            self._out = self._body()
        self._g = g
        self.state_img.copy_(saved[0])
        self.state_act.copy_(saved[1])
        self.seq_idx.copy_(saved[2])

    @torch.no_grad()
    def step(self, image, context) -> Dict[str, torch.Tensor]:
        """image: (b, 3, H, W) uint8 or [0, 1] float (any device); context: (b, 512).  Returns device tensors."""
        image = torch.as_tensor(image)
        if image.dtype != torch.uint8:
            image = (image.float().clamp(0, 1) * 255.0).round().to(torch.uint8)
        self.image.copy_(image.reshape(self.image.shape), non_blocking=True)
        self.context.copy_(torch.as_tensor(context, dtype=torch.float32).reshape(self.context.shape),
                           non_blocking=True)
        if not self.graph:
            out = self._body()
        else:
            if self._g is None:
                self._capture()
            self._g.replay()
            out = self._out
        self.last_logits = out["logits"]
        return out

    def latency_ms(self, steps: int = 50, warmup: int = 5) -> float:
        """Median wall time of one policy step (frame H2D + step + action D2H), for reports."""
        img = torch.randint(0, 256, tuple(self.image.shape), dtype=torch.uint8)
        ctx = torch.randn(tuple(self.context.shape))
        for _ in range(warmup):
            self.step(img, ctx)["action"].cpu()
        ts = []
        for _ in range(steps):
            t0 = time.perf_counter()
            self.step(img, ctx)["action"].cpu()
            ts.append(1e3 * (time.perf_counter() - t0))
        self.reset()
        return float(np.median(ts))
