"""Produce golden outputs of the *reference* RT-1 implementation for parity tests.

Runs the reference source read-only from /root/reference (never copied) with
throwaway shims for its missing imports (torchvision.ops, gym.spaces,
skimage.data) created under /tmp, and with its two hard-coded ``.to('cuda')``
calls patched out so it runs on CPU.  Weights are filled by the deterministic
``seeded_init`` procedure that ``tests/test_reference_parity.py`` applies to
this framework's model (identical key order = identical weights), so the
fixture only has to hold inputs' seeds and the outputs.

Usage:  python tools/make_reference_golden.py  -> tests/fixtures/reference_golden.json
"""
from __future__ import annotations

import json
import math
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
SHIM = "/tmp/rt1_ref_shim"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def _write(path, text):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        f.write(text)


def make_shims():
    _write(f"{SHIM}/torchvision/__init__.py", "")
    _write(f"{SHIM}/torchvision/ops/__init__.py", """
import torch, torch.nn as nn
class StochasticDepth(nn.Module):
    def __init__(self, p, mode):
        super().__init__(); self.p = p
    def forward(self, x):
        if not self.training or self.p == 0: return x
        s = 1 - self.p
        noise = torch.empty([x.shape[0]] + [1] * (x.ndim - 1), dtype=x.dtype, device=x.device).bernoulli_(s)
        return x * noise.div_(s)
""")
    _write(f"{SHIM}/torchvision/ops/misc.py", """
import torch.nn as nn
class Conv2dNormActivation(nn.Sequential):
    def __init__(self, cin, cout, kernel_size=3, stride=1, padding=None, groups=1, norm_layer=nn.BatchNorm2d,
                 activation_layer=nn.ReLU, dilation=1, inplace=None, bias=None):
        padding = (kernel_size - 1) // 2 * dilation if padding is None else padding
        bias = norm_layer is None if bias is None else bias
        layers = [nn.Conv2d(cin, cout, kernel_size, stride, padding, dilation=dilation, groups=groups, bias=bias)]
        if norm_layer is not None: layers.append(norm_layer(cout))
        if activation_layer is not None: layers.append(activation_layer())
        super().__init__(*layers)
""")
    _write(f"{SHIM}/gym/__init__.py", "")
    import pytorch_rt1_for_distributed_training_amd.spaces as sp
    _write(f"{SHIM}/gym/spaces.py", open(sp.__file__).read())
    _write(f"{SHIM}/skimage/__init__.py", "")
    _write(f"{SHIM}/skimage/data.py", "")


def seeded_init(module: torch.nn.Module, seed: int = 1234):
    """Deterministic non-trivial weights, assigned in state-dict order."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, t in module.state_dict().items():
            if not t.is_floating_point():
                continue
            if name.endswith("running_var"):
                t.copy_(0.5 + torch.rand(t.shape, generator=g))
            elif name.endswith("running_mean"):
                t.copy_(0.1 * torch.randn(t.shape, generator=g))
            elif t.dim() <= 1:
                t.copy_(1.0 + 0.1 * torch.randn(t.shape, generator=g) if "norm" in name.lower() or
                        name.endswith(".1.weight") else 0.05 * torch.randn(t.shape, generator=g))
            else:
                fan_in = t[0].numel()
                t.copy_(torch.randn(t.shape, generator=g) / math.sqrt(fan_in))


def inputs(b, t, h, w, seed=7):
    g = torch.Generator().manual_seed(seed)
    return {
        "image": torch.rand(b, t, 3, h, w, generator=g),
        "emb": torch.randn(b, t, 512, generator=g),
        "term": torch.randint(0, 2, (b, t), generator=g),
        "act": (torch.rand(b, t, 2, generator=g) - 0.5) * 0.24,
    }


def build_reference(h, w, T, layers):
    make_shims()
    sys.path.insert(0, SHIM)
    sys.path.insert(0, REF)
    from pytorch_robotics_transformer import transformer as rtf
    from pytorch_robotics_transformer.tokenizers import action_tokenizer as rat
    from pytorch_robotics_transformer import transformer_network as rtn
    from pytorch_robotics_transformer.film_efficientnet import pretrained_efficientnet_encoder as pee
    import torch.nn.functional as F

    def attention(q, k, v, key_dim, mask=None, dropout=None, return_attention_scores=False):
        scores = torch.matmul(q, k.transpose(-2, -1)) / math.sqrt(key_dim)
        if mask is not None:
            scores = scores.masked_fill(mask.unsqueeze(0).unsqueeze(1) == 0, -1e9)
        scores = F.softmax(scores, dim=-1)
        if dropout is not None:
            scores = dropout(scores)
        out = torch.matmul(scores, v)
        return (out, scores) if return_attention_scores else out
    rtf.attention = attention

    orig_tok = rat.RT1ActionTokenizer.tokenize

    def tokenize(self, action):
        out = []
        for k in self._action_order:
            a = action[k]
            sp = self._action_space[k]
            if hasattr(sp, "n"):
                out.append(a.unsqueeze(-1))
            else:
                low, high = torch.tensor(sp.low), torch.tensor(sp.high)
                a = torch.clamp(a, low, high)
                out.append(((a - low) / (high - low) * (self._vocab_size - 1)).to(torch.int32))
        return torch.concat(out, dim=-1)
    rat.RT1ActionTokenizer.tokenize = tokenize

    orig_init = pee.EfficientNetEncoder.__init__

    def enc_init(self, token_embedding_size=512, weights=None, early_film=True, include_top=False, pooling=True):
        orig_init(self, token_embedding_size, None, early_film, include_top, pooling)
    pee.EfficientNetEncoder.__init__ = enc_init

    from collections import OrderedDict
    from gym import spaces
    obs = spaces.Dict({"image": spaces.Box(0.0, 1.0, (3, h, w), np.float32),
                       "natural_language_embedding": spaces.Box(-np.inf, np.inf, (512,), np.float32)})
    act = spaces.Dict(OrderedDict([("terminate_episode", spaces.Discrete(2)),
                                   ("action", spaces.Box(-0.1, 0.1, (2,), np.float32))]))
    return rtn.TransformerNetwork(obs, act, vocab_size=256, token_embedding_size=512, num_layers=layers,
                                  layer_size=128, num_heads=8, feed_forward_size=512, dropout_rate=0.1,
                                  time_sequence_length=T, crop_size=236, use_token_learner=True)


def no_dropout(m):
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
        if type(mod).__name__ == "StochasticDepth":
            mod.p = 0.0


def run_case(name, h, w, T, layers, b, train_mode):
    torch.manual_seed(0)
    ref = build_reference(h, w, T, layers)
    seeded_init(ref)
    no_dropout(ref)
    ref.train(train_mode)
    x = inputs(b, T, h, w)
    ref.set_actions({"terminate_episode": x["term"], "action": x["act"]})
    state = {"context_image_tokens": torch.zeros(b, T, 8, 512), "action_tokens": torch.zeros(b, T, 3, dtype=torch.long),
             "seq_idx": torch.zeros(b, dtype=torch.long)}
    torch.manual_seed(42)  # the random-shift crop draws from the global RNG
    with torch.no_grad():
        out, _ = ref({"image": x["image"], "natural_language_embedding": x["emb"]}, state)
    loss = ref.get_actor_loss()
    aux = ref.get_aux_info()
    keys = [(k, list(v.shape)) for k, v in ref.state_dict().items()]
    return {
        "name": name, "h": h, "w": w, "T": T, "layers": layers, "b": b, "train_mode": train_mode,
        "loss": loss.double().tolist(),
        "mean_loss": float(loss.mean()),
        "action_predictions": aux["action_predictions"].tolist(),
        "out_action": out["action"].double().tolist(),
        "out_terminate": out["terminate_episode"].tolist(),
        "action_labels": aux["action_labels"].tolist(),
        "num_keys": len(keys), "keys": keys if name == "tiny_eval" else None,
    }


def main():
    cases = [run_case("tiny_eval", 64, 64, 2, 2, 2, False),
             run_case("tiny_train", 64, 64, 2, 2, 2, True),
             run_case("full_keys_eval", 96, 160, 6, 8, 1, False)]
    out = os.path.join(os.path.dirname(HERE), "tests", "fixtures", "reference_golden.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump({"generator": "tools/make_reference_golden.py", "cases": cases}, f)
    for c in cases:
        print(c["name"], c["mean_loss"], c["num_keys"])


if __name__ == "__main__":
    main()
