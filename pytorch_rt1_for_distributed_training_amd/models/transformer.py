"""Decoder-only RT-1 transformer and the RT-1 attention mask.

Spec: ``pytorch_robotics_transformer/transformer.py``:
* ``TF_MultiHeadAttention`` (``:29-79``): separate q/k/v Linear(d_model ->
  heads*key_dim) and out Linear(heads*key_dim -> d_model);
* ``attention`` (``:82-109``): ``softmax(QK^T/sqrt(key_dim)`` masked with
  -1e9 where mask==0) -> dropout -> @V;
* ``_TransformerLayer`` (``:112-144``): pre-LN attention residual, then
  ``LN -> Linear(d,d) -> Dropout -> +res`` (a single Linear, no activation);
* ``Transformer`` (``:146-198``): token Linear + learned positions (table of
  256), N layers, logits head, no final LayerNorm.

The RT-1 mask (``transformer_network.py:156-192``) is built vectorised here and
is also expressible arithmetically, which is what the HIP attention kernel does
(it never reads a mask tensor): with ``step = pos // L`` and ``is_act = pos % L
>= K`` (L tokens per step, K image tokens), query i may see key j iff
``j <= i and not is_act[j]`` or ``j <= i and not is_act[i] and is_act[j]``,
i.e. ``j <= i and (not is_act[j] or not is_act[i])``.
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F


def rt1_attention_mask(seq_steps: int, image_tokens: int, action_tokens: int) -> torch.Tensor:
    """(S, S) uint8 mask, 1 = attend.  S = seq_steps * (image_tokens + action_tokens)."""
    L = image_tokens + action_tokens
    S = seq_steps * L
    pos = torch.arange(S)
    is_act = (pos % L) >= image_tokens
    causal = pos[None, :] <= pos[:, None]
    both_act = is_act[:, None] & is_act[None, :]
    return (causal & ~both_act).to(torch.uint8)


def action_prediction_positions(seq_steps: int, image_tokens: int, action_tokens: int) -> torch.Tensor:
    """Output positions whose logits predict the action tokens (``_action_tokens_mask - 1``)."""
    L = image_tokens + action_tokens
    act_pos = torch.tensor([s * L + image_tokens + a for s in range(seq_steps) for a in range(action_tokens)])
    return act_pos - 1


def masked_attention(q, k, v, mask: Optional[torch.Tensor], dropout_p: float, training: bool,
                     return_scores: bool = False):
    """Eager reference: q,k,v (B, H, S, D)."""
    scores = torch.matmul(q, k.transpose(-2, -1)) / math.sqrt(q.shape[-1])
    if mask is not None:
        scores = scores.masked_fill(mask.to(scores.device)[None, None] == 0, -1e9)
    probs = torch.softmax(scores.float(), dim=-1).to(q.dtype)
    if dropout_p > 0 and training:
        probs = F.dropout(probs, dropout_p, True)
    out = torch.matmul(probs, v)
    return (out, probs) if return_scores else (out, None)


class TF_MultiHeadAttention(nn.Module):
    def __init__(self, heads: int, d_model: int, key_dim: int, value_dim: Optional[int] = None,
                 dropout: float = 0.1, return_attention_scores: bool = False):
        super().__init__()
        self.h = heads
        self.key_dim = key_dim
        self.value_dim = value_dim or key_dim
        self.return_attention_scores = return_attention_scores
        self.q_linear = nn.Linear(d_model, heads * key_dim)
        self.k_linear = nn.Linear(d_model, heads * key_dim)
        self.v_linear = nn.Linear(d_model, heads * self.value_dim)
        self.dropout = nn.Dropout(dropout)
        self.out = nn.Linear(heads * self.value_dim, d_model)

    def forward(self, q, k, v, mask=None):
        bs, s, _ = q.shape
        qh = self.q_linear(q).view(bs, s, self.h, self.key_dim).transpose(1, 2)
        kh = self.k_linear(k).view(bs, k.shape[1], self.h, self.key_dim).transpose(1, 2)
        vh = self.v_linear(v).view(bs, v.shape[1], self.h, self.value_dim).transpose(1, 2)
        o, scores = masked_attention(qh, kh, vh, mask, self.dropout.p, self.training, self.return_attention_scores)
        o = o.transpose(1, 2).reshape(bs, s, self.h * self.value_dim)
        out = self.out(o)
        return (out, scores) if self.return_attention_scores else out


class _TransformerLayer(nn.Module):
    def __init__(self, layer_size: int = 128, num_heads: int = 8, feed_forward_size: int = 512,
                 dropout_rate: float = 0.1, return_attention_scores: bool = False):
        super().__init__()
        self._return_attention_scores = return_attention_scores
        self.norm_1 = nn.LayerNorm(feed_forward_size)
        self.attn = TF_MultiHeadAttention(num_heads, feed_forward_size, layer_size, dropout=dropout_rate,
                                          return_attention_scores=return_attention_scores)
        self.ff = nn.Linear(feed_forward_size, feed_forward_size)
        self.norm_2 = nn.LayerNorm(feed_forward_size)
        self.dropout_1 = nn.Dropout(dropout_rate)

    def forward(self, x, mask):
        r = self.attn(*(3 * (self.norm_1(x),)), mask=mask)
        a, score = r if self._return_attention_scores else (r, None)
        x = x + a
        x = x + self.dropout_1(self.ff(self.norm_2(x)))
        return x, score


class Transformer(nn.Module):
    def __init__(self, num_layers: int = 8, layer_size: int = 128, num_heads: int = 8,
                 feed_forward_size: int = 512, dropout_rate: float = 0.1, vocab_size: int = 256,
                 input_token_emb_dim: int = 512, return_attention_scores: bool = False, max_seq_len: int = 256):
        super().__init__()
        self._layers = nn.ModuleList(
            _TransformerLayer(layer_size, num_heads, feed_forward_size, dropout_rate, return_attention_scores)
            for _ in range(num_layers))
        self._token_emb = nn.Linear(input_token_emb_dim, feed_forward_size)
        self._position_emb = nn.Embedding(max_seq_len, feed_forward_size)
        self._output_tokens = nn.Linear(feed_forward_size, vocab_size)
        self.max_seq_len = max_seq_len

    def embed(self, inputs: torch.Tensor) -> torch.Tensor:
        s = inputs.shape[1]
        if s > self.max_seq_len:
            raise ValueError(f"sequence of {s} tokens exceeds the learned position table ({self.max_seq_len})")
        return self._token_emb(inputs) + self._position_emb.weight[:s].to(inputs.dtype)

    def hidden(self, inputs: torch.Tensor, attention_mask: torch.Tensor) -> Tuple[torch.Tensor, List[torch.Tensor]]:
        x = self.embed(inputs)
        scores = []
        for layer in self._layers:
            x, sc = layer(x, attention_mask)
            if sc is not None:
                scores.append(sc)
        return x, scores

    def forward(self, inputs: torch.Tensor, attention_mask: torch.Tensor):
        x, scores = self.hidden(inputs, attention_mask)
        return self._output_tokens(x), scores
