"""RT-1 policy network (``TransformerNetwork``).

Behavioural spec: ``pytorch_robotics_transformer/transformer_network.py``
(constructor ``:38-123``, masks ``:156-192``, forward ``:195-339``, token
assembly ``:378-390``, image/action tokenisation ``:423-502``, accessors
``:517-532``).  The public API is kept: ``forward(observations,
network_state) -> (actions, network_state)``, ``set_actions``,
``get_actor_loss``, ``get_aux_info``, ``attention_scores``, ``_state_space``.

Deliberate differences (all result-preserving):

* ``train_forward`` is the engine's entry: it takes ``(images, context,
  actions)`` directly — no fabricated ``network_state`` per step;
* the logits head runs only on the ``T*A`` positions that predict action
  tokens (gather-then-GEMM instead of GEMM-then-gather);
* the embedding of action tokens is skipped, because the reference zeroes it
  before the transformer (``:383``) — ``_action_token_emb`` is still a
  registered (gradient-free) parameter so checkpoints keep all 806 keys;
* inference evaluates the transformer ONCE per call instead of once per action
  token: inserted action tokens never reach the transformer input (they are
  zeroed), so the three reference passes are identical (verified in
  ``tests/test_policy.py``);
* ``seq_idx`` is returned with shape ``(b,)`` (the reference returns a 0-d
  tensor and the eval policy re-wraps it, ``language_table/train/policy.py:83``).
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import spaces
from . import preprocess
from .action_tokenizer import RT1ActionTokenizer
from .image_tokenizer import RT1ImageTokenizer
from .transformer import Transformer, action_prediction_positions, rt1_attention_mask


class TransformerNetwork(nn.Module):
    def __init__(self, input_tensor_space: spaces.Dict, output_tensor_space: spaces.Dict,
                 train_step_counter: int = 0, vocab_size: int = 256, token_embedding_size: int = 512,
                 num_layers: int = 1, layer_size: int = 4096, num_heads: int = 8, feed_forward_size: int = 512,
                 dropout_rate: float = 0.1, time_sequence_length: int = 1, crop_size: int = 236,
                 use_token_learner: bool = True, return_attention_scores: bool = False,
                 width_coefficient: float = 1.2, depth_coefficient: float = 1.4, drop_connect_rate: float = 0.2,
                 crop_ratio: float = 0.07):
        super().__init__()
        self._input_tensor_space = input_tensor_space
        self._output_tensor_space = output_tensor_space
        self._train_step_counter = train_step_counter
        self._vocab_size = vocab_size
        self._token_embedding_size = token_embedding_size
        self._time_sequence_length = time_sequence_length
        self._crop_size = crop_size
        self._crop_ratio = crop_ratio
        self._actions = None
        self._aux_info: Dict[str, Any] = {}
        self._loss = None
        self._attention_scores: List[torch.Tensor] = []
        self._use_token_learner = use_token_learner
        _, height, width = input_tensor_space["image"].shape

        # registration order == checkpoint key order
        self._transformer = Transformer(num_layers, layer_size, num_heads, feed_forward_size, dropout_rate,
                                        vocab_size, token_embedding_size, return_attention_scores)
        self._image_tokenizer = RT1ImageTokenizer(token_embedding_size, use_token_learner, 8, height, width,
                                                  width_coefficient=width_coefficient,
                                                  depth_coefficient=depth_coefficient,
                                                  drop_connect_rate=drop_connect_rate)
        self._action_tokenizer = RT1ActionTokenizer(output_tensor_space, vocab_size)
        self._tokens_per_action = self._action_tokenizer.tokens_per_action
        self._tokens_per_context_image = self._image_tokenizer.tokens_per_context_image
        self._single_time_step_num_tokens = self._tokens_per_action + self._tokens_per_context_image
        self._all_num_tokens = time_sequence_length * self._single_time_step_num_tokens
        self._action_token_emb = nn.Linear(vocab_size, token_embedding_size)
        self._action_token_emb.requires_grad_(False)  # dead weight kept for checkpoint parity

        self.register_buffer("_default_attention_mask",
                             rt1_attention_mask(time_sequence_length, self._tokens_per_context_image,
                                                self._tokens_per_action), persistent=False)
        self.register_buffer("_predicted_positions",
                             action_prediction_positions(time_sequence_length, self._tokens_per_context_image,
                                                         self._tokens_per_action), persistent=False)
        self._action_tokens_mask = (self._predicted_positions + 1).tolist()

        self._state_space = spaces.Dict({
            "context_image_tokens": spaces.Box(-np.inf, np.inf,
                                               (time_sequence_length, self._tokens_per_context_image,
                                                token_embedding_size), np.float32),
            "action_tokens": spaces.MultiDiscrete(np.full((time_sequence_length, self._tokens_per_action),
                                                          vocab_size)),
            "seq_idx": spaces.Discrete(time_sequence_length + 1),
        })
        # kernel hooks installed by ops.install(); None = eager torch path
        self.fused = None

    # ------------------------------------------------------------------ accessors
    @property
    def attention_scores(self) -> List[torch.Tensor]:
        return self._attention_scores

    @property
    def tokens_per_step(self) -> int:
        return self._single_time_step_num_tokens

    def set_actions(self, actions: Dict[str, torch.Tensor]):
        self._actions = actions

    def get_actor_loss(self) -> torch.Tensor:
        return self._loss

    def get_aux_info(self) -> Dict[str, Any]:
        return self._aux_info

    def initial_state(self, batch_size: int = 1, device=None) -> Dict[str, torch.Tensor]:
        """Zero network_state (what the eval loop uses at episode start)."""
        T, K, E, A = (self._time_sequence_length, self._tokens_per_context_image, self._token_embedding_size,
                      self._tokens_per_action)
        return {"context_image_tokens": torch.zeros(batch_size, T, K, E, device=device),
                "action_tokens": torch.zeros(batch_size, T, A, dtype=torch.long, device=device),
                "seq_idx": torch.zeros(batch_size, dtype=torch.long, device=device)}

    # ------------------------------------------------------------------ building blocks
    def _outer_rank(self, observations) -> int:
        k = next(iter(observations.keys()))
        return observations[k].dim() - len(self._input_tensor_space[k].shape)

    def tokenize_images(self, images: torch.Tensor, context: Optional[torch.Tensor], shift=None) -> torch.Tensor:
        """images (b, t, 3, H, W) in [0,1] (or uint8), context (b, t, D) -> (b, t, K, E)."""
        if self.fused is not None:
            return self.fused.tokenize_images(self, images, context, shift)
        b, t = images.shape[:2]
        frames = images.reshape(b * t, *images.shape[2:])
        frames = preprocess.convert_dtype_and_crop_images(frames, self._crop_ratio, shift)
        return self._image_tokenizer(frames.reshape(b, t, *frames.shape[1:]), context)

    def assemble_tokens(self, image_tokens: torch.Tensor) -> torch.Tensor:
        """[image tokens, zeroed action tokens] per step -> (b, T*L, E) (``:378-390``)."""
        b, t, k, e = image_tokens.shape
        zeros = image_tokens.new_zeros(b, t, self._tokens_per_action, e)
        return torch.cat((image_tokens, zeros), dim=2).reshape(b, t * (k + self._tokens_per_action), e)

    def transformer_hidden(self, tokens: torch.Tensor) -> torch.Tensor:
        if self.fused is not None:
            return self.fused.transformer_hidden(self, tokens)
        h, self._attention_scores = self._transformer.hidden(tokens, self._default_attention_mask)
        return h

    def action_logits(self, hidden: torch.Tensor, positions: torch.Tensor) -> torch.Tensor:
        if self.fused is not None:
            return self.fused.action_logits(self, hidden, positions)
        return self._transformer._output_tokens(hidden[:, positions])

    def action_loss(self, logits: torch.Tensor, targets: torch.Tensor, b: int, t: int) -> torch.Tensor:
        """CE(reduction=none) / (b*t*L), mean over the A tokens -> (b, t)  (``:314-322``)."""
        if self.fused is not None:
            return self.fused.action_loss(self, logits, targets, b, t)
        ce = F.cross_entropy(logits.float().reshape(-1, logits.shape[-1]), targets.reshape(-1), reduction="none")
        num_items = float(b * t) * self._single_time_step_num_tokens
        return (ce.view(b, t, self._tokens_per_action) / num_items).mean(dim=-1)

    # ------------------------------------------------------------------ training
    def train_forward(self, images: torch.Tensor, context: torch.Tensor, actions: Dict[str, torch.Tensor],
                      shift=None, with_aux: bool = True) -> Tuple[torch.Tensor, Dict[str, Any]]:
        b, t = images.shape[:2]
        targets32 = None
        if self.fused is not None and images.is_cuda:
            # one HIP launch for the labels (and the int32 copy the fused head reads)
            targets, targets32 = self.fused.tokenize_actions(self._action_tokenizer, actions)
        else:
            targets = self._action_tokenizer.tokenize(actions)                   # (b, t, A)
        image_tokens = self.tokenize_images(images, context, shift)
        hidden = self.transformer_hidden(self.assemble_tokens(image_tokens.to(self._compute_dtype(image_tokens))))
        preds = None
        if self.fused is not None and self.fused.fused_head:
            # one HIP kernel: gather + logits + CE + argmax (ops/head.py)
            loss, preds = self.fused.head_and_loss(self, hidden, self._predicted_positions, targets, b, t, targets32)
            preds = preds.view(b, t, self._tokens_per_action).long()
        else:
            logits = self.action_logits(hidden, self._predicted_positions)        # (b, T*A, V)
            loss = self.action_loss(logits, targets, b, t)
        # kept detached: holding the autograd graph across steps would pin the AccumulateGrad nodes to the
        # stream of the first step (breaks hipGraph capture); the reference-style forward() re-attaches it
        self._loss = loss.detach()
        aux: Dict[str, Any] = {"action_labels": targets, "action_loss": self._loss}
        if with_aux:
            if preds is None:
                preds = logits.detach().view(b, t, self._tokens_per_action, -1).argmax(dim=-1)
            aux.update({"action_predictions": preds,
                        "actor_loss_mask": torch.ones(b, dtype=torch.float32, device=loss.device),
                        "predicted_tokens_for_output": preds[:, -1]})
        self._aux_info = aux
        return loss, aux

    def _compute_dtype(self, x):
        return x.dtype

    # ------------------------------------------------------------------ reference-style entry
    def forward(self, observations: Dict[str, torch.Tensor], network_state: Dict[str, torch.Tensor]):
        outer_rank = self._outer_rank(observations)
        if outer_rank not in (1, 2):
            raise ValueError("outer rank should be 1 or 2")
        if outer_rank == 2:
            if self._actions is None:
                b, t = observations["image"].shape[:2]
                actions = {k: torch.zeros(b, t, *sp.shape, device=observations["image"].device)
                           for k, sp in self._output_tensor_space.items()}
            else:
                actions = self._actions
            loss, aux = self.train_forward(observations["image"], observations.get("natural_language_embedding"),
                                           actions)
            self._loss = loss                      # reference get_actor_loss() is backpropagated
            out = self._action_tokenizer.detokenize(aux["predicted_tokens_for_output"])
            return out, network_state
        return self._inference_step(observations, network_state)

    @torch.no_grad()
    def _inference_step(self, observations, network_state):
        T, L, K = self._time_sequence_length, self._single_time_step_num_tokens, self._tokens_per_context_image
        image = observations["image"]                                            # (b, 3, H, W)
        b = image.shape[0]
        ctx = observations.get("natural_language_embedding")
        ctx = ctx[:, None] if ctx is not None else None
        seq_idx_t = network_state["seq_idx"].reshape(-1)[0]
        seq_idx = int(seq_idx_t)
        time_step = min(seq_idx, T - 1)
        new_tokens = self.tokenize_images(image[:, None], ctx)                   # (b, 1, K, E)
        state_img = network_state["context_image_tokens"].to(new_tokens.device)
        state_act = network_state["action_tokens"].to(new_tokens.device)
        if seq_idx == T:
            state_img = torch.roll(state_img, -1, 1)
            state_act = torch.roll(state_act, -1, 1)
        state_img = torch.cat([state_img[:, :time_step], new_tokens.to(state_img.dtype),
                               state_img[:, time_step + 1:]], dim=1)
        hidden = self.transformer_hidden(self.assemble_tokens(state_img.to(new_tokens.dtype)))
        start = K - 1 + time_step * L
        pos = torch.arange(start, start + self._tokens_per_action, device=hidden.device)
        logits = self.action_logits(hidden, pos)                                 # (b, A, V)
        tokens = logits.argmax(dim=-1)
        state_act = state_act.clone()
        state_act[:, time_step] = tokens.to(state_act.dtype)
        new_state = {"context_image_tokens": state_img, "action_tokens": state_act,
                     "seq_idx": torch.full((b,), min(seq_idx + 1, T), dtype=torch.long, device=hidden.device)}
        self._aux_info = {"action_labels": state_act, "action_predictions_logits": logits}
        self._loss = torch.tensor(0.0)
        return self._action_tokenizer.detokenize(tokens), new_state
