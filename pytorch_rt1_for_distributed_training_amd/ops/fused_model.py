"""The ``hip`` backend of the RT-1 policy: routes hot paths to HIP kernels.

``TransformerNetwork`` calls ``model.fused.<hook>`` when a FusedRT1 is
installed.  Each hook uses the fused HIP implementation of its component and
keeps the eager module as the numerical oracle (``tests/test_kernels_gpu.py``).
"""
from __future__ import annotations

import torch

from ..models import preprocess
from . import rng


class FusedRT1:
    def __init__(self, model, cfg):
        self.cfg = cfg
        self.dtype = torch.bfloat16 if cfg.dtype == "bf16" else torch.float32
        # fused gather + logits + CE + argmax kernel (csrc/kernels/head.hip) for the bf16 training path
        from .head import head_supported
        self.fused_head = self.dtype == torch.bfloat16 and head_supported(model._transformer._output_tokens)
        self._positions = {}
        self._flat = None
        self._bf16 = None
        self._views = {}
        self._tf_layers = list(model._transformer._layers) if hasattr(model, "_transformer") else []
        self._qkv_copy = None      # (dst list, src list): per-step packing of the Q/K/V weight / bias shadows
        self._packs = {}           # this model's fused Q/K/V buffers (attention._QKV while its forward runs)
        self._film_packs = {}      # ... and its packed FiLM projection operands (backbone._FILM_PACK)
        # the image tokenizer (a submodule: no reference back to this object, so no model <-> FusedRT1 cycle)
        self._tokenizer = getattr(model, "_image_tokenizer", None)
        if cfg.channels_last:
            model._image_tokenizer.to(memory_format=torch.channels_last)

    def attach_flat(self, flat):
        """Keep a bf16 shadow of the flat fp32 master weights: refreshed by ONE cast kernel at the start of
        every forward, it replaces the ~110 per-use weight casts of the encoder's GEMM calls."""
        if flat.data.device.type != "cuda" or self.dtype != torch.bfloat16:
            return
        self._flat = flat
        self._bf16 = torch.empty(flat.data.numel(), dtype=torch.bfloat16, device=flat.data.device)
        self._views = {}
        for p, off in zip(flat.params, flat.offsets):
            self._views[p.data_ptr()] = self._bf16[off:off + p.numel()].view(p.shape)
        self._pack_qkv()

    def _pack_qkv(self):
        """Per decoder layer, bf16 [3HD, E] / [3HD] buffers that hold the Q / K / V weight and bias shadows side by
        side; ``_refresh_shadow`` fills all of them in one multi-copy launch, so the layer's fused projection needs no
        per-step concatenation (3 launches per layer)."""
        from . import attention
        packs, dst, src = {}, [], []
        for ly in self._tf_layers:
            a = getattr(ly, "attn", None)
            lins = [getattr(a, n, None) for n in ("q_linear", "k_linear", "v_linear")] if a is not None else []
            if len(lins) != 3 or any(l is None or l.bias is None for l in lins):
                continue
            ws = [self._views.get(l.weight.data_ptr()) for l in lins]
            bs = [self._views.get(l.bias.data_ptr()) for l in lins]
            if any(v is None for v in ws + bs):
                continue
            W = torch.empty((sum(w.shape[0] for w in ws), ws[0].shape[1]), dtype=torch.bfloat16, device=ws[0].device)
            b = torch.empty(W.shape[0], dtype=torch.bfloat16, device=W.device)
            r = 0
            for w, bb in zip(ws, bs):
                dst += [W[r:r + w.shape[0]], b[r:r + w.shape[0]]]
                src += [w, bb]
                r += w.shape[0]
            packs[lins[0].weight.data_ptr()] = (W, b)
        self._film_packs = self._pack_film(dst, src)
        self._qkv_copy = (dst, src) if dst else None
        self._packs = packs
        attention.set_qkv_packs(packs)

    def _pack_film(self, dst, src):
        """The FiLM projections' bf16 weight shadows [sum C, 512] and fp32 biases [sum C] side by side (the operands
        of backbone.FilmFn's single GEMM), filled by the same per-step multi-copy launch as the Q/K/V packs."""
        from . import backbone
        enc = getattr(self._tokenizer, "_tokenizer", None)
        net = getattr(enc, "net", None)
        if net is None or not hasattr(net, "films") or not hasattr(enc, "film_layer"):
            return {}
        ws, bs, _ = backbone.film_params(net, enc)
        wv = [self._views.get(w.data_ptr()) for w in ws]
        if any(v is None for v in wv) or len({v.shape[1] for v in wv}) != 1:
            return {}
        W = torch.empty((sum(v.shape[0] for v in wv), wv[0].shape[1]), dtype=torch.bfloat16, device=wv[0].device)
        b = torch.empty(W.shape[0], dtype=torch.float32, device=W.device)
        r = 0
        for v, bb in zip(wv, bs):
            dst += [W[r:r + v.shape[0]], b[r:r + v.shape[0]]]
            src += [v, bb.data]
            r += v.shape[0]
        return {ws[0].data_ptr(): (W, b)}

    def _refresh_shadow(self):
        from . import backbone
        if self._flat is None:
            from . import attention
            backbone.set_weight_shadow(None)
            backbone.set_film_packs({})
            attention.set_qkv_packs({})
            return
        self._bf16.copy_(self._flat.data[:self._bf16.numel()])
        if self._qkv_copy is not None:
            from ._ext import load
            load().multi_copy_(*self._qkv_copy)
        backbone.set_weight_shadow(self._views)
        backbone.set_film_packs(self._film_packs)
        # re-installed every forward, like the weight shadow: another FusedRT1 (an eval model in the same process)
        # may have replaced the module-global packs since this model's attach_flat
        from . import attention
        attention.set_qkv_packs(self._packs)

    def _autocast(self):
        return torch.autocast("cuda", dtype=self.dtype, enabled=self.dtype != torch.float32)

    def device_shift(self, model, h, w, device, shift=None):
        """Random-shift offsets as a device int32[2] (graph-replayable RNG)."""
        if shift is not None:
            return torch.tensor(shift, dtype=torch.int32, device=device)
        ud, lr = preprocess.shift_pads(h, w, model._crop_ratio)
        return torch.cat([torch.randint(-ud, ud + 1, (1,), device=device, dtype=torch.int32),
                          torch.randint(-lr, lr + 1, (1,), device=device, dtype=torch.int32)])

    def tokenize_images(self, model, images, context, shift):
        from .backbone import encoder_forward
        b, t = images.shape[:2]
        frames = images.reshape(b * t, *images.shape[2:])
        if frames.dtype not in (torch.uint8, torch.float32):
            frames = frames.float()
        frames = frames.contiguous()
        rng.begin_forward(frames.device)
        dshift = self.device_shift(model, frames.shape[-2], frames.shape[-1], frames.device, shift)
        tok = model._image_tokenizer
        self._refresh_shadow()
        ctx = context.reshape(b * t, -1) if context is not None else None
        feats = encoder_forward(tok._tokenizer, frames, ctx, dshift, tok.training)   # [N, P, E] bf16
        if not tok._use_token_learner:
            return feats.reshape(b, t, feats.shape[1], -1)
        from .token_learner import supported, token_learner
        if self.dtype == torch.bfloat16 and supported(tok._token_learner, feats.shape[1]):
            tokens = token_learner(tok._token_learner, feats)             # csrc/kernels/tokenlearner.hip
        else:
            with self._autocast():
                tokens = tok._token_learner.forward_nhwc(feats)
        return tokens.reshape(b, t, tokens.shape[1], -1)

    def transformer_hidden(self, model, tokens):
        from .attention import fused_layer, fused_layer_supported, transformer_layer
        tf = model._transformer
        L, Kimg = model.tokens_per_step, model._tokens_per_context_image
        from . import embed as emb
        fused = self.dtype == torch.bfloat16 and all(fused_layer_supported(ly) for ly in tf._layers)
        if fused and emb.supported(tf, tokens):
            x = emb.embed(tf, tokens)                    # MFMA GEMM + bias + position rows -> fp32 (K11)
        else:
            with self._autocast():
                x = tf.embed(tokens)
        if fused:
            # fp32 residual stream through the fused HIP layers (LN / residual / dropout / attention kernels)
            x = x.float()
            layers = list(tf._layers)
            aux = None
            for i, layer in enumerate(layers):
                nxt = layers[i + 1].norm_1 if i + 1 < len(layers) else None
                x, aux = fused_layer(layer, x, L, Kimg, tf.training, aux, nxt)
        else:
            with self._autocast():
                for layer in tf._layers:
                    x = transformer_layer(layer, x, L, Kimg, tf.training)
        model._attention_scores = []
        return x

    def action_loss(self, model, logits, targets, b, t):
        import torch.nn.functional as F
        ce = F.cross_entropy(logits.float().reshape(-1, logits.shape[-1]), targets.reshape(-1), reduction="none")
        num_items = float(b * t) * model._single_time_step_num_tokens
        return (ce.view(b, t, model._tokens_per_action) / num_items).mean(dim=-1)

    def tokenize_actions(self, tokenizer, actions):
        """Action labels in one HIP launch (csrc/kernels/head.hip action_tokenize): -> (int64 labels, int32 copy for
        the fused CE head), or (labels, None) from the torch tokenizer when a component is not a GPU tensor."""
        keys, dims, low, high = tokenizer.flat_spec()
        comps = [actions[k] for k in keys]
        ok = all(isinstance(c, torch.Tensor) and c.is_cuda for c in comps) and len(low) <= 32 and len(keys) <= 8
        if ok:
            comps = [(c.float() if d > 0 else c).contiguous() for c, d in zip(comps, dims)]
            ok = all((c.dtype == torch.float32) if d > 0 else (c.dtype in (torch.int64, torch.int32))
                     for c, d in zip(comps, dims))
        if not ok:
            return tokenizer.tokenize(actions), None
        from . import load
        t64, t32 = load().action_tokenize(comps, dims, low, high, tokenizer._vocab_size)
        return t64, t32

    def head_and_loss(self, model, hidden, positions, targets, b, t, targets32=None):
        """Fused head: returns the reference loss (b, t) and the argmax action tokens (b, T*A)."""
        from .head import head_ce
        key = (positions.data_ptr(), positions.device)
        pos = self._positions.get(key)
        if pos is None:
            pos = positions.to(torch.int32).contiguous()
            self._positions[key] = pos
        ce, pred = head_ce(model._transformer._output_tokens, hidden, pos, targets, targets32)
        num_items = float(b * t) * model._single_time_step_num_tokens
        loss = (ce.view(b, t, model._tokens_per_action) / num_items).mean(dim=-1)
        return loss, pred.view(b, -1)

    def action_logits(self, model, hidden, positions):
        with self._autocast():
            return model._transformer._output_tokens(hidden[:, positions])
