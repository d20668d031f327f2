"""Model / run configurations.

The reference hard-codes the RT-1 hyper-parameters in ``RT1_Lightning.__init__``
(``distribute_train.py:42-55``) and takes the rest from argparse
(``distribute_train.py:270-293``).  Here they live in one dataclass so the five
BASELINE configurations (tiny CPU, full bf16, DDP-8, long history, 456x456) are named presets rather than edited
literals.  Configuration 5 runs in bf16: an fp8 (e4m3fn) forward-GEMM path was built and measured 2.2 % slower than
bf16 at 456x456 in rounds 2-3 (profiles/r3_bench_b456_fp8.log vs r3_bench_b456_bf16.log: the GEMMs it covered are
HBM-bound, so the quantisation passes cost more than the faster MFMA saved) and was removed in round 5.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field
from typing import List, Optional


@dataclass
class RT1Config:
    # image / history
    height: int = 256
    width: int = 456
    seq_len: int = 6                 # time_sequence_length (T)
    # transformer
    vocab_size: int = 256
    token_embedding_size: int = 512
    num_layers: int = 8
    layer_size: int = 128            # key_dim per head
    num_heads: int = 8
    feed_forward_size: int = 512     # d_model
    dropout_rate: float = 0.1
    max_seq_len: int = 256           # learned position table (transformer.py:156)
    # image tokenizer
    use_token_learner: bool = True
    num_image_tokens: int = 8
    width_coefficient: float = 1.2   # EfficientNet-B3
    depth_coefficient: float = 1.4
    drop_connect_rate: float = 0.2
    text_embedding_size: int = 512
    crop_ratio: float = 0.07         # random-shift pad ratio (preprocessors.py:37)
    # action space (distribute_train.py:35-40)
    action_low: float = -0.1
    action_high: float = 0.1
    action_dim: int = 2
    terminate_classes: int = 2
    # numerics / backend
    dtype: str = "bf16"              # compute dtype: fp32 | bf16
    backend: str = "auto"            # torch | hip | auto (hip when the extension is present on GPU)
    channels_last: bool = True
    pretrained: Optional[str] = None  # torchvision efficientnet_b3 state dict for the backbone (weights='imagenet')

    @property
    def tokens_per_action(self) -> int:
        return 1 + self.action_dim

    @property
    def tokens_per_image(self) -> int:
        return self.num_image_tokens if self.use_token_learner else None

    def replace(self, **kw) -> "RT1Config":
        return dataclasses.replace(self, **kw)


def preset(name: str) -> RT1Config:
    """Named configurations from BASELINE.json ``configs``."""
    name = name.lower()
    if name in ("tiny", "rt1-tiny"):
        # RT-1-tiny (history=2, 64x64, 2-layer transformer) CPU fwd+bwd plumbing.
        return RT1Config(height=64, width=64, seq_len=2, num_layers=2, dtype="fp32", backend="torch",
                         channels_last=False)
    if name in ("full", "rt1", "full-300"):
        return RT1Config(height=300, width=300, seq_len=6)
    if name in ("ref", "full-256x456"):
        return RT1Config(height=256, width=456, seq_len=6)
    if name in ("long", "long-history"):
        return RT1Config(height=300, width=300, seq_len=15)
    if name in ("hires", "456"):
        return RT1Config(height=456, width=456, seq_len=6)
    if name in ("hires-fp8", "456-fp8"):
        raise ValueError("config 5 runs in bf16 (preset 'hires'): the fp8 forward-GEMM path measured 2.2 % slower "
                         "than bf16 at 456x456 (profiles/r3_bench_b456_fp8.log) and was removed")
    raise KeyError(f"unknown preset {name!r}")
