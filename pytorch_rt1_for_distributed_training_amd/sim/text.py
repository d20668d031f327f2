"""Instruction -> 512-d embedding for the RT-1 context input.

The reference embeds instructions with the Universal Sentence Encoder (large/5) from TF-Hub
(``rlds_np_convert.py:26-33,48``, ``language_table/common/rt1_tokenizer.py``), re-loading the hub
model on every call.  Neither TensorFlow nor the model is available offline, so the default encoder here is a
deterministic hashed bag-of-words projection (unit norm, 512-d, same shape and dtype as USE).  It is only a
stand-in with the same interface: pass any ``text -> np.ndarray[512]`` callable (e.g. a real USE) to the env
wrappers to use real sentence embeddings.
"""
from __future__ import annotations

import hashlib
from functools import lru_cache

import numpy as np

DIM = 512


@lru_cache(maxsize=4096)
def _word_vector(word: str) -> np.ndarray:
    seed = int.from_bytes(hashlib.sha256(word.encode("utf-8")).digest()[:8], "little")
    return np.random.default_rng(seed).standard_normal(DIM).astype(np.float32)


class HashedTextEncoder:
    def __init__(self, dim: int = DIM):
        if dim != DIM:
            raise ValueError("RT-1 context embeddings are 512-d")

    @lru_cache(maxsize=1024)
    def __call__(self, text: str) -> np.ndarray:
        words = text.lower().replace(",", " ").replace(".", " ").split()
        if not words:
            return np.zeros(DIM, np.float32)
        v = np.sum([_word_vector(w) for w in words], axis=0)
        # word order matters a little (bigrams), as it does for a sentence encoder
        v = v + 0.5 * np.sum([_word_vector(a + "_" + b) for a, b in zip(words, words[1:])], axis=0) \
            if len(words) > 1 else v
        return (v / (np.linalg.norm(v) + 1e-12)).astype(np.float32)


def encode_batch(texts) -> np.ndarray:
    """[n] strings -> [n, 512] float32 (the ``--encoder module:function`` form of tools/rlds_convert.py)."""
    enc = HashedTextEncoder()
    return np.stack([enc(t) for t in texts]) if len(texts) else np.zeros((0, DIM), np.float32)
