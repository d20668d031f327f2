#!/usr/bin/env python3
"""Language-Table RLDS -> episode files (reference D4, ``rlds_np_convert.py``).

Reads ``language_table_blocktoblock_sim`` (or any RLDS builder directory) with tensorflow_datasets,
flattens every step (observation keys merged into the step, as the reference's ``:13-25``), replaces
the instruction bytes by a 512-d sentence embedding, and writes one ``episode_{id}.npz`` per episode
in this framework's pickle-free format (``data/episodes.py``).  Split as the reference (``:35-37``):
the first ``--train`` episodes -> train/, the next ``--val`` -> val/, the next ``--test`` -> test/.

TensorFlow / tensorflow_datasets and the Universal Sentence Encoder are optional dependencies that are
NOT part of the training image: the import is deferred and fails with a clear message.  The embedding
can also come from any callable ``--encoder module:function`` mapping a list of strings to (n, 512).

  python tools/rlds_convert.py --builder_dir /data/language_table_blocktoblock_sim/0.0.1 --out /data/lt
"""
from __future__ import annotations

import argparse
import importlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_rt1_for_distributed_training_amd.data.episodes import write_episode  # noqa: E402


def decode_instruction(raw) -> str:
    """Language-Table stores the instruction as a fixed-length int32 array of UTF-8 bytes, 0-padded."""
    arr = np.asarray(raw).reshape(-1)
    arr = arr[arr != 0].astype(np.uint8)
    return bytes(arr.tolist()).decode("utf-8", errors="ignore")


def flatten_step(step: dict) -> dict:
    """Merge ``observation`` into the step (reference rlds_np_convert.py:13-25)."""
    out = {k: v for k, v in step.items() if k != "observation"}
    out.update(step.get("observation", {}))
    return out


def episode_arrays(steps, encode):
    steps = [flatten_step(s) for s in steps]
    texts = [decode_instruction(s["instruction"]) for s in steps]
    emb = np.asarray(encode(texts), np.float32).reshape(len(steps), -1)
    return dict(rgb=np.stack([np.asarray(s["rgb"], np.uint8) for s in steps]), instruction=emb,
                action=np.stack([np.asarray(s["action"], np.float32)[:2] for s in steps]),
                is_terminal=np.array([bool(s["is_terminal"]) for s in steps]),
                is_first=np.array([bool(s.get("is_first", i == 0)) for i, s in enumerate(steps)]))


def load_encoder(spec: str):
    if spec == "use":
        try:
            import tensorflow_hub as hub  # noqa: F401
        except ImportError as e:
            raise SystemExit("the Universal Sentence Encoder needs tensorflow_hub (not installed); "
                             "pass --encoder module:function instead") from e
        model = hub.load("https://tfhub.dev/google/universal-sentence-encoder-large/5")
        return lambda texts: model(texts).numpy()
    mod, fn = spec.split(":")
    return getattr(importlib.import_module(mod), fn)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--builder_dir", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--train", type=int, default=7800)
    ap.add_argument("--val", type=int, default=100)
    ap.add_argument("--test", type=int, default=100)
    ap.add_argument("--encoder", default="use", help="'use' (tf-hub USE large/5) or module:function")
    a = ap.parse_args(argv)
    try:
        import tensorflow_datasets as tfds
    except ImportError as e:
        raise SystemExit("tensorflow_datasets is required to read RLDS (not installed in the training image)") from e
    encode = load_encoder(a.encoder)
    ds = tfds.builder_from_directory(a.builder_dir).as_dataset(split="train")
    splits = [("train", a.train), ("val", a.val), ("test", a.test)]
    si, count = 0, 0
    for ep_id, episode in enumerate(tfds.as_numpy(ds)):
        while si < len(splits) and count >= splits[si][1]:
            si, count = si + 1, 0
        if si == len(splits):
            break
        name, _ = splits[si]
        os.makedirs(os.path.join(a.out, name), exist_ok=True)
        arr = episode_arrays(list(episode["steps"]), encode)
        write_episode(os.path.join(a.out, name, f"episode_{count}.npz"), **arr)
        count += 1
    print("done")


if __name__ == "__main__":
    main()
