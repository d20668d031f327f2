#!/usr/bin/env python3
"""Language-Table RLDS -> episode files (reference D4, ``rlds_np_convert.py``).

Reads ``language_table_blocktoblock_sim`` (or any RLDS builder directory) with tensorflow_datasets,
flattens every step (observation keys merged into the step, as the reference's ``:13-25``), replaces
the instruction bytes by a 512-d sentence embedding, and writes one ``episode_{id}.npz`` per episode
in this framework's pickle-free format (``data/episodes.py``).  Split as the reference (``:35-37``):
the first ``--train`` episodes -> train/, the next ``--val`` -> val/, the next ``--test`` -> test/.

The shards are read without TensorFlow by default (``--reader native``: ``data/tfrecord.py`` decodes the
TFRecord framing, the ``tf.train.Example`` protobufs and the per-step PNG / JPEG images itself);
``--reader tfds`` uses tensorflow_datasets when it is installed.  The Universal Sentence Encoder is an optional
dependency that is NOT part of the training image: the embedding can come from any callable
``--encoder module:function`` mapping a list of strings to (n, 512) (e.g. the in-tree hashed stand-in,
``pytorch_rt1_for_distributed_training_amd.sim.text:encode_batch``).

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


def steps_list(steps) -> list:
    """tfds yields ``steps`` as a sequence of step dicts; the native reader as one dict of [T, ...] arrays."""
    if not isinstance(steps, dict):
        return list(steps)

    def lengths(d):
        for v in d.values():
            if isinstance(v, dict):
                yield from lengths(v)
            else:
                yield len(v)

    def pick(d, t):
        return {k: pick(v, t) if isinstance(v, dict) else v[t] for k, v in d.items()}
    n = min(lengths(steps))
    return [pick(steps, t) for t in range(n)]


def iter_episodes(builder_dir: str, reader: str = "native"):
    if reader == "native":
        from pytorch_rt1_for_distributed_training_amd.data.tfrecord import read_rlds_episodes
        yield from read_rlds_episodes(builder_dir, "train")
        return
    try:
        import tensorflow_datasets as tfds
    except ImportError as e:
        raise SystemExit("tensorflow_datasets is not installed: use --reader native") from e
    yield from tfds.as_numpy(tfds.builder_from_directory(builder_dir).as_dataset(split="train"))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--builder_dir", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--train", type=int, default=7800)
    ap.add_argument("--val", type=int, default=100)
    ap.add_argument("--test", type=int, default=100)
    ap.add_argument("--encoder", default="use", help="'use' (tf-hub USE large/5) or module:function")
    ap.add_argument("--reader", default="native", choices=("native", "tfds"),
                    help="native: TensorFlow-free TFRecord / Example decoder (data/tfrecord.py)")
    a = ap.parse_args(argv)
    encode = load_encoder(a.encoder)
    splits = [("train", a.train), ("val", a.val), ("test", a.test)]
    si, count = 0, 0
    for ep_id, episode in enumerate(iter_episodes(a.builder_dir, a.reader)):
        while si < len(splits) and count >= splits[si][1]:
            si, count = si + 1, 0
        if si == len(splits):
            break
        name, _ = splits[si]
        os.makedirs(os.path.join(a.out, name), exist_ok=True)
        arr = episode_arrays(steps_list(episode["steps"]), encode)
        write_episode(os.path.join(a.out, name, f"episode_{count}.npz"), **arr)
        count += 1
    print("done")


if __name__ == "__main__":
    main()
