#!/usr/bin/env python3
"""Iterate an episode dataset the way training does (the role of the reference's
``language_table/examples/dataset_example.py`` and ``load_np_dataset.py``'s inspector).

With ``--data_dir`` it reads converted episodes (``tools/rlds_convert.py`` / ``data.episodes``); without it, it
first writes a few tiny fake episodes in the same on-disk format.

  python examples/dataset_example.py [--data_dir /data/lt] [--window 6] [--batch 4]
"""
from __future__ import annotations

import argparse
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_rt1_for_distributed_training_amd.data.episodes import (EpisodeWindowDataset, collate_fn,  # noqa: E402
                                                                     make_fake_episodes)


def _shapes(tree, prefix=""):
    for k, v in tree.items():
        if isinstance(v, dict):
            _shapes(v, prefix + k + ".")
        else:
            print(f"  {prefix}{k}: {tuple(v.shape)} {v.dtype}")


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--data_dir", default="")
    ap.add_argument("--episodes", type=int, default=3)
    ap.add_argument("--window", type=int, default=6)
    ap.add_argument("--batch", type=int, default=4)
    a = ap.parse_args(argv)
    data_dir = a.data_dir
    if data_dir:
        ids = sorted(int(f.split("_")[1].split(".")[0]) for f in os.listdir(data_dir) if f.startswith("episode_"))
    else:
        data_dir = tempfile.mkdtemp(prefix="rt1_episodes_")
        ids = make_fake_episodes(data_dir, a.episodes)
        print("wrote fake episodes to", data_dir)
    ds = EpisodeWindowDataset(data_dir, ids, a.window)
    print(f"{len(ids)} episodes -> {len(ds)} windows of {a.window} steps")
    loader = torch.utils.data.DataLoader(ds, batch_size=a.batch, shuffle=True, collate_fn=collate_fn)
    batch = next(iter(loader))
    print("batch:")
    _shapes(batch)
    return 0


if __name__ == "__main__":
    sys.exit(main())
