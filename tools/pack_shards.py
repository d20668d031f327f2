#!/usr/bin/env python3
"""Pack per-episode ``.npz`` splits into memory-mapped shards for the GPU input path (``data/shards.py``).

  python tools/pack_shards.py --src data/lt_npz --dst data/lt_shard --splits train test val
Each ``<src>/<split>/episode_{id}.npz`` set becomes ``<dst>/<split>/{frames.u8, meta.npz}``.
Also ``--fake N --steps S --hw 360 640`` writes N random episodes per split first (throughput rehearsals).
"""
from __future__ import annotations

import argparse
import glob
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_rt1_for_distributed_training_amd.data.episodes import make_fake_episodes  # noqa: E402
from pytorch_rt1_for_distributed_training_amd.data.shards import pack_shard  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", required=True)
    ap.add_argument("--dst", required=True)
    ap.add_argument("--splits", nargs="+", default=["train", "test", "val"])
    ap.add_argument("--fake", type=int, default=0, help="first write this many random episodes per split")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--hw", type=int, nargs=2, default=[360, 640])
    a = ap.parse_args()
    for i, split in enumerate(a.splits):
        src = os.path.join(a.src, split)
        if a.fake:
            make_fake_episodes(src, a.fake if split == "train" else max(2, a.fake // 10), steps=a.steps,
                               height=a.hw[0], width=a.hw[1], seed=i)
        ids = sorted(int(re.search(r"episode_(\d+)\.npz$", p).group(1))
                     for p in glob.glob(os.path.join(src, "episode_*.npz")))
        n = pack_shard(src, ids, os.path.join(a.dst, split))
        print(f"{split}: {len(ids)} episodes, {n} frames -> {os.path.join(a.dst, split)}", flush=True)


if __name__ == "__main__":
    main()
