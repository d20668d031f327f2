"""HBM-resident input path (data/resident.py) against the host-gather shard path (CPU device here; the GPU kernel
is compared with Pillow in tests/test_imgproc_gpu.py)."""
import os

import numpy as np
import pytest
import torch

from pytorch_rt1_for_distributed_training_amd.data import episodes as E
from pytorch_rt1_for_distributed_training_amd.data import resident as R
from pytorch_rt1_for_distributed_training_amd.data import shards as S


@pytest.fixture()
def fake(tmp_path):
    src = tmp_path / "npz"
    ids = E.make_fake_episodes(str(src), 7, steps=6, height=40, width=56, seed=3)
    dst = tmp_path / "shard"
    S.pack_shard(str(src), ids, str(dst))
    return str(dst)


def test_partition_episodes_contiguous_balanced():
    lengths = np.array([40, 10, 10, 40, 30, 30, 40, 10])
    for world in (1, 2, 3, 4, 8):
        parts = R.partition_episodes(lengths, world)
        assert len(parts) == world and parts[0][0] == 0 and parts[-1][1] == len(lengths)
        assert all(a < b for a, b in parts) and all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))
    frames = [int(lengths[a:b].sum()) for a, b in R.partition_episodes(lengths, 2)]
    assert frames == [100, 110]
    with pytest.raises(ValueError):
        R.partition_episodes(lengths, 9)  # 8 episodes


def test_resident_plan_decode_equals_host_gather(fake):
    """Same windows and crop boxes: the resident gather + decode == host gather + decode_on_device, and the
    per-frame vectors match the shard."""
    res = R.ResidentShard(fake, "cpu")
    ld = R.ResidentBatchLoader(res, 4, 3, crop_factor=0.95, shuffle=True, seed=2, pin=False)
    plan = next(iter(ld))
    assert plan["plan_rows"].shape == (4, 3) and plan["crop_boxes"].shape == (4, 3, 4)
    out = R.decode_resident(res, plan, 30, 24)
    rows = plan["plan_rows"].numpy() + res.f_lo
    host = {"train_observation": {"raw_frames": torch.from_numpy(np.asarray(res.shard.frames[rows])),
                                  "crop_boxes": plan["crop_boxes"]}}
    ref = S.decode_on_device(host, 30, 24)["train_observation"]["image"]
    assert torch.equal(out["train_observation"]["image"], ref)
    torch.testing.assert_close(out["train_observation"]["natural_language_embedding"],
                               torch.from_numpy(res.shard.instruction[rows]))
    torch.testing.assert_close(out["action_label"]["action"], torch.from_numpy(res.shard.action[rows]))
    assert torch.equal(out["action_label"]["terminate_episode"],
                       torch.from_numpy(res.shard.is_terminal[rows].astype(np.int64)))


def test_resident_ranks_cover_dataset_once_per_epoch(fake):
    seen, lens = [], []
    for r in range(2):
        res = R.ResidentShard(fake, "cpu", rank=r, world=2)
        ld = R.ResidentBatchLoader(res, 2, 2, shuffle=True, seed=0, pin=False)
        lens.append(len(ld))
        seen.append(set(res.window_ids.tolist()))
        # frames of the windows a rank plans are inside its resident range
        for plan in ld:
            rows = plan["plan_rows"].numpy()
            assert rows.min() >= 0 and rows.max() < res.frames.shape[0]
    assert lens[0] == lens[1] > 0                    # same step count on every rank
    assert not (seen[0] & seen[1]) and len(seen[0] | seen[1]) == len(S.Shard(fake))
    # a fresh order per epoch
    res = R.ResidentShard(fake, "cpu")
    ld = R.ResidentBatchLoader(res, 2, 2, shuffle=True, seed=0, pin=False)
    e0 = [p["plan_rows"].clone() for p in ld]
    ld.set_epoch(1)
    e1 = [p["plan_rows"].clone() for p in ld]
    assert not all(torch.equal(a, b) for a, b in zip(e0, e1))


def test_resident_budget_refuses(fake):
    with pytest.raises(MemoryError):
        R.ResidentShard(fake, "cpu", max_gb=1e-6)


def test_distribute_train_resident_cpu(fake, tmp_path):
    """The training entrypoint on the resident path (CPU, tiny model)."""
    root = tmp_path / "ds"
    root.mkdir()
    for split in ("train", "test", "val"):
        os.symlink(fake, root / split)
    import distribute_train as dt
    rc = dt.main(["--device", "cpu", "--mode", "train", "--dataset_dir", str(root), "--height", "64", "--width",
                  "64", "--seq_len", "2", "--num_layers", "2", "--batch_size", "2", "--max_epochs", "1",
                  "--limit_train_batches", "2", "--limit_val_batches", "1", "--dtype", "fp32", "--num_workers", "2",
                  "--data_residency", "hbm", "--log_dir", str(tmp_path / "logs"), "--ckpt_dir", str(tmp_path / "ck"),
                  "--log_every_n_steps", "1"])
    assert rc == 0
    assert os.path.exists(tmp_path / "ck" / "exp_rt1" / "last.ckpt")
