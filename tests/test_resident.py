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


def test_assign_episodes_random_balanced_deterministic():
    """The training deal: every episode owned exactly once, frame counts balanced, deterministic per seed, not the
    storage-order split (rank 0 must not get the first episodes), different for another seed."""
    rng = np.random.default_rng(0)
    lengths = rng.integers(20, 80, size=400)
    for world in (1, 2, 3, 8):
        parts = R.assign_episodes(lengths, world, seed=5)
        allv = np.concatenate(parts)
        assert len(parts) == world and sorted(allv.tolist()) == list(range(len(lengths)))
        assert all(np.all(np.diff(p) > 0) for p in parts)
        frames = np.array([lengths[p].sum() for p in parts])
        assert frames.max() - frames.min() <= lengths.max()
        again = R.assign_episodes(lengths, world, seed=5)
        assert all(np.array_equal(a, b) for a, b in zip(parts, again))
    p8 = R.assign_episodes(lengths, 8, seed=5)
    assert not np.array_equal(p8[0], np.arange(len(p8[0])))          # not a contiguous prefix
    assert p8[0].max() > len(lengths) * 3 // 4 and p8[0].min() < len(lengths) // 4   # spread over the whole store
    other = R.assign_episodes(lengths, 8, seed=6)
    assert not all(np.array_equal(a, b) for a, b in zip(p8, other))
    with pytest.raises(ValueError):
        R.assign_episodes(lengths[:3], 4)


def test_resident_plan_decode_equals_host_gather(fake):
    """Same windows and crop boxes: the resident gather + decode == host gather + decode_on_device, and the
    per-frame vectors match the shard."""
    res = R.ResidentShard(fake, "cpu")
    ld = R.ResidentBatchLoader(res, 4, 3, crop_factor=0.95, shuffle=True, seed=2, pin=False)
    plan = next(iter(ld))
    assert plan["plan_rows"].shape == (4, 3) and plan["crop_boxes"].shape == (4, 3, 4)
    out = R.decode_resident(res, plan, 30, 24)
    rows = res.global_rows(plan["plan_rows"].numpy())
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
    # the two ranks hold disjoint frame sets whose union is the shard
    sets = [set(R.ResidentShard(fake, "cpu", rank=r, world=2).global_rows(
        np.arange(R.ResidentShard(fake, "cpu", rank=r, world=2).frames.shape[0])).tolist()) for r in range(2)]
    assert not (sets[0] & sets[1]) and len(sets[0] | sets[1]) == int(S.Shard(fake).lengths.sum())
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


def test_distribute_train_auto_falls_back_when_episodes_too_few(fake, monkeypatch):
    """'auto' residency with more ranks than episodes: the host path, not a crash."""
    import types
    import distribute_train as dt
    args = types.SimpleNamespace(data_residency="auto", hbm_data_gb=96.0, batch_size=2, random_crop_factor=0.95,
                                 seed=0)
    ctx = types.SimpleNamespace(device=torch.device("cuda"), world_size=64, rank=3, is_main=False)
    cfg = types.SimpleNamespace(seq_len=2)
    assert dt._resident_train_loader(args, cfg, ctx, fake) is None
    args.data_residency = "hbm"
    with pytest.raises(ValueError):
        dt._resident_train_loader(args, cfg, ctx, fake)


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
