"""Packed shards + whole-batch loader (data/shards.py) against the per-episode dataset semantics."""
import os

import numpy as np
import pytest
import torch

from pytorch_rt1_for_distributed_training_amd.data import episodes as E
from pytorch_rt1_for_distributed_training_amd.data import shards as S


@pytest.fixture()
def fake(tmp_path):
    src = tmp_path / "npz"
    ids = E.make_fake_episodes(str(src), 5, steps=7, height=40, width=56, seed=1)
    dst = tmp_path / "shard"
    n = S.pack_shard(str(src), ids, str(dst))
    assert n == 35 and S.is_shard(str(dst))
    return str(src), ids, str(dst)


def test_shard_windows_match_episode_dataset(fake):
    src, ids, dst = fake
    T = 4
    ref = E.EpisodeWindowDataset(src, ids, T, transform=None)
    sh = S.Shard(dst)
    assert len(sh) == len(ref)
    for w in [0, 3, 6, 7, 20, 34]:
        rows = sh.frame_index(np.array([w]), T)[0]
        r = ref[w]
        img = torch.from_numpy(np.asarray(sh.frames[rows])).permute(0, 3, 1, 2).float() / 255.0
        torch.testing.assert_close(img, r["train_observation"]["image"])
        torch.testing.assert_close(torch.from_numpy(sh.instruction[rows]),
                                   r["train_observation"]["natural_language_embedding"])
        torch.testing.assert_close(torch.from_numpy(sh.action[rows]), r["action_label"]["action"])
        assert torch.equal(torch.from_numpy(sh.is_terminal[rows].astype(np.int64)),
                           r["action_label"]["terminate_episode"])


def test_loader_decode_matches_pil_transform(fake):
    """Boxes drawn by the loader + decode_on_device (Pillow on CPU) == DecodeAndRandomResizedCrop on that box."""
    _, _, dst = fake
    ld = S.ShardBatchLoader(dst, 3, 2, crop_factor=0.95, shuffle=True, seed=4, threads=2, pin=False)
    batch = next(iter(ld))
    obs = batch["train_observation"]
    assert obs["raw_frames"].shape == (3, 2, 40, 56, 3) and obs["crop_boxes"].dtype == torch.int32
    boxes = obs["crop_boxes"].reshape(-1, 4).numpy()
    assert (boxes[:, 0] >= 0).all() and (boxes[:, 2] <= 56).all() and (boxes[:, 3] <= 40).all()
    assert set(boxes[:, 2] - boxes[:, 0]) == {round(56 * 0.95)} and set(boxes[:, 3] - boxes[:, 1]) == {38}
    out = S.decode_on_device(batch, 30, 24)
    img = out["train_observation"]["image"]
    assert img.shape == (3, 2, 3, 30, 24) and img.dtype == torch.uint8
    from PIL import Image
    raw = obs["raw_frames"].reshape(-1, 40, 56, 3).numpy()
    for i in range(raw.shape[0]):
        ref = np.asarray(Image.fromarray(raw[i]).crop(tuple(int(v) for v in boxes[i])).resize((24, 30),
                                                                                             Image.BILINEAR))
        assert np.array_equal(img.reshape(-1, 3, 30, 24)[i].permute(1, 2, 0).numpy(), ref)


def test_loader_epochs_and_rank_partition(fake):
    _, _, dst = fake
    seen = []
    for r in range(2):
        ld = S.ShardBatchLoader(dst, 4, 2, shuffle=True, rank=r, world=2, seed=0, threads=1, pin=False)
        ld.set_epoch(3)
        assert len(ld) == (35 // 2) // 4
        idx = ld._indices()
        seen.append(set(idx.tolist()))
        assert len(list(iter(ld))) == len(ld)
    assert not (seen[0] & seen[1])
    a = S.ShardBatchLoader(dst, 4, 2, shuffle=True, seed=0, pin=False)
    a.set_epoch(0)
    i0 = a._indices().copy()
    a.set_epoch(1)
    assert not np.array_equal(i0, a._indices())


def test_distribute_train_on_shards_cpu(fake, tmp_path):
    """The training entrypoint consumes a packed shard end to end (CPU, tiny model, 1 epoch, 2 batches)."""
    _, ids, dst = fake
    root = tmp_path / "ds"
    for split in ("train", "test", "val"):
        os.symlink(dst, root / split) if root.exists() else (root.mkdir(), os.symlink(dst, root / split))
    import distribute_train as dt
    rc = dt.main(["--device", "cpu", "--mode", "train", "--dataset_dir", str(root), "--height", "64", "--width",
                  "64", "--seq_len", "2", "--num_layers", "2", "--batch_size", "2", "--max_epochs", "1",
                  "--limit_train_batches", "2", "--limit_val_batches", "1", "--dtype", "fp32", "--num_workers", "2",
                  "--log_dir", str(tmp_path / "logs"), "--ckpt_dir", str(tmp_path / "ck"), "--log_every_n_steps",
                  "1"])
    assert rc == 0
    assert os.path.exists(tmp_path / "ck" / "exp_rt1" / "last.ckpt")


def test_gpu_crop_tap_budget():
    """The GPU resize keeps <= 16 Pillow taps per axis: frames that would need more take the Pillow path."""
    from pytorch_rt1_for_distributed_training_amd.data.shards import gpu_crop_supported
    assert gpu_crop_supported(360, 640, 300, 300)           # Language-Table frames -> 300x300
    assert gpu_crop_supported(256, 456, 256, 456)
    assert gpu_crop_supported(7 * 64, 7 * 64, 64, 64)       # 7x: ceil(14) + 1 = 15 taps
    assert not gpu_crop_supported(8 * 64, 64, 64, 64)       # 8x: 17 taps
    assert not gpu_crop_supported(64, 1000, 64, 100)
