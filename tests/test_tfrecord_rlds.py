"""TensorFlow-free TFRecord / tf.train.Example codec and the native RLDS reader.

Reference: ``rlds_np_convert.py:1-40`` reads the Language-Table RLDS release through tensorflow_datasets.  Neither
TF nor the dataset is available here, so the fixtures are synthetic tfds-layout shards written by this codec: the
CRC-32C is pinned to the published check value, the Example wire format to hand-assembled bytes, and the
converter end to end on a two-shard builder directory with PNG frames.  Parity with real tfds shards is unpinned.
"""
import io
import json
import os
import struct
import sys

import numpy as np
import pytest

from pytorch_rt1_for_distributed_training_amd.data import tfrecord as tfr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_crc32c_check_value_and_mask():
    assert tfr.crc32c(b"123456789") == 0xE3069283                     # CRC-32C catalogue check value
    c = tfr.crc32c(b"abc")
    assert tfr.masked_crc(b"abc") == ((((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF)


def test_records_round_trip_and_corruption(tmp_path):
    p = str(tmp_path / "x.tfrecord")
    recs = [b"", b"a", os.urandom(1000)]
    tfr.write_records(p, recs)
    assert list(tfr.read_records(p, verify_data=True)) == recs
    raw = bytearray(open(p, "rb").read())
    raw[-3] ^= 0xFF                                                   # flip a byte of the last data CRC
    open(p, "wb").write(bytes(raw))
    assert len(list(tfr.read_records(p))) == 3                        # length CRCs still fine
    with pytest.raises(ValueError, match="corrupt record data"):
        list(tfr.read_records(p, verify_data=True))
    raw[8] ^= 0xFF                                                    # first length CRC
    open(p, "wb").write(bytes(raw))
    with pytest.raises(ValueError, match="corrupt record length"):
        list(tfr.read_records(p))


def test_example_wire_format():
    # Example{features{feature{key:"a" value{int64_list{value:[1, -2]}}}}} assembled by hand (packed int64)
    neg = tfr._enc_varint(-2)
    assert len(neg) == 10
    int_list = b"\x0a" + bytes([1 + len(neg)]) + b"\x01" + neg
    feat = b"\x1a" + bytes([len(int_list)]) + int_list
    entry = b"\x0a\x01a" + b"\x12" + bytes([len(feat)]) + feat
    features = b"\x0a" + bytes([len(entry)]) + entry
    ex = b"\x0a" + bytes([len(features)]) + features
    out = tfr.parse_example(ex)
    np.testing.assert_array_equal(out["a"], [1, -2])
    assert tfr.encode_example({"a": np.array([1, -2])}) == ex
    # unpacked floats (wire type 5) decode too
    fl = b"\x0d" + struct.pack("<f", 1.5) + b"\x0d" + struct.pack("<f", -3.0)
    feat = b"\x12" + bytes([len(fl)]) + fl
    entry = b"\x0a\x01f" + b"\x12" + bytes([len(feat)]) + feat
    features = b"\x0a" + bytes([len(entry)]) + entry
    np.testing.assert_array_equal(tfr.parse_example(b"\x0a" + bytes([len(features)]) + features)["f"], [1.5, -3.0])
    rt = tfr.parse_example(tfr.encode_example({"b": [b"x", b"yz"], "f": np.array([0.25], np.float32)}))
    assert rt["b"] == [b"x", b"yz"] and rt["f"].dtype == np.float32


def _png(img):
    from PIL import Image
    buf = io.BytesIO()
    Image.fromarray(img).save(buf, format="PNG")
    return buf.getvalue()


def _write_builder(d, n_eps=5, T=4, H=18, W=32, shards=2):
    rng = np.random.RandomState(0)
    eps = []
    for e in range(n_eps):
        rgb = rng.randint(0, 256, (T, H, W, 3)).astype(np.uint8)
        instr = np.zeros((T, 512), np.int64)
        text = f"push the red moon {e}".encode()
        instr[:, :len(text)] = list(text)
        act = rng.uniform(-0.1, 0.1, (T, 2)).astype(np.float32)
        term = np.zeros(T, np.int64)
        term[-1] = 1
        eps.append((rgb, instr, act, term, text.decode()))
    per = (n_eps + shards - 1) // shards
    for s in range(shards):
        recs = []
        for rgb, instr, act, term, _ in eps[s * per:(s + 1) * per]:
            first = np.zeros(T, np.int64)
            first[0] = 1
            recs.append(tfr.encode_example({
                "steps/observation/rgb": [_png(f) for f in rgb], "steps/observation/instruction": instr,
                "steps/action": act, "steps/is_terminal": term, "steps/is_first": first,
                "steps/is_last": term, "steps/reward": np.zeros(T, np.float32)}))
        tfr.write_records(os.path.join(d, f"language_table-train.tfrecord-{s:05d}-of-{shards:05d}"), recs)
    feats = {"featuresDict": {"features": {"steps": {"sequence": {"feature": {"featuresDict": {"features": {
        "action": {"tensor": {"shape": {"dimensions": ["2"]}, "dtype": "float32"}}}}}}}}}}
    json.dump(feats, open(os.path.join(d, "features.json"), "w"))
    return eps


def test_native_rlds_reader(tmp_path):
    eps = _write_builder(str(tmp_path))
    got = list(tfr.read_rlds_episodes(str(tmp_path)))
    assert len(got) == len(eps)
    for (rgb, instr, act, term, _), g in zip(eps, got):
        st = g["steps"]
        np.testing.assert_array_equal(st["observation"]["rgb"], rgb)
        np.testing.assert_array_equal(st["observation"]["instruction"], instr)
        np.testing.assert_array_equal(st["action"], act)
        assert st["is_terminal"].dtype == bool and st["is_terminal"].tolist() == term.astype(bool).tolist()


def test_rlds_convert_native_end_to_end(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import rlds_convert
    src, dst = tmp_path / "rlds", tmp_path / "out"
    src.mkdir()
    eps = _write_builder(str(src))
    rlds_convert.main(["--builder_dir", str(src), "--out", str(dst), "--train", "3", "--val", "1", "--test", "1",
                       "--encoder", "pytorch_rt1_for_distributed_training_amd.sim.text:encode_batch"])
    assert sorted(os.listdir(dst / "train")) == ["episode_0.npz", "episode_1.npz", "episode_2.npz"]
    z = np.load(dst / "test" / "episode_0.npz")                       # allow_pickle=False (default)
    rgb, _, act, term, text = eps[4]
    np.testing.assert_array_equal(z["rgb"], rgb)
    np.testing.assert_array_equal(z["action"], act)
    assert z["is_terminal"].tolist() == term.astype(bool).tolist() and z["is_first"][0]
    from pytorch_rt1_for_distributed_training_amd.sim.text import HashedTextEncoder
    np.testing.assert_allclose(z["instruction"][0], HashedTextEncoder()(text), rtol=1e-6)


def test_train_lava_from_rlds_shards(tmp_path):
    """J3: the LAVA trainer reads RLDS shards directly (reference input_pipeline_rlds.py), episodes dealt by rank."""
    from pytorch_rt1_for_distributed_training_amd.data import sim_demos
    src = tmp_path / "rlds"
    src.mkdir()
    eps = _write_builder(str(src), n_eps=3, T=3, H=36, W=64)
    got = sim_demos.rlds_episodes(str(src), rank=1, world_size=2)
    assert len(got) == 1
    np.testing.assert_array_equal(got[0]["rgb"], eps[1][0])
    np.testing.assert_array_equal(got[0]["action"], eps[1][2])
    assert got[0]["instruction_embedding"].shape == (3, 512)
    sys.path.insert(0, ROOT)
    import train_lava
    res = train_lava.main(["--rlds", str(src), "--steps", "2", "--batch_size", "4", "--sequence_length", "2",
                           "--d_model", "32", "--log_every", "1", "--device", "cpu",
                           "--ckpt", str(tmp_path / "ck" / "last.pt")])
    assert res["windows"] == 9 and np.isfinite(res["final_loss"])


def test_inspect_dataset_rlds_mode(tmp_path, capsys):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import inspect_dataset
    _write_builder(str(tmp_path))
    ep = inspect_dataset.main(["--rlds", str(tmp_path)])
    out = capsys.readouterr().out
    assert "2 shards, 5 episodes (3, 2)" in out and "episode.steps.observation.rgb: shape=(4, 18, 32, 3)" in out
    assert ep["steps"]["action"].shape == (4, 2)


def test_jpeg_frames_decode():
    from PIL import Image
    img = np.full((8, 16, 3), 200, np.uint8)
    buf = io.BytesIO()
    Image.fromarray(img).save(buf, format="JPEG", quality=95)
    ex = tfr.parse_example(tfr.encode_example({"steps/observation/rgb": [buf.getvalue()] * 2,
                                               "steps/is_first": np.array([1, 0]),
                                               "steps/language": [b"push", b"push"]}))
    ep = tfr.episode_from_example(ex)
    assert ep["steps"]["observation"]["rgb"].shape == (2, 8, 16, 3)
    assert np.abs(ep["steps"]["observation"]["rgb"].astype(int) - 200).max() <= 2
    assert ep["steps"]["language"] == [b"push", b"push"]                # non-image bytes stay bytes


def test_rlds_rank_selection_before_decode(tmp_path, monkeypatch):
    """A rank parses / decodes only its own records (i % world == rank); the others cost a framing read only.  A limit
    below the world size, or a rank left without episodes, is an error rather than an empty dataset."""
    from pytorch_rt1_for_distributed_training_amd.data import sim_demos
    _write_builder(str(tmp_path))                                    # 5 episodes over 2 shards
    parsed = []
    real = tfr.parse_example
    monkeypatch.setattr(tfr, "parse_example", lambda rec: parsed.append(1) or real(rec))
    got = sim_demos.rlds_episodes(str(tmp_path), rank=0, world_size=4)
    assert len(got) == 2 and len(parsed) == 2                        # records 0 and 4 of 5
    parsed.clear()
    got = sim_demos.rlds_episodes(str(tmp_path), rank=0, world_size=2, limit=3)
    assert len(got) == 2 and len(parsed) == 2                        # records 0 and 2 of the first 3
    with pytest.raises(ValueError):
        sim_demos.rlds_episodes(str(tmp_path), rank=0, world_size=4, limit=2)
    with pytest.raises(ValueError):
        sim_demos.rlds_episodes(str(tmp_path), rank=5, world_size=6)
