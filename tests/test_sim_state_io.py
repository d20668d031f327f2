"""Board save / restore files, the asset-driven world and pixel -> table rays.

Reference behaviour: ``language_table/environments/utils/utils_pybullet.py:158-196`` (image ray -> table plane) and
``:376-445`` (gzip-JSON state files with typed records and a version check); ``language_table.py:738-760`` (blocks
loaded from URDFs).  pybullet is not importable, so parity with its numbers is unpinned; these tests pin the
round trips and the consistency between the generated assets and the built-in world.
"""
import gzip
import json

import numpy as np
import pytest

from pytorch_rt1_for_distributed_training_amd.sim import state_io
from pytorch_rt1_for_distributed_training_amd.sim.env import LanguageTable


def _env(seed=0, **kw):
    from pytorch_rt1_for_distributed_training_amd.sim import tasks
    return LanguageTable(seed=seed, reward_factory=tasks.BlockToBlockReward, **kw)


def test_state_file_round_trip_replays_bitwise(tmp_path):
    env = _env(seed=5)
    rng = np.random.RandomState(0)
    start = env.get_state()
    acts = [rng.uniform(-0.05, 0.05, 2) for _ in range(6)]
    ref = [env.step(a) for a in acts]
    ref_obs = [r[0] for r in ref]
    path = str(tmp_path / "board.json.gz")
    state_io.write_state(path, start, task=env.instruction_str, actions=acts)
    data = state_io.read_state(path)
    assert data["task"] == env.instruction_str and len(data["actions"]) == 6
    other = _env(seed=99)                                   # a different board, overwritten by the file
    obs = state_io.replay(other, data)
    for a, b in zip(obs, ref_obs):
        for k in ("effector_translation", "effector_target_translation", "instruction", "rgb"):
            np.testing.assert_array_equal(a[k], b[k])
    assert type(other.get_state()["task_info"]) is type(start["task_info"])
    # the reward calculator's task and the env rng come back too: rewards replay, and so does the next reset
    other.set_state(data["state"])
    assert [other.step(a)[1:3] for a in data["actions"]] == [r[1:3] for r in ref]
    env.set_state(start)
    for _ in acts:
        env.step(np.zeros(2))
    other.set_state(data["state"])
    np.testing.assert_array_equal(env.reset()["rgb"], other.reset()["rgb"])


def test_typed_records_and_version_check(tmp_path):
    env = _env(seed=2)
    s = env.get_state()
    back = state_io.deserialize(json.loads(json.dumps(state_io.serialize(s))))
    for k in ("pos", "yaw", "active", "effector", "effector_target"):
        assert back[k].dtype == s[k].dtype and back[k].shape == s[k].shape
        np.testing.assert_array_equal(back[k], s[k])
    np.testing.assert_array_equal(back["robot"]["q"], s["robot"]["q"])
    assert back["task_info"].instruction == s["task_info"].instruction
    path = str(tmp_path / "old.json.gz")
    with gzip.open(path, "wb") as fh:
        fh.write(json.dumps({"state": {}, "state_version": 0}).encode())
    with pytest.raises(ValueError, match="incompatible"):
        state_io.read_state(path)
    with pytest.raises(ValueError):
        state_io.serialize({"x": object()})


def test_world_from_generated_assets_matches_builtin(tmp_path):
    a = LanguageTable(seed=3, asset_root=str(tmp_path / "assets"), use_arm=False)
    b = LanguageTable(seed=3, use_arm=False)
    assert set(a.world.bodies) == set(a.world.names)
    np.testing.assert_allclose(a.world.radius, b.world.radius, atol=2e-6)   # OBJ vertices carry 6 decimals
    np.testing.assert_array_equal(a.world.color, b.world.color)
    np.testing.assert_array_equal(a.render(), b.render())


def test_assets_drive_geometry_and_colour(tmp_path):
    from pytorch_rt1_for_distributed_training_amd.sim import assets
    paths = assets.write_assets(str(tmp_path))
    # scale the red moon's mesh up 2x and repaint it: the world follows the files
    txt = open(paths["red_moon"]).read().replace('scale="1.0 1.0 1.0"', 'scale="2.0 2.0 2.0"')
    txt = txt.replace(" ".join(f"{c:g}" for c in assets._rgba("red")), "0 1 0 1")
    open(paths["red_moon"], "w").write(txt)
    from pytorch_rt1_for_distributed_training_amd.sim.world import PlanarWorld, BLOCK_RADIUS
    w = PlanarWorld().load_assets(paths)
    i = w.index["red_moon"]
    assert abs(w.radius[i] - 2 * BLOCK_RADIUS) < 1e-5
    assert tuple(w.color[i]) == (0, 255, 0)


def test_pixel_to_table_inverts_projection():
    from pytorch_rt1_for_distributed_training_amd.sim.world import Camera
    cam = Camera()
    for x, y in [(0.3, 0.0), (0.45, -0.2), (0.2, 0.25)]:
        r, c = cam.project([x, y, 0.0])[0]
        np.testing.assert_allclose(cam.pixel_to_table(r - 0.5, c - 0.5), [x, y], atol=1e-9)
    xy = cam.table_points()
    np.testing.assert_allclose(cam.pixel_to_table(17, 211), xy[17, 211], atol=1e-12)
