"""In-tree Language-Table board (sim/): instruction language, block sets, env API, rewards, oracle, eval."""
import math

import numpy as np
import pytest
import torch

from pytorch_rt1_for_distributed_training_amd import sim
from pytorch_rt1_for_distributed_training_amd.sim import board, phrases, tasks
from pytorch_rt1_for_distributed_training_amd.sim.board import BlockMode


@pytest.mark.parametrize("mode,count", [(BlockMode.BLOCK_4, 12652), (BlockMode.BLOCK_8, 30264),
                                        (BlockMode.N_CHOOSE_K, 80368)])
def test_instruction_counts_match_reference(mode, count):
    # golden numbers: language_table/environments/rewards/instructions_test.py:28-36
    insts = phrases.generate_all_instructions(mode)
    assert len(insts) == count
    assert all(len(i.encode()) <= board.INSTRUCTION_LENGTH for i in insts)


def test_block_sets_and_n_choose_k_split():
    assert board.block_subsets(BlockMode.BLOCK_8) == [board.FIXED_8]
    train, test = board.n_choose_k_split()
    total = sum(math.comb(16, k) for k in range(4, 11))
    assert len(train) + len(test) == total and len(train) == int(total * 0.9)
    assert not set(train) & set(test)
    assert board.blocks_text(BlockMode.BLOCK_4) == ["red moon", "blue cube", "green star", "yellow pentagon"]


def test_block_synonyms_disambiguate():
    on = board.FIXED_8
    assert phrases.block_synonyms("blue_cube", on) == ["blue cube"]      # blue x2, cube x2
    assert phrases.block_synonyms("red_moon", board.FIXED_4) == ["red block", "moon", "red moon"]


def test_instruction_bytes_roundtrip():
    s = "push the red moon next to the blue cube"
    enc = sim.LanguageTable.encode_instruction(s)
    assert enc.shape == (512,) and enc.dtype == np.int32
    assert sim.LanguageTable.decode_instruction(enc) == s
    assert sim.LanguageTable.decode_instruction(sim.LanguageTable.encode_instruction("")) == ""


def _env(reward="block2block", seed=0, mode=BlockMode.BLOCK_8):
    return sim.LanguageTable(mode, reward_factory=sim.REWARDS[reward], seed=seed)


def test_env_observations_in_space_and_blocks_apart():
    env = _env()
    obs = env.reset()
    assert env.observation_space.contains(obs)
    assert obs["rgb"].shape == (180, 320, 3) and obs["rgb"].dtype == np.uint8
    st = env.compute_state()
    on = [b for b in board.all_block_names() if st[f"block_{b}_mask"][0] == 1.0]
    assert sorted(on) == sorted(board.FIXED_8)
    xy = np.stack([st[f"block_{b}_translation"] for b in on])
    d = np.linalg.norm(xy[:, None] - xy[None], axis=-1) + np.eye(len(on))
    assert d.min() > 2 * sim.world.BLOCK_RADIUS - 1e-4            # settled: no interpenetration
    assert env.instruction_str and sim.LanguageTable.decode_instruction(obs["instruction"]) == env.instruction_str


def test_env_seeded_determinism_and_state_restore_replay():
    a, b = _env(seed=3), _env(seed=3)
    assert a.instruction_str == b.instruction_str
    rng = np.random.RandomState(0)
    acts = rng.uniform(-0.05, 0.05, (12, 2))
    for x in acts[:4]:
        a.step(x)
        b.step(x)
    saved = a.get_state()
    first = [a.step(x)[0]["effector_translation"].copy() for x in acts[4:]]
    first_state = a.compute_state()
    a.set_state(saved)
    second = [a.step(x)[0]["effector_translation"].copy() for x in acts[4:]]
    for p, q in zip(first, second):
        np.testing.assert_array_equal(p, q)
    for k, v in first_state.items():
        if k.endswith("translation"):
            np.testing.assert_array_equal(v, a.compute_state()[k])


def test_effector_clipped_to_workspace_and_pushes_blocks():
    env = sim.LanguageTable(BlockMode.BLOCK_1, seed=0)
    for _ in range(30):
        env.step([0.1, 0.1])
    e = env.compute_state()["effector_target_translation"]
    np.testing.assert_allclose(e, board.WORKSPACE_BOUNDS[1], atol=1e-6)
    w = env.world
    w.place("green_star", (0.40, 0.0))
    w.effector = np.array([0.33, 0.0])
    w.effector_target = np.array([0.33, 0.0])
    for _ in range(3):
        env.step([0.03, 0.0])
    assert w.pos[w.index["green_star"], 0] > 0.40 + 0.02          # pushed along +x


def test_block2block_reward_fires_when_blocks_touch():
    env = _env("block2block", seed=5)
    rc = env._reward_calculator
    info = env._task_info
    assert isinstance(info, tasks.Block2BlockTaskInfo)
    st = env.compute_state()
    assert rc.reward(st) == (0.0, False)
    st[f"block_{info.block1}_translation"] = st[f"block_{info.block2}_translation"] + np.array([0.03, 0.0])
    assert rc.reward(st) == (100.0, True)


def test_delay_reward_steps():
    env = sim.LanguageTable(BlockMode.BLOCK_8, reward_factory=sim.REWARDS["block2block"], seed=2,
                            delay_reward_steps=2)
    rc, info = env._reward_calculator, env._task_info
    st = env.compute_state()
    st[f"block_{info.block1}_translation"] = st[f"block_{info.block2}_translation"]
    assert [rc.reward(st)[1] for _ in range(3)] == [False, False, True]


@pytest.mark.parametrize("reward", ["block2block", "point2block", "block2relativelocation",
                                    "block2absolutelocation", "block2block_relative_location", "block1_to_corner"])
def test_oracle_solves_tasks(reward):
    env = _env(reward, seed=11)
    solved = 0
    for _ in range(6):
        env.reset()
        o = sim.PushOracle(env)
        for _ in range(100):
            _, r, done, _ = env.step(o.action())
            if done:
                solved += 1
                assert r == 100.0
                break
    assert solved >= 5, solved


def test_every_reward_family_resets():
    for name, R in sim.REWARDS.items():
        mode = BlockMode.BLOCK_4 if name == "play" else BlockMode.BLOCK_8
        env = sim.LanguageTable(mode, reward_factory=R, seed=4)
        assert env.instruction_str, name
        assert env._reward_calculator.reward(env.compute_state())[1] in (False, True)


def test_plan_succeeds_restores_state():
    env = _env(seed=8)
    before = env.get_state()
    assert sim.plan_succeeds(env, 100)
    after = env.get_state()
    np.testing.assert_array_equal(before["pos"], after["pos"])
    np.testing.assert_array_equal(before["effector"], after["effector"])


def test_text_encoder_deterministic_unit_norm():
    enc = sim.HashedTextEncoder()
    a = enc("push the red moon to the blue cube")
    assert a.shape == (512,) and abs(float(np.linalg.norm(a)) - 1) < 1e-5
    np.testing.assert_array_equal(a, sim.HashedTextEncoder()("push the red moon to the blue cube"))
    assert float(a @ enc("push the blue cube to the red moon")) < 0.999


def test_rt1_rollout_on_sim_env(tmp_path):
    import pytorch_rt1_for_distributed_training_amd as rt1
    from pytorch_rt1_for_distributed_training_amd.eval import CentralCropResize, RT1Policy, evaluate, make_sim_env
    from pytorch_rt1_for_distributed_training_amd.models import build_rt1
    from pytorch_rt1_for_distributed_training_amd.utils import checkpoint as C
    torch.manual_seed(0)
    cfg = rt1.preset("tiny")
    path = str(tmp_path / "m.ckpt")
    C.save_checkpoint(path, C.build_checkpoint(build_rt1(cfg), epoch=0, global_step=0))
    pol = RT1Policy.from_checkpoint(path, cfg, device="cpu")
    env = make_sim_env("block2block", seed=1)
    res = evaluate(pol, env, episodes=2, max_episode_steps=3, crop=CentralCropResize(cfg.width, cfg.height, 0.95),
                   history_length=cfg.seq_len, video_dir=str(tmp_path / "v"))
    assert res["episodes"] == 2 and 0.0 <= res["success_rate"] <= 1.0
