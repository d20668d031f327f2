"""Checkpoint format, logging, data pipeline, trainer loop + resume (CPU)."""
import csv
import glob
import os

import numpy as np
import torch

import pytorch_rt1_for_distributed_training_amd as rt1
from pytorch_rt1_for_distributed_training_amd import data as D
from pytorch_rt1_for_distributed_training_amd.engine.step import TrainEngine
from pytorch_rt1_for_distributed_training_amd.engine.trainer import Trainer
from pytorch_rt1_for_distributed_training_amd.models import build_rt1
from pytorch_rt1_for_distributed_training_amd.utils import checkpoint as C
from pytorch_rt1_for_distributed_training_amd.utils.logging import CSVLogger, MultiLogger, TensorBoardLogger
from pytorch_rt1_for_distributed_training_amd.utils.tfevents import read_scalars, crc32c


def test_crc32c_known_vector():
    assert crc32c(b"123456789") == 0xE3069283


def test_lightning_checkpoint_layout_and_roundtrip(tmp_path):
    torch.manual_seed(0)
    cfg = rt1.preset("tiny")
    m = build_rt1(cfg)
    eng = TrainEngine(m, cfg, order_probe=False)
    batch = D.make_batch(2, cfg.seq_len, cfg.height, cfg.width, uint8=True)
    eng.train_step(batch)
    ck = C.build_checkpoint(m, eng.optimizer, eng.scheduler, epoch=3, global_step=7)
    for k in ("epoch", "global_step", "pytorch-lightning_version", "state_dict", "optimizer_states", "lr_schedulers",
              "callbacks", "loops"):
        assert k in ck
    keys = list(ck["state_dict"])
    assert all(k.startswith("model.") for k in keys)
    assert keys[0] == "model._transformer._layers.0.norm_1.weight"
    assert keys[-1] == "model._action_token_emb.bias"
    opt = ck["optimizer_states"][0]
    # torch-Adam layout: params indexed in model.parameters() order, state only for trainable ones
    assert len(opt["param_groups"][0]["params"]) == len(list(m.parameters()))
    assert len(opt["state"]) == sum(1 for p in m.parameters() if p.requires_grad)
    path = str(tmp_path / "x.ckpt")
    C.save_checkpoint(path, ck)
    m2 = build_rt1(cfg)
    C.load_model_state(m2, path)
    for (n, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), n
    eng2 = TrainEngine(m2, cfg, order_probe=False)
    eng2.optimizer.load_state_dict(C.load_checkpoint(path)["optimizer_states"][0])
    assert eng2.optimizer.step_count == 1
    torch.testing.assert_close(eng2.optimizer.exp_avg_sq.sum(), eng.optimizer.exp_avg_sq.sum())


def test_filename_template():
    name = C.format_filename("{epoch}-{eval_loss:.6f}-{train_loss_epoch:.6f}", {"eval_loss": 0.022458,
                             "train_loss_epoch": 0.000278}, 54)
    assert name == "epoch=54-eval_loss=0.022458-train_loss_epoch=0.000278"


def test_episode_dataset_windows(tmp_path):
    ids = D.make_fake_episodes(str(tmp_path), 3, steps=5, height=32, width=48)
    ds = D.EpisodeWindowDataset(str(tmp_path), ids, window_length=3,
                                transform=D.DecodeAndRandomResizedCrop(0.95, (40, 24)))
    assert len(ds) == 15  # one window per step (left padding with window-1 copies of step 0)
    s = ds[0]
    assert s["train_observation"]["image"].shape == (3, 3, 24, 40)
    ep = np.load(tmp_path / "episode_0.npz")
    # window 0 = [step0, step0, step0]; window 4 = [step2, step3, step4]
    assert torch.equal(s["action_label"]["action"], torch.from_numpy(ep["action"][[0, 0, 0]]))
    assert torch.equal(ds[4]["action_label"]["action"], torch.from_numpy(ep["action"][[2, 3, 4]]))
    assert ds[4]["action_label"]["terminate_episode"].tolist() == [0, 0, 1]
    batch = D.collate_fn([ds[0], ds[1]])
    assert batch["train_observation"]["natural_language_embedding"].shape == (2, 3, 512)


def test_trainer_fit_logs_checkpoints_and_resumes(tmp_path):
    torch.manual_seed(0)
    cfg = rt1.preset("tiny")
    ds = D.SyntheticDataset(8, cfg.seq_len, cfg.height, cfg.width, uint8=True)
    loader = torch.utils.data.DataLoader(ds, batch_size=2, collate_fn=D.collate_fn)
    m = build_rt1(cfg)
    eng = TrainEngine(m, cfg, milestones=[1], order_probe=False)
    ck = C.ModelCheckpoint(str(tmp_path / "ckpt"))
    loggers = [CSVLogger(str(tmp_path / "csv"), "exp"), TensorBoardLogger(str(tmp_path / "tb"), "exp")]
    tr = Trainer(eng, max_epochs=2, log_every_n_steps=2, checkpoint=ck, logger=MultiLogger(loggers))
    tr.fit(loader, loader)
    tr.test(loader)
    files = sorted(os.listdir(tmp_path / "ckpt"))
    assert "last.ckpt" in files and len(files) == 3
    assert abs(eng.lr - 5e-5) < 1e-12  # MultiStepLR milestone 1, gamma 0.1
    rows = list(csv.DictReader(open(loggers[0].path)))
    assert {"train_loss_step", "train_loss_epoch", "eval_loss", "lr-Adam", "test_loss"} <= set(rows[0].keys())
    tags = {t for _, t, _ in read_scalars(glob.glob(str(tmp_path / "tb/exp/version_0/events*"))[0])}
    assert {"train_loss_step", "eval_loss", "test_loss"} <= tags
    # resume
    m2 = build_rt1(cfg)
    eng2 = TrainEngine(m2, cfg, milestones=[1], order_probe=False)
    tr2 = Trainer(eng2, max_epochs=3, log_every_n_steps=100)
    tr2.resume(str(tmp_path / "ckpt" / "last.ckpt"))
    assert tr2.current_epoch == 2 and eng2.global_step == 8
    assert abs(eng2.lr - 5e-5) < 1e-12
    tr2.fit(loader, None)
    assert eng2.global_step == 12


def test_eval_rollout_toy_env(tmp_path):
    from pytorch_rt1_for_distributed_training_amd.eval import CentralCropResize, RT1Policy, ToyPushEnv, evaluate
    torch.manual_seed(0)
    cfg = rt1.preset("tiny")
    m = build_rt1(cfg)
    ck = C.build_checkpoint(m, epoch=0, global_step=0)
    path = str(tmp_path / "m.ckpt")
    C.save_checkpoint(path, ck)
    pol = RT1Policy.from_checkpoint(path, cfg, device="cpu")
    res = evaluate(pol, ToyPushEnv(seed=1), episodes=2, max_episode_steps=5,
                   crop=CentralCropResize(cfg.width, cfg.height, 0.95), history_length=cfg.seq_len,
                   video_dir=str(tmp_path / "videos"))
    assert res["episodes"] == 2 and 0 <= res["success_rate"] <= 1
    assert len(os.listdir(tmp_path / "videos")) == 2
    a = pol.action(np.zeros((64, 64, 3), np.uint8), np.zeros(512, np.float32))
    assert a.shape == (2,) and np.all(np.abs(a) <= 0.03 + 1e-7)
    assert int(pol.state["seq_idx"][0]) >= 1


def test_data_tools_inspect_and_rlds_helpers(tmp_path):
    """tools/inspect_dataset.py (D5) on fake episodes; tools/rlds_convert.py (D4) step helpers."""
    import numpy as np
    from pytorch_rt1_for_distributed_training_amd.data.episodes import make_fake_episodes
    from tools import inspect_dataset, rlds_convert
    make_fake_episodes(str(tmp_path), 2, steps=5, height=40, width=60)
    out = str(tmp_path / "f.png")
    sample, batch = inspect_dataset.main(["--dataset_dir", str(tmp_path), "--height", "32", "--width", "48",
                                          "--seq_len", "3", "--out", out])
    assert sample["train_observation"]["image"].shape == (3, 3, 32, 48)
    assert batch["action_label"]["action"].shape == (2, 3, 2)
    assert os.path.exists(out)
    raw = np.zeros(512, np.int32)
    raw[:5] = np.frombuffer(b"push ", np.uint8)
    assert rlds_convert.decode_instruction(raw) == "push "
    steps = [{"observation": {"rgb": np.zeros((4, 6, 3), np.uint8), "instruction": raw},
              "action": np.array([0.01, -0.02], np.float32), "is_terminal": i == 2, "is_first": i == 0}
             for i in range(3)]
    arr = rlds_convert.episode_arrays(steps, lambda texts: np.ones((len(texts), 512)))
    assert arr["rgb"].shape == (3, 4, 6, 3) and arr["instruction"].shape == (3, 512)
    assert arr["is_terminal"].tolist() == [False, False, True]


def test_engine_snapshot_restore_replays_step_bitwise():
    """The state the bench's graph == eager check restores between its two steps (parameters, Adam moments and
    step, BN running statistics, torch RNG, dropout counter): a step, a restore and the same step again give
    bitwise-equal losses, gradients and parameters (dropout and drop-path on)."""
    torch.manual_seed(0)
    cfg = rt1.preset("tiny")
    eng = TrainEngine(build_rt1(cfg), cfg, order_probe=False)
    b0 = D.make_batch(2, cfg.seq_len, cfg.height, cfg.width, uint8=True)
    eng.train_step(b0)
    batch = D.make_batch(2, cfg.seq_len, cfg.height, cfg.width, uint8=True)
    snap = eng._snapshot()
    l1 = eng.train_step(batch)
    g1, p1 = eng.flat.grad.clone(), eng.flat.data.clone()
    bufs1 = [b.clone() for b in eng.model.buffers()]
    eng._restore(snap)
    assert eng.optimizer.step_count == snap["step"] and torch.equal(eng.flat.data, snap["data"])
    l2 = eng.train_step(batch)
    assert torch.equal(l1, l2)
    assert torch.equal(g1, eng.flat.grad) and torch.equal(p1, eng.flat.data)
    assert all(torch.equal(a, b) for a, b in zip(bufs1, eng.model.buffers()))
    assert eng.graph_eager_check(batch) is None                 # no captured graph on the CPU


def test_flat_grads_stolen_then_gathered():
    """zero_grad(set_to_none=True) releases .grad so AccumulateGrad steals each gradient; gather_grads lands
    them in the flat buffer (one foreach copy) with .grad re-pointed at the flat views."""
    from pytorch_rt1_for_distributed_training_amd.parallel.flat import FlatParameters
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Tanh(), torch.nn.Linear(16, 3))
    ref = [torch.nn.Parameter(p.detach().clone()) for p in net.parameters()]
    x = torch.randn(5, 8)
    flat = FlatParameters(list(net.parameters()))
    for _ in range(2):   # second pass: stale values must not accumulate
        flat.zero_grad(set_to_none=True)
        assert all(p.grad is None for p in net.parameters())
        net(x).square().sum().backward()
        flat.gather_grads()
    y = torch.nn.functional.linear(torch.tanh(torch.nn.functional.linear(x, ref[0], ref[1])), ref[2], ref[3])
    y.square().sum().backward()
    for p, r, v in zip(net.parameters(), ref, flat.views):
        assert p.grad.data_ptr() == v.data_ptr()
        torch.testing.assert_close(p.grad, r.grad)


def test_tuned_gemms_env(monkeypatch):
    """utils.tuned_gemms: read-only TunableOp settings pointing at the shipped per-device result files; an explicit
    PYTORCH_TUNABLEOP_ENABLED or RT1_TUNED_GEMMS=0 wins."""
    import os
    from pytorch_rt1_for_distributed_training_amd.utils import tuned_gemms as tg
    for k in ("PYTORCH_TUNABLEOP_ENABLED", "PYTORCH_TUNABLEOP_TUNING", "PYTORCH_TUNABLEOP_FILENAME", "RT1_TUNED_GEMMS"):
        monkeypatch.delenv(k, raising=False)
    assert tg.enable_tuned_gemms()
    assert os.environ["PYTORCH_TUNABLEOP_ENABLED"] == "1" and os.environ["PYTORCH_TUNABLEOP_TUNING"] == "0"
    base = os.environ["PYTORCH_TUNABLEOP_FILENAME"]
    assert base.endswith("tunableop_results.csv")
    for r in range(8):   # one file per local rank / device ordinal
        path = base.replace(".csv", f"{r}.csv")
        with open(path) as f:
            head = f.read(400)
        assert "Validator,GCN_ARCH_NAME,gfx950" in head
    monkeypatch.setenv("RT1_TUNED_GEMMS", "0")
    monkeypatch.delenv("PYTORCH_TUNABLEOP_ENABLED")
    assert not tg.enable_tuned_gemms()


def test_yfree_expand_backward_identity():
    """The algebra behind pwbwd.hip pw_bwd_z / ops.backbone.expand_bwd_z_wide (fp64, CPU): with y1 = x @ We^T and the
    BN1 backward dy1 = k1*dz + k2*y1 + k0, the expand conv's gradients only need dz and x:
        dx  = dy1 @ We   = (k1*dz) @ We + x @ Mk + r0,      Mk = We^T diag(k2) We,  r0 = k0 @ We
        dWe = dy1^T @ x  = diag(k1) dz^T x + diag(k2) We G + k0 (x) sx,   G = x^T x,  sx = sum_m x"""
    import torch
    g = torch.Generator().manual_seed(0)
    M, Ce, Cin = 257, 48, 8
    x = torch.randn(M, Cin, generator=g, dtype=torch.float64) + 0.7
    We = torch.randn(Ce, Cin, generator=g, dtype=torch.float64)
    dz = torch.randn(M, Ce, generator=g, dtype=torch.float64)
    k1, k2, k0 = (torch.randn(Ce, generator=g, dtype=torch.float64) for _ in range(3))
    y1 = x @ We.t()
    dy1 = k1 * dz + k2 * y1 + k0
    Mk = We.t() @ torch.diag(k2) @ We
    r0 = k0 @ We
    G, sx = x.t() @ x, x.sum(0)
    torch.testing.assert_close((k1 * dz) @ We + x @ Mk + r0, dy1 @ We)
    torch.testing.assert_close(torch.diag(k1) @ dz.t() @ x + torch.diag(k2) @ We @ G + torch.outer(k0, sx), dy1.t() @ x)
