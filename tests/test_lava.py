"""LAVA behaviour-cloning family (models/lava.py, engine/bc.py, data/normalization.py, data/sim_demos.py)."""
import os
import socket

import numpy as np
import torch
import torch.multiprocessing as mp

from pytorch_rt1_for_distributed_training_amd.data import normalization, sim_demos
from pytorch_rt1_for_distributed_training_amd.models.lava import LavaConfig, SequenceLAVMSE, sincos_1d, sincos_2d


def _small_cfg():
    return LavaConfig(d_model=32, num_layers=2, temporal_layers=1, dense_resnet_width=64, height=48, width=64,
                      dropout=0.0)


def _obs(b=2, t=4, h=48, w=64, seed=0):
    g = torch.Generator().manual_seed(seed)
    return {"rgb": torch.randint(0, 256, (b, t, h, w, 3), dtype=torch.uint8, generator=g),
            "instruction_embedding": torch.randn(b, t, 512, generator=g)}


def test_lava_forward_shapes_and_default_config():
    m = SequenceLAVMSE(_small_cfg())
    assert m(_obs()).shape == (2, 2)
    full = SequenceLAVMSE(LavaConfig())                       # language_table_sim_local sizes
    assert full.cfg.d_model == 128 and len(full.cross) == 4 and len(full.temporal) == 2
    assert full.head.inp.out_features == 1024 and len(full.head.blocks) == 2


def test_positional_encodings():
    pe = sincos_1d(4, 8)
    assert torch.allclose(pe[0, 0::2], torch.zeros(4)) and torch.allclose(pe[0, 1::2], torch.ones(4))
    p2 = sincos_2d(16, 3, 5)                                  # (h*w, d); column in the first half of the channels
    assert p2.shape == (15, 16)
    row0 = p2.view(3, 5, 16)
    assert torch.allclose(row0[:, 0, 0::2][:, :4], torch.zeros(3, 4))   # sin(col=0)
    assert torch.allclose(row0[0, :, 8::2], torch.zeros(5, 4))          # sin(row=0)
    assert torch.allclose(row0[1, 2, :8], row0[0, 2, :8])              # column part independent of the row


def test_chan_statistics_match_numpy():
    rng = np.random.default_rng(0)
    chunks = [rng.normal(3.0, 2.0, (n, 3)) for n in (5, 17, 1, 40)]
    st = normalization.ChanStats()
    for c in chunks:
        st.update(c)
    allx = np.concatenate(chunks)
    np.testing.assert_allclose(st.mean, allx.mean(0), rtol=1e-10)
    np.testing.assert_allclose(st.std, allx.std(0), rtol=1e-10)
    n = normalization.StdNormalizer([1.0, 2.0], [2.0, 4.0], eps=0.0)
    x = torch.tensor([[3.0, 10.0]])
    assert torch.allclose(n.denormalize(n.normalize(x)), x)
    mm = normalization.MinMaxNormalizer([-0.1, -0.1], [0.1, 0.1], eps=0.0)
    assert torch.allclose(mm.normalize(torch.tensor([0.1, -0.1])), torch.tensor([1.0, -1.0]))


def test_bc_trainer_overfits_and_checkpoints(tmp_path):
    from pytorch_rt1_for_distributed_training_amd.engine.bc import BCTrainer
    torch.manual_seed(0)
    eps = sim_demos.synthetic_episodes(2, steps=6, height=48, width=64)
    ds = sim_demos.WindowDataset(eps, 4)
    assert len(ds) == 12
    s0 = ds[0]["observation"]["rgb"]
    assert torch.equal(s0[0], s0[3])                         # front padding with step 0
    stats = normalization.compute_dataset_statistics(sim_demos.action_batches(ds), num_samples=len(ds))
    tr = BCTrainer(SequenceLAVMSE(_small_cfg()), stats, lr=1e-3, device=torch.device("cpu"))
    batch = sim_demos.collate([ds[i] for i in range(8)])
    losses = [float(tr.train_step(batch)) for _ in range(40)]
    assert losses[-1] < 0.2 * losses[0], losses[::8]
    path = str(tmp_path / "lava.pt")
    tr.save(path)
    tr2 = BCTrainer(SequenceLAVMSE(_small_cfg()), stats, device=torch.device("cpu"))
    assert tr2.restore_or_init(path) and tr2.step == 40
    torch.testing.assert_close(tr2.predict(batch["observation"]), tr.predict(batch["observation"]))


def test_sim_demos_and_lava_policy():
    from pytorch_rt1_for_distributed_training_amd.eval.policy import LavaPolicy
    eps = sim_demos.collect_episodes(2, "block2block", seed=3, max_steps=40)
    assert all(e["rgb"].shape[1:] == (180, 320, 3) for e in eps)
    assert sum(bool(e["success"]) for e in eps) >= 1            # the oracle solves most boards
    ds = sim_demos.WindowDataset(eps, 4)
    stats = normalization.compute_dataset_statistics(sim_demos.action_batches(ds), num_samples=len(ds))
    pol = LavaPolicy(SequenceLAVMSE(LavaConfig(d_model=32, num_layers=1, temporal_layers=1,
                                               dense_resnet_width=64)), stats, device="cpu")
    a = pol.action(eps[0]["rgb"][0], eps[0]["instruction_embedding"][0])
    assert a.shape == (2,) and np.all(np.abs(a) <= 0.03 + 1e-7)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(2)
    from pytorch_rt1_for_distributed_training_amd.engine.bc import BCTrainer
    from pytorch_rt1_for_distributed_training_amd.parallel import dist as pdist
    pdist.init_distributed("cpu")
    torch.manual_seed(100 + rank)                             # different init: the parameter broadcast must fix it
    eps = sim_demos.synthetic_episodes(2, steps=4, height=48, width=64, seed=1)
    ds = sim_demos.WindowDataset(eps, 4)
    stats = {"action": {"mean": np.zeros(2, np.float32), "std": np.ones(2, np.float32)}}
    tr = BCTrainer(SequenceLAVMSE(_small_cfg()), stats, device=torch.device("cpu"), bucket_cap_mb=0.05)
    full = sim_demos.collate([ds[i] for i in range(8)])
    shard = {"observation": {k: v[rank * 4:(rank + 1) * 4] for k, v in full["observation"].items()},
             "action": full["action"][rank * 4:(rank + 1) * 4]}
    tr.ddp.prepare()
    tr.optimizer.zero_grad()
    tr.model.eval()                                           # dropout off: deterministic comparison
    tr.loss(shard).backward()
    tr.ddp.finish()
    torch.save({"grad": tr.flat.grad * tr.ddp.grad_scale, "data": tr.flat.data.clone(),
                "nb": len(tr.ddp.buckets)}, os.path.join(out, f"r{rank}.pt"))
    pdist.shutdown()


def test_bc_data_parallel_gloo_matches_single_process(tmp_path):
    from pytorch_rt1_for_distributed_training_amd.engine.bc import BCTrainer
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r0, r1 = (torch.load(tmp_path / f"r{i}.pt", weights_only=True) for i in range(2))
    assert r0["nb"] > 1
    assert torch.equal(r0["data"], r1["data"]) and torch.equal(r0["grad"], r1["grad"])
    # single process, full batch, rank-0 initialisation
    torch.manual_seed(100)
    eps = sim_demos.synthetic_episodes(2, steps=4, height=48, width=64, seed=1)
    ds = sim_demos.WindowDataset(eps, 4)
    stats = {"action": {"mean": np.zeros(2, np.float32), "std": np.ones(2, np.float32)}}
    tr = BCTrainer(SequenceLAVMSE(_small_cfg()), stats, device=torch.device("cpu"))
    torch.testing.assert_close(tr.flat.data, r0["data"])
    tr.optimizer.zero_grad()
    tr.model.eval()
    tr.loss(sim_demos.collate([ds[i] for i in range(8)])).backward()
    tr.flat.gather_grads()
    torch.testing.assert_close(tr.flat.grad, r0["grad"], rtol=1e-4, atol=1e-6)
