"""Language-Table BC stack networks: ResNet-V1 (parameter counts pinned to the reference's
``resnet_v1_test.py:24-40``), the multiscale trunk, PixelLangMSE, and the BC trainer's freeze / pretrained-load
options (``bc.py:91-140``)."""
import pytest
import torch

from pytorch_rt1_for_distributed_training_amd.models import resnet_v1 as R


@pytest.mark.parametrize("ctor,count", [(R.ResNet18, 11_689_512), (R.ResNet34, 21_797_672),
                                        (R.ResNet50, 25_557_032), (R.ResNet101, 44_549_160),
                                        (R.ResNet152, 60_192_808), (R.ResNet200, 64_673_832)])
def test_resnet_v1_parameter_counts(ctor, count):
    m = ctor(num_classes=1000)
    assert R.count_parameters(m) == count


def test_resnet_forward_same_padding_and_init():
    torch.manual_seed(0)
    m = R.ResNet18(num_classes=10).eval()
    x = torch.rand(2, 224, 224, 3)
    y = m(x)
    assert y.shape == (2, 10)
    assert torch.count_nonzero(y) == 0                       # zero-initialised head (reference)
    # SAME padding of a stride-2 7x7 conv: 224 -> 112, extra pad on the bottom/right
    c = m.init_conv(x.permute(0, 3, 1, 2))
    assert c.shape[-2:] == (112, 112)
    ref = torch.nn.functional.conv2d(torch.nn.functional.pad(x.permute(0, 3, 1, 2), (2, 3, 2, 3)),
                                     m.init_conv.weight, stride=2)
    torch.testing.assert_close(c, ref)
    # basic blocks zero their second BN scale; bottleneck blocks do not zero bn3 (as the reference code does)
    assert float(m.stages[0][0].bn2.weight.abs().sum()) == 0.0
    b50 = R.ResNet50(num_classes=10)
    assert float(b50.stages[0][0].bn3.weight.abs().sum()) > 0


def test_multiscale_resnet_pyramid():
    m = R.MultiscaleResNet(R.ResNetBlock, (2, 2, 2, 2)).eval()
    outs = m(torch.rand(1, 128, 160, 3))
    shapes = [tuple(o.shape) for o in outs]
    assert shapes == [(1, 64, 80, 64), (1, 32, 40, 64), (1, 32, 40, 64), (1, 16, 20, 128), (1, 8, 10, 256),
                      (1, 4, 5, 512)]


def test_pixel_lang_mse_forward_backward():
    from pytorch_rt1_for_distributed_training_amd.models.lava import PixelLangMSE
    torch.manual_seed(0)
    m = PixelLangMSE(action_size=2, dense_resnet_width=64, dense_resnet_num_blocks=2, sequence_length=4)
    obs = {"rgb": torch.randint(0, 256, (3, 4, 48, 64, 3), dtype=torch.uint8),
           "clip_embedding": torch.randn(3, 4, 512)}
    a = m(obs)
    assert a.shape == (3, 2)
    a.square().mean().backward()
    assert m.encoder.convs[0].weight.grad is not None
    # only the LAST step's language embedding conditions the network
    obs2 = dict(obs, clip_embedding=obs["clip_embedding"].clone())
    obs2["clip_embedding"][:, :3] = 0
    torch.testing.assert_close(m(obs2), m(obs))
    # the first conv is not language-fused (fuse_from = 2), the others are
    assert m.encoder._fuse == [False, True, True, True]


def test_bc_trainer_freeze_and_pretrained_prefix_load(tmp_path):
    import numpy as np
    from pytorch_rt1_for_distributed_training_amd.engine.bc import BCTrainer
    from pytorch_rt1_for_distributed_training_amd.models.lava import PixelLangMSE
    torch.manual_seed(0)
    src = PixelLangMSE(dense_resnet_width=64)
    path = tmp_path / "pre.pt"
    # a "pretrained" checkpoint whose encoder lives under another prefix
    torch.save({("tower." + k[len("encoder."):]): v for k, v in src.state_dict().items() if k.startswith("encoder.")},
               path)
    torch.manual_seed(1)
    m = PixelLangMSE(dense_resnet_width=64)
    stats = {"action": {"mean": np.zeros(2, np.float32), "std": np.ones(2, np.float32)}}
    tr = BCTrainer(m, stats, freeze_keys=("encoder.convs.0",), device=torch.device("cpu"),
                   pretrained_checkpoints=[(str(path), [("tower.", "encoder.")])])
    assert len(tr.loaded_pretrained) == len([k for k in src.state_dict() if k.startswith("encoder.")])
    for k, v in src.state_dict().items():
        if k.startswith("encoder."):
            assert torch.equal(m.state_dict()[k], v), k
    frozen = m.encoder.convs[0].weight.detach().clone()
    other = m.encoder.convs[1].weight.detach().clone()
    batch = {"observation": {"rgb": torch.rand(2, 4, 32, 32, 3), "clip_embedding": torch.randn(2, 4, 512)},
             "action": torch.randn(2, 2)}
    tr.train_step(batch)
    assert torch.equal(m.encoder.convs[0].weight, frozen)          # set_to_zero for frozen keys
    assert not torch.equal(m.encoder.convs[1].weight, other)


import pytest


@pytest.mark.parametrize("which", ["pixel", "pyramid"])
def test_conv_init_matches_flax_defaults(which):
    """PixelLangMSE's encoder convs (pixel.py:56) and the LAVA pyramid encoder (lava.py:43) use Flax nn.Conv's init:
    truncated LeCun-normal weights, zero bias."""
    import math
    import torch
    from pytorch_rt1_for_distributed_training_amd.models.lava import ConvMaxpoolEncoder, PixelLangMSE
    torch.manual_seed(0)
    m = PixelLangMSE(dense_resnet_width=64) if which == "pixel" else ConvMaxpoolEncoder()
    convs = [mod for mod in m.modules() if isinstance(mod, torch.nn.Conv2d) and mod.kernel_size == (3, 3)]
    assert len(convs) >= 4
    for c in convs:
        fan_in = c.in_channels * 9
        w = c.weight.detach()
        assert torch.count_nonzero(c.bias) == 0
        # truncated at 2 sigma of the pre-truncation std (std / 0.8796); the truncated std itself is 1/sqrt(fan_in)
        lim = 2 * math.sqrt(1.0 / fan_in) / 0.87962566103423978
        assert float(w.abs().max()) <= lim * (1 + 1e-5)
        if w.numel() >= 2000:
            assert abs(float(w.std()) * math.sqrt(fan_in) - 1.0) < 0.08
