"""On-device BC augmentation (reference input_pipeline_rlds.py:325-457).  Parity unpinned against
tf.image (TensorFlow is not in the image); the tests pin the transforms' defining properties."""
import colorsys

import numpy as np
import torch

from pytorch_rt1_for_distributed_training_amd.data import augment as A


def _img(B=2, T=3, H=24, W=40):
    g = torch.Generator().manual_seed(0)
    return (torch.rand(B, T, H, W, 3, generator=g) * 255).to(torch.uint8)


def test_crop_without_factor_at_same_size_is_identity():
    x = _img()
    y = A.random_resized_crop(x, None, (24, 40))
    assert torch.allclose(y, x.permute(0, 1, 4, 2, 3).float() / 255, atol=1e-6)


def test_crop_is_an_integer_offset_window_shared_over_time():
    H, W = 20, 30
    yy, xx = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
    frame = torch.stack([yy, xx, yy * 0], -1).float() / 255               # channel 0 = row, 1 = col
    x = frame.expand(2, 3, H, W, 3).clone()
    g = torch.Generator().manual_seed(3)
    f = 0.5
    y = A.random_resized_crop(x, f, (10, 15), g)                         # crop 10x15 -> no resampling
    for b in range(2):
        rows = y[b, :, 0] * 255
        cols = y[b, :, 1] * 255
        oy, ox = rows[0, 0, 0].item(), cols[0, 0, 0].item()
        assert abs(oy - round(oy)) < 1e-3 and abs(ox - round(ox)) < 1e-3
        assert 0 <= oy <= H - 10 and 0 <= ox <= W - 15
        assert torch.allclose(rows, oy + torch.arange(10.0)[None, :, None].expand_as(rows), atol=1e-3)
        assert torch.allclose(cols, ox + torch.arange(15.0)[None, None, :].expand_as(cols), atol=1e-3)


def test_hsv_round_trip_matches_colorsys():
    g = torch.Generator().manual_seed(1)
    x = torch.rand(1, 1, 3, 4, 5, generator=g)
    h, s, v = A._rgb_to_hsv(x)
    for i in range(4):
        for j in range(5):
            r, gg, b = x[0, 0, :, i, j].tolist()
            hh, ss, vv = colorsys.rgb_to_hsv(r, gg, b)
            assert np.allclose([h[0, 0, i, j], s[0, 0, i, j], v[0, 0, i, j]], [hh, ss, vv], atol=1e-5)
    assert torch.allclose(A._hsv_to_rgb(h, s, v), x, atol=1e-5)


def test_neutral_photometric_is_identity_and_default_stays_in_range():
    x = A._to_float_cf(_img())
    neutral = A.PhotometricDistortions(0.0, 1.0, 1.0, 0.0, 1.0, 1.0)
    assert torch.equal(neutral(x), x)
    y = A.PhotometricDistortions()(x, torch.Generator().manual_seed(0))
    assert y.shape == x.shape and y.min() >= 0 and y.max() <= 1
    assert (y - x).abs().max() > 0.01


def test_contrast_keeps_the_channel_mean():
    x = A._to_float_cf(_img()) * 0.5 + 0.25                 # away from the clip range
    only_contrast = A.PhotometricDistortions(0.0, 0.8, 1.2, 0.0, 1.0, 1.0)
    y = only_contrast(x, torch.Generator().manual_seed(0))
    assert torch.allclose(y.mean(dim=(-2, -1)), x.mean(dim=(-2, -1)), atol=1e-5)


def test_bc_augment_layout_and_reproducibility():
    x = _img(H=36, W=64)
    a1, a2 = A.BCAugment(resize_size=(18, 32), seed=5), A.BCAugment(resize_size=(18, 32), seed=5)
    y1, y2 = a1(x), a2(x)
    assert y1.shape == (2, 3, 18, 32, 3) and torch.equal(y1, y2)
    ev = a1(x, train=False)
    assert torch.equal(ev, A.BCAugment(resize_size=(18, 32), seed=9)(x, train=False))
