"""GPU random-resized-crop (csrc/kernels/imgproc.hip) is bit-exact with Pillow's crop + BILINEAR resize, the
reference transform (load_np_dataset.py:8-39)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("h,w,H,W,factor", [(360, 640, 300, 300, 0.95), (360, 640, 256, 456, 0.95),
                                            (180, 320, 300, 300, 0.95), (64, 96, 64, 96, None),
                                            (90, 70, 37, 53, 0.5)])
def test_crop_resize_bit_exact_with_pillow(h, w, H, W, factor):
    from PIL import Image
    from pytorch_rt1_for_distributed_training_amd.data.shards import crop_boxes
    from pytorch_rt1_for_distributed_training_amd.ops import load
    rng = np.random.default_rng(h * w + H)
    n = 6
    raw = rng.integers(0, 256, (n, h, w, 3), dtype=np.uint8)
    raw[0] = np.linspace(0, 255, w, dtype=np.uint8)[None, :, None]          # smooth ramps too
    boxes = crop_boxes(rng, n, h, w, factor)
    got = load().crop_resize_u8(torch.from_numpy(raw).cuda(), torch.from_numpy(boxes).cuda(), H, W).cpu().numpy()
    for i in range(n):
        ref = np.asarray(Image.fromarray(raw[i]).crop(tuple(int(v) for v in boxes[i])).resize((W, H), Image.BILINEAR))
        assert np.array_equal(got[i].transpose(1, 2, 0), ref), (i, int(np.abs(got[i].transpose(1, 2, 0).astype(int) - ref).max()))


def test_decode_on_device_matches_cpu_path():
    from pytorch_rt1_for_distributed_training_amd.data.shards import crop_boxes, decode_on_device
    rng = np.random.default_rng(0)
    raw = torch.from_numpy(rng.integers(0, 256, (2, 3, 120, 160, 3), dtype=np.uint8))
    boxes = torch.from_numpy(crop_boxes(rng, 6, 120, 160, 0.9).reshape(2, 3, 4))
    batch = {"train_observation": {"raw_frames": raw, "crop_boxes": boxes,
                                   "natural_language_embedding": torch.zeros(2, 3, 512)},
             "action_label": {}}
    cpu = decode_on_device(batch, 64, 80)["train_observation"]["image"]
    gb = {"train_observation": {k: v.cuda() for k, v in batch["train_observation"].items()}, "action_label": {}}
    gpu = decode_on_device(gb, 64, 80)["train_observation"]["image"].cpu()
    assert torch.equal(cpu, gpu)
