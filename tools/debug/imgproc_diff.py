"""Where does the GPU crop+resize differ from Pillow?  Per channel: mismatch count, first rows / columns."""
import numpy as np
import torch
from PIL import Image
from pytorch_rt1_for_distributed_training_amd.data.shards import crop_boxes
from pytorch_rt1_for_distributed_training_amd.ops import load

for (h, w, H, W) in [(360, 640, 300, 300), (64, 96, 64, 96)]:
    rng = np.random.default_rng(h * w + H)
    n = 4
    raw = rng.integers(0, 256, (n, h, w, 3), dtype=np.uint8)
    boxes = crop_boxes(rng, n, h, w, 0.95)
    got = load().crop_resize_u8(torch.from_numpy(raw).cuda(), torch.from_numpy(boxes).cuda(), H, W).cpu().numpy()
    for i in range(n):
        ref = np.asarray(Image.fromarray(raw[i]).crop(tuple(int(v) for v in boxes[i])).resize((W, H), Image.BILINEAR))
        g = got[i].transpose(1, 2, 0)
        for c in range(3):
            bad = np.argwhere(g[:, :, c] != ref[:, :, c])
            print(h, w, "frame", i, "box", boxes[i].tolist(), "ch", c, "bad", len(bad),
                  "rows", sorted(set(bad[:, 0].tolist()))[:12], "cols", sorted(set(bad[:, 1].tolist()))[:12])
