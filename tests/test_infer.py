"""Device-resident inference engine (engine/infer.py) == the reference-style network_state forward."""
import torch

import pytorch_rt1_for_distributed_training_amd as rt1
from pytorch_rt1_for_distributed_training_amd.engine.infer import InferenceEngine
from pytorch_rt1_for_distributed_training_amd.models import build_rt1


def test_inference_engine_matches_state_forward_through_the_roll():
    cfg = rt1.preset("tiny").replace(seq_len=3, crop_ratio=0.0)
    torch.manual_seed(0)
    ref = build_rt1(cfg).eval()
    torch.manual_seed(0)
    eng = InferenceEngine(build_rt1(cfg), cfg, device="cpu", backend="torch")
    state = ref.initial_state(1)
    g = torch.Generator().manual_seed(1)
    for step in range(8):                       # T=3: steps 3.. roll the window
        img = torch.randint(0, 256, (1, 3, 64, 64), generator=g, dtype=torch.uint8)
        ctx = torch.randn(1, 512, generator=g)
        with torch.no_grad():
            out_ref, state = ref({"image": img.float() / 255.0, "natural_language_embedding": ctx}, state)
        out = eng.step(img, ctx)
        torch.testing.assert_close(out["logits"], ref._aux_info["action_predictions_logits"].float(),
                                   rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(out["action"], out_ref["action"].float())
        assert torch.equal(out["terminate_episode"].long(), out_ref["terminate_episode"].long())
        assert int(eng.seq_idx) == int(state["seq_idx"][0]) == min(step + 1, 3)
        torch.testing.assert_close(eng.state_img, state["context_image_tokens"].float(), rtol=1e-5, atol=1e-5)
    eng.reset()
    assert int(eng.seq_idx) == 0 and float(eng.state_img.abs().sum()) == 0.0
