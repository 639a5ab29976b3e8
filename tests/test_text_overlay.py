"""CPU: utils.text_encoder_overlay restates zero_shot_learning.py:28-35 — the checkpoint's
text_encoder.* entries replace the CLIP text tower's (prefix stripped, cast to the tower's
dtype), other checkpoint keys are ignored, keys the checkpoint lacks keep the base values
(strict=False), and a text_encoder.* key the tower lacks raises KeyError as the reference's
dtype lookup does."""
import numpy as np
import pytest
import torch

from multimodal_reid_amd import utils


def test_overlay_semantics(tmp_path):
    base = {"ln_final.weight": torch.ones(4, dtype=torch.float16), "positional_embedding": torch.zeros(3, 4)}
    ck = {"text_encoder.ln_final.weight": torch.full((4,), 2.5), "image_encoder.conv1.weight": torch.ones(2),
          "bottleneck.weight": torch.ones(2)}
    out = utils.text_encoder_overlay(base, ck)
    assert out["ln_final.weight"].dtype == torch.float16 and torch.equal(out["ln_final.weight"], torch.full((4,), 2.5).half())
    assert out["positional_embedding"] is base["positional_embedding"]
    assert set(out) == set(base)
    path = tmp_path / "ck.pth"
    torch.save(ck, path)
    assert torch.equal(utils.text_encoder_overlay(base, str(path))["ln_final.weight"], out["ln_final.weight"])
    assert utils.text_encoder_overlay(base, None) == base
    with pytest.raises(KeyError):
        utils.text_encoder_overlay(base, {"text_encoder.not_in_the_tower": torch.ones(1)})
    np_base = {"ln_final.weight": np.ones(4, np.float32)}
    assert utils.text_encoder_overlay(np_base, ck)["ln_final.weight"].dtype == torch.float32
