"""Host-side weight-format boundary (§8f-2), CPU only: the positional-embedding resize
against the reference's own utils.resize_pos_embed / maple.build_model outputs, and the
weights-only checkpoint reader."""
import numpy as np
import pytest
import torch

from multimodal_reid_amd import synthetic as syn
from multimodal_reid_amd import model as rm
from multimodal_reid_amd import utils
from conftest import golden


@pytest.mark.parametrize("model_name,grid", [("ViT-B/16", 14), ("ViT-L/14", 16)])
def test_resize_pos_embed_bitexact_vs_reference(model_name, grid):
    """utils.py:111-125: square pretrained grid -> 21x10 (bicubic), bit for bit."""
    g = golden("adaptor.npz")
    W = syn.VIT_SPECS[model_name]["width"]
    pe = syn._normal(f"pe{grid}", (grid * grid + 1, W), W ** -0.5, 16)
    got = rm.resize_pos_embed(pe, 21, 10).numpy()
    assert np.array_equal(got.view(np.uint32), g[f"resized_{grid}"].view(np.uint32))


def test_build_model_pos_resize_bitexact():
    """maple.build_model (maple.py:1027-1041,1077-1080) resizes visual.positional_embedding
    the same way; the IVLP fixture holds the model's resized table."""
    g = golden("ivlp.npz")
    sd = syn.openai_state_dict("ViT-B/16", seed=6, vpt_ctx=2, text_ctx=2)
    got = rm.resize_pos_embed(sd["visual.positional_embedding"], 21, 10).numpy()
    assert np.array_equal(got.view(np.uint32), g["pos_resized"].view(np.uint32))


def test_load_checkpoint_weights_only(tmp_path):
    sd = {"module.image_encoder.proj": torch.randn(4, 3), "module.bottleneck.weight": torch.ones(4)}
    p = tmp_path / "a.pth"
    torch.save({"state_dict": sd}, p)
    got = utils.load_checkpoint(str(p))
    assert set(got) == {"image_encoder.proj", "bottleneck.weight"}
    assert torch.equal(got["image_encoder.proj"], sd["module.image_encoder.proj"])


class _Evil:
    pass


def test_load_checkpoint_refuses_code(tmp_path):
    """Pickled objects and TorchScript archives carry code: both are refused."""
    p = tmp_path / "b.pth"
    torch.save({"x": _Evil()}, p)
    with pytest.raises(Exception):
        utils.load_checkpoint(str(p))
    m = torch.jit.script(torch.nn.Linear(2, 2))
    q = tmp_path / "c.pt"
    torch.jit.save(m, str(q))
    with pytest.raises(Exception):
        utils.load_checkpoint(str(q))


def test_round_like_convert_weights_keys():
    """syn.round_like_convert_weights rounds exactly the tensors convert_weights casts
    (utils.py:145-166): Conv/Linear/MHA weights+biases, proj, text_projection."""
    sd = syn.openai_state_dict("ViT-B/16", seed=1, vpt_ctx=2, text_ctx=2)
    r = syn.round_like_convert_weights(sd)
    changed = {k for k in sd if not np.array_equal(sd[k], r[k])}
    for k in changed:
        assert (k.endswith(("weight", "bias", "proj", "text_projection")) and "ln_" not in k
                and "embedding" not in k and "VPT" not in k), k
    assert "visual.proj" in changed and "text_projection" in changed and "visual.conv1.weight" in changed
    assert not any("ln_" in k or "VPT" in k or "embedding" in k for k in changed)
