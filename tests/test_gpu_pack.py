"""The checkpoint boundary of SURVEY.md §8b through the C ABI: reidmi_vit_weights_pack /
reidmi_text_weights_pack (pack.hip) turn the reference's fp32 tensors, in its key layout
(custom_clip_model.VisionTransformer / the CLIP text tower: utils.py:169-221,
zero_shot_learning.py:28-35), into the packed towers reidmi_vit_forward / reidmi_text_forward
run.  Every packed byte is checked against a host restatement of the packing:
model.fold_layernorm (fp16(fp32(W gamma)), exact column sums, fsum-rounded folded bias), plain
fp16 casts, the zero-padded conv1 and the transposed projections, fp32 copies."""
import ctypes

import numpy as np
import pytest
import torch

from multimodal_reid_amd import synthetic as syn

pytestmark = pytest.mark.gpu


def _read(buf, ptr, n, dtype):
    off = ptr - buf.data_ptr()
    nb = n * np.dtype(dtype).itemsize
    assert 0 <= off and off + nb <= buf.numel(), "packed pointer outside the caller's buffer"
    return buf[off:off + nb].cpu().numpy().view(dtype)


def _same(got, exp, what):
    """Bytes equal; on a mismatch report how many and the first few (index, got, expected)."""
    got, exp = np.asarray(got).ravel(), np.asarray(exp).ravel()
    assert got.shape == exp.shape, (what, got.shape, exp.shape)
    bad = np.nonzero(got != exp)[0]
    assert len(bad) == 0, (what, len(bad), [(int(i), int(got[i]), int(exp[i])) for i in bad[:8]])


def _f16(a):
    return np.asarray(a, np.float32).astype(np.float16)


def _check_blocks(m, sd, W, layers):
    from multimodal_reid_amd.model import fold_layernorm
    buf = m._packed
    for i in range(layers):
        p = f"transformer.resblocks.{i}."
        b = m._blocks[i]
        for wk, bk, g, be, N, (pw, pb, ps) in (
                ("attn.in_proj_weight", "attn.in_proj_bias", "ln_1.weight", "ln_1.bias", 3 * W, ("qkv_w", "qkv_b", "qkv_s")),
                ("mlp.c_fc.weight", "mlp.c_fc.bias", "ln_2.weight", "ln_2.bias", 4 * W, ("fc1_w", "fc1_b", "fc1_s"))):
            wf, s, bf = fold_layernorm(sd[p + wk], sd[p + bk], sd[p + g], sd[p + be])
            _same(_read(buf, getattr(b, pw), N * W, np.uint16), wf.numpy().view(np.uint16), (i, pw))
            _same(_read(buf, getattr(b, ps), N, np.uint32), s.numpy().view(np.uint32), (i, ps))
            _same(_read(buf, getattr(b, pb), N, np.uint32), bf.numpy().view(np.uint32), (i, pb))
        _same(_read(buf, b.out_w, W * W, np.uint16), _f16(sd[p + "attn.out_proj.weight"]).view(np.uint16), (i, "out_w"))
        _same(_read(buf, b.fc2_w, W * 4 * W, np.uint16), _f16(sd[p + "mlp.c_proj.weight"]).view(np.uint16), (i, "fc2"))
        for f, k in (("out_b", "attn.out_proj.bias"), ("fc2_b", "mlp.c_proj.bias"), ("ln1_w", "ln_1.weight"),
                     ("ln2_b", "ln_2.bias")):
            ref = np.asarray(sd[p + k], np.float32).ravel()
            assert np.array_equal(_read(buf, getattr(b, f), ref.size, np.float32), ref), (i, f)
        if (p + "VPT_shallow") in sd:
            ref = np.asarray(sd[p + "VPT_shallow"], np.float32).ravel()
            assert np.array_equal(_read(buf, b.prompt, ref.size, np.float32), ref)
        else:
            assert not b.prompt


@pytest.mark.parametrize("model,vpt", [("ViT-B/16", 0), ("ViT-B/16", 2)])
def test_vit_weights_pack_bytes(gpu, model, vpt):
    from multimodal_reid_amd.model import VisionTransformer
    sd = syn.vit_state_dict(model, seed=40 + vpt, vpt_ctx=vpt) if vpt else syn.vit_state_dict(model, seed=40)
    m = VisionTransformer(sd, device=gpu)
    torch.cuda.synchronize()
    w = m.weights
    W, P, E = m.width, m.patch, m.out_dim
    assert (w.width, w.layers, w.heads, w.patch, w.stride, w.out_dim, w.n_ctx) == (W, m.layers, W // 64, P, 12, E, vpt)
    conv = np.asarray(sd["conv1.weight"], np.float32).reshape(W, -1)
    cp = np.zeros((W, w.kpad), np.float32)
    cp[:, :conv.shape[1]] = conv
    assert w.kpad % 64 == 0
    _same(_read(m._packed, w.conv_w, W * w.kpad, np.uint16), _f16(cp).view(np.uint16), "conv_w")
    proj = np.asarray(sd["proj"], np.float32)
    _same(_read(m._packed, w.proj_t, E * W, np.uint16), _f16(proj.T).view(np.uint16), "proj_t")
    pos = np.asarray(sd["positional_embedding"], np.float32).ravel()
    assert np.array_equal(_read(m._packed, w.pos_emb, pos.size, np.float32), pos)
    if vpt:
        assert np.array_equal(_read(m._packed, w.vpt, vpt * W, np.float32), np.asarray(sd["VPT"], np.float32).ravel())
    _check_blocks(m, sd, W, m.layers)


def test_text_weights_pack_bytes(gpu):
    from multimodal_reid_amd.model import TextTransformer
    sd = syn.text_state_dict(seed=41)
    m = TextTransformer(sd, device=gpu)
    torch.cuda.synchronize()
    w = m.weights
    W, E = m.width, m.out_dim
    tp = np.asarray(sd["text_projection"], np.float32)
    _same(_read(m._packed, w.proj_t, E * W, np.uint16), _f16(tp.T).view(np.uint16), "text proj_t")
    tok = np.asarray(sd["token_embedding.weight"], np.float32).ravel()
    assert np.array_equal(_read(m._packed, w.tok_emb, tok.size, np.float32), tok)
    _check_blocks(m, sd, W, m.layers)


def test_pack_rejects_bad_buffers(gpu):
    """A buffer smaller than reidmi_vit_pack_bytes, or misaligned, is refused with a message."""
    from multimodal_reid_amd import _lib, model as mdl
    sd = syn.vit_state_dict("ViT-B/16", seed=42, layers=12)
    m = mdl.VisionTransformer(sd, device=gpu)
    vs = mdl.VitSrc()
    vs.width, vs.layers, vs.patch, vs.stride, vs.out_dim, vs.grid_h, vs.grid_w, vs.n_ctx = 768, 12, 16, 12, 512, 21, 10, 0
    vs.blocks = (mdl.BlockSrc * 12)()
    n = mdl._fn("reidmi_vit_pack_bytes")(ctypes.byref(vs))
    assert n > 150e6  # ViT-B/16: ~172 MB packed
    buf = torch.empty(1024, dtype=torch.uint8, device=gpu)
    out, blocks = mdl.VitWeights(), (mdl.BlockWeights * 12)()
    rc = mdl._fn("reidmi_vit_weights_pack")(ctypes.byref(vs), buf.data_ptr(), 1024, ctypes.byref(out), blocks,
                                             _lib.stream())
    assert rc != 0 and b"buffer" in _lib.load().reidmi_last_error()
    vs.layers = 11
    assert mdl._fn("reidmi_vit_pack_bytes")(ctypes.byref(vs)) == -1  # resblocks[:12] run: >= 12 layers
    del m
