"""Pins the CPU oracle against fixtures produced by the reference itself
(tests/golden/make_goldens.py) and against numpy's own arithmetic."""
import numpy as np
import pytest
import torch

import oracle
from multimodal_reid_amd import synthetic as syn
from conftest import golden


def test_np_exp_emulation_bitexact():
    r = np.random.default_rng(0)
    x = np.concatenate([-r.random(200000) * 3, r.standard_normal(50000) * 20, [0.0, -0.0, 1e-30, -88.0]]).astype(np.float32)
    L = oracle.lib()
    mine = np.array([L.orc_np_expf(float(v)) for v in x], np.float32)
    assert np.array_equal(mine.view(np.uint32), np.exp(x).view(np.uint32))


@pytest.mark.parametrize("n", [1, 3, 7, 8, 9, 15, 16, 17, 64, 127, 128, 129, 130, 255, 256, 257, 1000, 1377])
def test_pairwise_sums_match_numpy(n):
    r = np.random.default_rng(n)
    a = np.exp(-r.random(n) * 9).astype(np.float32)
    assert oracle.lib().orc_pairwise_f32(a, n) == a.sum()
    d = r.random(n) * (r.random(n) < 0.3)
    assert oracle.lib().orc_pairwise_f64(d, n) == d.sum()


def test_f2h_matches_numpy():
    r = np.random.default_rng(1)
    bits = np.concatenate([r.integers(0, 2**32, 300000, dtype=np.uint64).astype(np.uint32),
                           np.arange(0x33000000 - 5, 0x33000000 + 5, dtype=np.uint32),
                           np.arange(0x477fe000, 0x47800010, 0x100, dtype=np.uint32)])
    f = bits.view(np.float32)
    f = f[np.isfinite(f)]
    L = oracle.lib()
    mine = np.array([L.orc_f2h(float(v)) for v in f], np.uint16)
    assert np.array_equal(mine, f.astype(np.float16).view(np.uint16))


def _backend_inputs(seed=1):
    qp, gp, qc, gc = syn.labels(100, 500, num_ids=60, num_cams=6, seed=seed, distractor_frac=0.1,
                                junk_frac=0.04 if seed == 1 else 0.0)
    qf, gf = syn.features(qp, gp, dim=1280, seed=seed, noise=4.0)
    return qf, gf


def test_l2norm_and_distmat_close_to_reference():
    g = golden("backend_small.npz")
    qf, gf = _backend_inputs()
    feats = np.concatenate([qf, gf])
    n_ref = torch.nn.functional.normalize(torch.from_numpy(feats), dim=1, p=2).numpy()
    n_orc = oracle.l2norm(feats)
    assert np.abs(n_orc - n_ref).max() < 1e-7
    d = oracle.distmat(n_orc[:100], n_orc[100:])
    assert np.abs(d - g["distmat"]).max() < 1e-5  # ~17 ulp at 2.0: BLAS vs sequential k order


def test_eval_func_bitexact_on_reference_distmat():
    g = golden("backend_small.npz")
    cmc, mAP = oracle.eval_func(g["distmat"], g["q_pids"], g["g_pids"], g["q_cams"], g["g_cams"], 50)
    assert np.array_equal(cmc, g["cmc_stable"]) and cmc.dtype == np.float32
    assert mAP == g["map_stable"]
    # no exact ties among these rows: the unstable reference agrees too
    assert np.array_equal(cmc, g["cmc_unstable"]) and mAP == g["map_unstable"]
    assert np.array_equal(oracle.topk_rows(g["distmat"], 50), g["rank50_stable"])


def test_eval_func_bitexact_with_ties():
    g = golden("backend_ties.npz")
    cmc, mAP = oracle.eval_func(g["distmat"], g["q_pids"], g["g_pids"], g["q_cams"], g["g_cams"], 20)
    assert np.array_equal(cmc, g["cmc_stable"])
    assert mAP == g["map_stable"]
    assert np.array_equal(oracle.topk_rows(g["distmat"], 20), g["rank20_stable"])


@pytest.mark.parametrize("k1,k2", [(50, 15), (20, 6)])
def test_rerank_stages_bitexact(k1, k2):
    g = golden("rerank_small.npz")
    tag = f"k{k1}_{k2}"
    final, rank, vqe, jac = oracle.rerank_from_dist(g["dist_all"], 100, k1, k2, 0.3, debug=True)
    assert np.array_equal(rank[:, :k1 + 1], g[f"initial_rank_{tag}"])
    assert np.array_equal(vqe, g[f"vqe_{tag}"])
    assert np.array_equal(jac[:, :], g[f"jaccard_{tag}"])
    assert np.array_equal(final.view(np.uint32), g[f"final_{tag}"].view(np.uint32))
    cmc, mAP = oracle.eval_func(final, g["q_pids"], g["g_pids"], g["q_cams"], g["g_cams"], 50)
    assert np.array_equal(cmc, g[f"cmc_{tag}"]) and mAP == g[f"map_{tag}"]


@pytest.mark.parametrize("k1,k2", [(50, 15), (20, 6)])
def test_rerank_full_path_close(k1, k2):
    """From features: the reference's torch-BLAS distance differs from the oracle's by
    a few ulp, which moves exp() weights and fp16 Jaccard sums; parity is therefore
    stated at mAP level (|dmAP| <= 1e-3, BASELINE.json) with a bounded distance error."""
    g = golden("rerank_small.npz")
    qf, gf = syn.features(g["q_pids"], g["g_pids"], dim=1280, seed=3, noise=4.0)
    feats = oracle.l2norm(np.concatenate([qf, gf]))
    final = oracle.re_ranking(feats[:100], feats[100:], k1, k2, 0.3)
    ref = g[f"final_full_k{k1}_{k2}"]
    assert np.abs(final - ref).max() < 5e-3
    args = (g["q_pids"], g["g_pids"], g["q_cams"], g["g_cams"], 50)
    assert abs(oracle.eval_func(final, *args)[1] - oracle.eval_func(ref, *args)[1]) <= 1e-3


# ------------------------------------------------------------------ encoders (fp32 restatement)
def _cos(a, b):
    a = np.asarray(a, np.float64).reshape(len(a), -1)
    b = np.asarray(b, np.float64).reshape(len(b), -1)
    return (a * b).sum(1) / np.linalg.norm(a, axis=1) / np.linalg.norm(b, axis=1)


def test_vit_b16_oracle_vs_reference():
    """oracle/vit_ref.py (fp32) vs the reference VisionTransformer's outputs
    (custom_clip_model.py:77-100) on the same seeded weights/images, plain and TTA view."""
    from oracle import vit_ref
    g = golden("vit_b16.npz")
    sd = syn.vit_state_dict("ViT-B/16", seed=0)
    imgs = syn.images(3, seed=0)
    with torch.no_grad():
        x11, x12, xp = vit_ref.vit_forward(sd, imgs)
        _, t12, tp = vit_ref.vit_forward(sd, imgs, tta=g["tta_offsets"])
    for got, ref in ((x12[:, 0], g["x12cls"]), (xp[:, 0], g["projcls"]), (x11[:, 0], g["x11cls"]),
                     (x12[0, :8], g["x12_tok"]), (xp[0, 100:104], g["proj_tok"]),
                     (t12[:, 0], g["tta_x12cls"]), (tp[:, 0], g["tta_projcls"])):
        assert np.abs(got.numpy() - ref).max() < 2e-5


def test_fast_vit_port_equals_reference_module_outputs():
    """vit_ref.FastVit (the CPU baseline bench.py times) runs the reference modules' op sequence
    (custom_clip_model.py:77-100) and reproduces their fp32 outputs on the fixture, TTA view too."""
    from oracle import vit_ref
    g = golden("vit_b16.npz")
    fv = vit_ref.FastVit(syn.vit_state_dict("ViT-B/16", seed=0))
    imgs = syn.images(3, seed=0)
    x11, x12, xp = fv(imgs)
    _, t12, tp = fv(imgs, tta=g["tta_offsets"])
    for got, ref in ((x12[:, 0], g["x12cls"]), (xp[:, 0], g["projcls"]), (x11[:, 0], g["x11cls"]),
                     (x12[0, :8], g["x12_tok"]), (xp[0, 100:104], g["proj_tok"]),
                     (t12[:, 0], g["tta_x12cls"]), (tp[:, 0], g["tta_projcls"])):
        assert np.abs(got.numpy() - ref).max() < 2e-5


def test_vit_l14_oracle_vs_reference():
    """ViT-L/14 (configs[4]) as the reference executes it (resblocks[:11] + [11])."""
    from oracle import vit_ref
    g = golden("vit_l14.npz")
    sd = syn.vit_state_dict("ViT-L/14", seed=0, layers=12)
    imgs = syn.images(2, seed=4)
    with torch.no_grad():
        x11, x12, xp = vit_ref.vit_forward(sd, imgs)
    for got, ref in ((x12[:, 0], g["x12cls"]), (xp[:, 0], g["projcls"]), (x11[:, 0], g["x11cls"]),
                     (x12[1, 200:204], g["x12_tok"])):
        assert np.abs(got.numpy() - ref).max() < 2e-5
        assert _cos(got.numpy(), ref).min() > 0.999999


def test_tta_view_matches_augmented_images():
    """The flip + pad + crop view the kernels build from offsets equals the host restatement
    of the augmented loader's transform (data_prepare.py:263-270)."""
    from oracle import vit_ref
    imgs = syn.images(4, seed=9)
    offs = syn.tta_offsets(4, seed=9)
    a = vit_ref.tta_view(torch.from_numpy(imgs), offs).numpy()
    b = syn.tta_images_np(imgs, offs)
    assert np.array_equal(a, b)


def test_text_oracle_vs_reference():
    """oracle text tower vs text_encoder.TextEncoder (text_encoder.py:14-24) outputs."""
    from oracle import vit_ref
    g = golden("text.npz")
    sd = syn.text_state_dict(seed=0)
    with torch.no_grad():
        f = vit_ref.text_forward(sd, g["tokens"])
    assert np.abs(f.numpy() - g["text_feat"]).max() < 2e-5


def test_ivlp_oracle_vs_reference_build_model():
    """oracle IVLP towers (vision VPT + per-block VPT_shallow, text prompts) vs the
    reference's maple.build_model CLIP (maple.py:617-644,754-785,971-984) run in fp32 on
    convert_weights-rounded weights: pins the IVLP restatement to the reference."""
    from oracle import vit_ref
    from multimodal_reid_amd.model import resize_pos_embed
    g = golden("ivlp.npz")
    sd = syn.round_like_convert_weights(syn.openai_state_dict("ViT-B/16", seed=6, vpt_ctx=2, text_ctx=2))
    vis = {k[len("visual."):]: v for k, v in sd.items() if k.startswith("visual.")}
    vis["positional_embedding"] = resize_pos_embed(vis["positional_embedding"], 21, 10).numpy()
    txt = {k: v for k, v in sd.items() if not k.startswith("visual.")}
    imgs = syn.images(2, seed=6)
    with torch.no_grad():
        x11, x12, xp = vit_ref.vit_forward(vis, imgs)
        t = vit_ref.text_forward(txt, g["tokens"])
    for got, ref in ((x12[:, 0], g["x12cls"]), (x11[:, 0], g["x11cls"]), (xp[:, 0], g["projcls"]),
                     (x12[1, -2:], g["x12_prompt"]), (xp[0, 100:103], g["proj_tok"]), (t, g["text_feat"])):
        assert np.abs(got.numpy() - ref).max() < 2e-5


def test_threaded_oracle_is_deterministic():
    """The C restatement's parallel loops (bench.py's CPU baseline runs them on the host's
    cores) give bit-identical results for any thread count."""
    qp, gp, qc, gc = syn.labels(90, 410, num_ids=50, num_cams=5, seed=8)
    qf, gf = syn.features(qp, gp, dim=256, seed=8)
    outs = []
    for th in (1, 5):
        oracle.set_threads(th)
        d = oracle.distmat(qf, gf)
        outs.append((d, *oracle.eval_rows(d, qp, gp, qc, gc), oracle.re_ranking(qf, gf, 20, 6, 0.3),
                     oracle.topk_rows(d, 33)))
    oracle.set_threads(1)
    for a, b in zip(*outs):
        assert np.array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8))
