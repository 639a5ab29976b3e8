"""Generate the committed parity fixtures by running the REFERENCE code itself.

Runs only in the build container (it imports /root/reference read-only; the
reference never travels to the GPU box).  Modules imported as-is, no stubs:
evaluate.py, reranking.py, custom_clip_model.py, text_encoder.py.
Inputs come from multimodal_reid_amd.synthetic, so the GPU box regenerates the
exact same inputs/weights from seeds and only the outputs are stored here.

Tie canonicalisation: the reference's np.argsort is the
unstable introsort.  Fixtures named *_stable were produced by running the
reference with its module-global ``np`` swapped for a proxy whose ``argsort``
is ``kind="stable"`` — the reference code path is otherwise untouched.

    python tests/golden/make_goldens.py [--out tests/golden]
"""
import argparse
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import synthetic as syn  # noqa: E402

sys.path.insert(0, REF)
import evaluate as ref_eval  # noqa: E402  (reference)
import reranking as ref_rr  # noqa: E402  (reference)
import custom_clip_model as ref_ccm  # noqa: E402  (reference)
import text_encoder as ref_te  # noqa: E402  (reference)


class _StableNp(types.ModuleType):
    """numpy proxy whose argsort is stable; records every argsort result."""

    def __init__(self):
        super().__init__("numpy_stable_proxy")
        self.calls = []
        self.zeros_like_out = []

    def __getattr__(self, name):
        return getattr(np, name)

    def argsort(self, a, axis=-1, **kw):
        r = np.argsort(a, axis=axis, kind="stable")
        self.calls.append(r)
        return r

    def zeros_like(self, *a, **kw):
        r = np.zeros_like(*a, **kw)
        self.zeros_like_out.append(r)
        return r


def _with_stable(mod, fn, *args, **kw):
    proxy = _StableNp()
    saved = mod.np
    mod.np = proxy
    try:
        return fn(*args, **kw), proxy
    finally:
        mod.np = saved


def backend_fixtures(out):
    torch.manual_seed(0)
    # config 1: 100 q x 500 g, D=1280 (BASELINE.json configs[0])
    Q, G, D = 100, 500, 1280
    qp, gp, qc, gc = syn.labels(Q, G, num_ids=60, num_cams=6, seed=1, distractor_frac=0.1, junk_frac=0.04)
    qf, gf = syn.features(qp, gp, dim=D, seed=1, noise=4.0)
    feats = torch.nn.functional.normalize(torch.from_numpy(np.concatenate([qf, gf])), dim=1, p=2)
    qn, gn = feats[:Q], feats[Q:]
    dist = ref_eval.euclidean_distance(qn, gn)
    cmc_u, map_u = ref_eval.eval_func(dist, qp, gp, qc, gc, max_rank=50)
    (cmc_s, map_s), px = _with_stable(ref_eval, ref_eval.eval_func, dist, qp, gp, qc, gc, max_rank=50)
    rank50 = px.calls[0][:, :50].astype(np.int32)
    # R1_mAP_eval end to end (evaluate.py:91-135) from raw features
    ev = ref_eval.R1_mAP_eval(Q, max_rank=50, feat_norm=True)
    ev.reset()
    ev.update((torch.from_numpy(np.concatenate([qf, gf])), np.concatenate([qp, gp]), np.concatenate([qc, gc])))
    (cmc_e, map_e), _ = _with_stable(ref_eval, ev.compute)
    # cosine_similarity (evaluate.py:16-26)
    cos = ref_eval.cosine_similarity(torch.from_numpy(qf), torch.from_numpy(gf))
    # inputs are regenerated from seeds (synthetic.labels/features seed=1); only outputs stored
    np.savez_compressed(os.path.join(out, "backend_small.npz"), q_pids=qp, g_pids=gp,
                        q_cams=qc, g_cams=gc, distmat=dist,
                        cmc_unstable=cmc_u, map_unstable=np.float64(map_u), cmc_stable=cmc_s,
                        map_stable=np.float64(map_s), rank50_stable=rank50, cmc_r1map=cmc_e,
                        map_r1map=np.float64(map_e), cosine=cos)

    # tie-heavy distance matrix: quantised distances => many exact ties
    Qt, Gt = 60, 300
    qp2, gp2, qc2, gc2 = syn.labels(Qt, Gt, num_ids=30, num_cams=4, seed=2, distractor_frac=0.1)
    r = np.random.default_rng(2)
    dist_t = (np.round(r.random((Qt, Gt)) * 16) / 16).astype(np.float32)
    same = (qp2[:, None] == gp2[None, :])
    dist_t[same] = (np.round(r.random(same.sum()) * 6) / 16).astype(np.float32)
    (cmc_t, map_t), px = _with_stable(ref_eval, ref_eval.eval_func, dist_t, qp2, gp2, qc2, gc2, max_rank=20)
    np.savez_compressed(os.path.join(out, "backend_ties.npz"), distmat=dist_t, q_pids=qp2, g_pids=gp2,
                        q_cams=qc2, g_cams=gc2, cmc_stable=cmc_t, map_stable=np.float64(map_t),
                        rank20_stable=px.calls[0][:, :20].astype(np.int32))
    print("backend fixtures ok", map_s, map_u, map_t)


def rerank_fixtures(out):
    Q, G, D = 100, 500, 1280
    qp, gp, qc, gc = syn.labels(Q, G, num_ids=60, num_cams=6, seed=3, distractor_frac=0.1)
    qf, gf = syn.features(qp, gp, dim=D, seed=3, noise=4.0)
    feats = torch.nn.functional.normalize(torch.from_numpy(np.concatenate([qf, gf])), dim=1, p=2)
    qn, gn = feats[:Q], feats[Q:]
    # a fixed N x N distance matrix, produced by the reference's own distance code
    dist_all = ref_eval.euclidean_distance(feats, feats)
    res = dict(q_pids=qp, g_pids=gp, q_cams=qc, g_cams=gc, dist_all=dist_all)
    for (k1, k2, lam) in ((50, 15, 0.3), (20, 6, 0.3)):
        tag = f"k{k1}_{k2}"
        # (a) stages R2..R7 from a given distance matrix (reranking.py:29-35 only_local path)
        final, px = _with_stable(ref_rr, ref_rr.re_ranking, qn, gn, k1, k2, lam,
                                 local_distmat=dist_all, only_local=True)
        res[f"final_{tag}"] = final
        res[f"initial_rank_{tag}"] = px.calls[0][:, :k1 + 1].astype(np.int32)
        # zeros_like outputs in call order (reranking.py:47,74,84): V's fp32 seed, V_qe, jaccard_dist
        res[f"vqe_{tag}"] = np.ascontiguousarray(px.zeros_like_out[1]).view(np.uint16)
        res[f"jaccard_{tag}"] = np.ascontiguousarray(px.zeros_like_out[2]).view(np.uint16)
        cmc, mAP = ref_eval.eval_func(final, qp, gp, qc, gc, max_rank=50)
        res[f"cmc_{tag}"] = cmc
        res[f"map_{tag}"] = np.float64(mAP)
        # (b) the full path from features (torch addmm distance inside reranking.py:36-41)
        full, _ = _with_stable(ref_rr, ref_rr.re_ranking, qn, gn, k1, k2, lam)
        res[f"final_full_{tag}"] = full
        print("rerank", tag, "mAP", mAP)
    np.savez_compressed(os.path.join(out, "rerank_small.npz"), **res)


def _load_vit(sd, model="ViT-B/16", height=256, width=128, stride=12):
    spec = syn.VIT_SPECS[model]
    gh, gw = syn.vit_grid(height, width, stride, spec["patch"])
    m = ref_ccm.VisionTransformer(gh, gw, spec["patch"], stride, spec["width"], spec["layers"],
                                  spec["width"] // 64, spec["out_dim"])
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    return m.eval()


def vit_fixtures(out):
    torch.manual_seed(0)
    sd = syn.vit_state_dict("ViT-B/16", seed=0)
    m = _load_vit(sd)
    imgs = syn.images(3, seed=0)
    offs = syn.tta_offsets(3, seed=0)
    aug = syn.tta_images_np(imgs, offs)
    with torch.no_grad():
        x11, x12, xp = m(torch.from_numpy(imgs))
        a11, a12, ap = m(torch.from_numpy(aug))
        # the reference's GPU dtype: conv/linear/MHA/proj in fp16, LN upcast (utils.py:145-166)
        mh = _load_vit(sd)
        for mod in mh.modules():
            if isinstance(mod, (torch.nn.Conv2d, torch.nn.Linear)):
                mod.weight.data = mod.weight.data.half()
                if mod.bias is not None:
                    mod.bias.data = mod.bias.data.half()
            if isinstance(mod, torch.nn.MultiheadAttention):
                mod.in_proj_weight.data = mod.in_proj_weight.data.half()
                mod.in_proj_bias.data = mod.in_proj_bias.data.half()
        mh.proj.data = mh.proj.data.half()
        mh.class_embedding.data = mh.class_embedding.data
        try:
            h11, h12, hp = mh(torch.from_numpy(imgs).half())
            half = dict(x12cls_fp16=h12[:, 0].float().numpy(), projcls_fp16=hp[:, 0].float().numpy())
        except Exception as e:  # fp16 conv may be unsupported on some CPU builds
            print("fp16 variant skipped:", e)
            half = {}
    np.savez_compressed(os.path.join(out, "vit_b16.npz"), tta_offsets=offs,
                        x11cls=x11[:, 0].numpy(), x12cls=x12[:, 0].numpy(), projcls=xp[:, 0].numpy(),
                        x12_tok=x12[0, :8].numpy(), x11_tok=x11[0, -4:].numpy(), proj_tok=xp[0, 100:104].numpy(),
                        tta_x12cls=a12[:, 0].numpy(), tta_projcls=ap[:, 0].numpy(), **half)
    print("vit fixtures ok")


def vitl_fixtures(out):
    """ViT-L/14 (configs[4]) as the reference executes it: resblocks[:11] + resblocks[11]
    (custom_clip_model.py:91-92), so a 12-layer state dict covers the executed path."""
    torch.manual_seed(0)
    sd = syn.vit_state_dict("ViT-L/14", seed=0, layers=12)
    spec = syn.VIT_SPECS["ViT-L/14"]
    gh, gw = syn.vit_grid(256, 128, 12, spec["patch"])
    m = ref_ccm.VisionTransformer(gh, gw, spec["patch"], 12, spec["width"], 12, spec["width"] // 64,
                                  spec["out_dim"])
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    m.eval()
    imgs = syn.images(2, seed=4)
    with torch.no_grad():
        x11, x12, xp = m(torch.from_numpy(imgs))
    np.savez_compressed(os.path.join(out, "vit_l14.npz"), x11cls=x11[:, 0].numpy(), x12cls=x12[:, 0].numpy(),
                        projcls=xp[:, 0].numpy(), x12_tok=x12[1, 200:204].numpy())
    print("vit-l fixtures ok")


class _FakeClip:
    """Holder with the attributes text_encoder.TextEncoder reads (text_encoder.py:6-12)."""


def text_fixtures(out):
    torch.manual_seed(0)
    sd = syn.text_state_dict(seed=0)
    spec = syn.TEXT_SPEC
    mask = torch.empty(spec["ctx"], spec["ctx"]).fill_(float("-inf")).triu_(1)  # maple.py:956-962
    tr = ref_ccm.Transformer(spec["width"], spec["layers"], spec["heads"], attn_mask=mask)
    tr.load_state_dict({k[len("transformer."):]: torch.from_numpy(v) for k, v in sd.items()
                        if k.startswith("transformer.")}, strict=True)
    c = _FakeClip()
    c.transformer = tr.eval()
    c.positional_embedding = torch.nn.Parameter(torch.from_numpy(sd["positional_embedding"]))
    c.ln_final = ref_ccm.LayerNorm(spec["width"])
    c.ln_final.weight.data = torch.from_numpy(sd["ln_final.weight"])
    c.ln_final.bias.data = torch.from_numpy(sd["ln_final.bias"])
    c.text_projection = torch.nn.Parameter(torch.from_numpy(sd["text_projection"]))
    c.dtype = torch.float32
    enc = ref_te.TextEncoder(c)
    tokens = syn.token_ids(6, seed=0)
    emb = torch.from_numpy(sd["token_embedding.weight"])[torch.from_numpy(tokens)]
    with torch.no_grad():
        feats = enc(emb, torch.from_numpy(tokens))
    np.savez_compressed(os.path.join(out, "text.npz"), tokens=tokens, text_feat=feats.numpy())
    print("text fixtures ok")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=HERE)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    todo = a.only.split(",") if a.only else ["backend", "rerank", "vit", "vitl", "text"]
    for t in todo:
        globals()[f"{t}_fixtures"](a.out)
