"""Deterministic synthetic inputs for tests, goldens and bench.

There are no datasets, checkpoints or BPE vocab in this environment (SURVEY.md
§0.6), so every parity fixture is built from the generators here:

* weights: per-tensor numpy PCG64 streams keyed by ``crc32(name) ^ seed``, with
  CLIP's initialisation scales (maple.py:915-935 ``initialize_parameters``,
  custom_clip_model.py:67-75).  Generating a tensor never depends on which other
  tensors were generated, so the GPU box regenerates exactly the weights the
  goldens were made with.
* images: U(-1, 1) crops, the post-``Normalize(0.5, 0.5)`` range of
  data_prepare.py:257-261.
* labels: Market/Duke/MSMT17-shaped pid/camid arrays.
* features: identity-clustered Gaussians for back-end-only runs.
"""
import zlib

import numpy as np

# (width, layers, heads, patch, out_dim) of the CLIP vision towers the
# reference builds (utils.py:184-195 derives them from checkpoint shapes).
VIT_SPECS = {
    "ViT-B/16": dict(width=768, layers=12, heads=12, patch=16, out_dim=512),
    "ViT-L/14": dict(width=1024, layers=24, heads=16, patch=14, out_dim=768),
}
TEXT_SPEC = dict(width=512, layers=12, heads=8, ctx=77, vocab=49408, out_dim=512)

DATASET_SPLITS = {  # SURVEY.md §8d; sizes from datasets/*.py docstrings
    "market1501": dict(num_query=3368, num_gallery=15913, num_ids=750, num_cams=6),
    "dukemtmc": dict(num_query=2228, num_gallery=17661, num_ids=1110, num_cams=8),
    "msmt17": dict(num_query=11659, num_gallery=82161, num_ids=3060, num_cams=15),
}


def _rng(name, seed):
    return np.random.Generator(np.random.PCG64((zlib.crc32(name.encode()) ^ (seed * 0x9E3779B1)) & 0xFFFFFFFF))


def _normal(name, shape, std, seed, mean=0.0):
    return (mean + std * _rng(name, seed).standard_normal(shape)).astype(np.float32)


def vit_grid(height, width, stride=12, patch=16):
    """Patch grid of the overlapping stride-12 conv (custom_clip_model.py:64-65)."""
    return (height - patch) // stride + 1, (width - patch) // stride + 1


def vit_state_dict(model="ViT-B/16", height=256, width=128, stride=12, seed=0, layers=None,
                   width_override=None, heads_override=None, vpt_ctx=0, resid_gain=1.0):
    """State dict (numpy fp32) with the key layout of custom_clip_model.VisionTransformer
    (and, with ``vpt_ctx>0``, the IVLP extras of maple.VisionTransformer: ``VPT`` and
    per-block ``VPT_shallow`` for blocks 1..L-1, maple.py:604-611,737-743).  ``resid_gain``
    scales the residual branches' output projections (attn.out_proj, mlp.c_proj): at CLIP's
    init (1.0) each block adds little to the residual stream, so the CLS output barely depends
    on the image (concentrated embeddings); a trained tower's blocks do not."""
    spec = dict(VIT_SPECS[model])
    if width_override:
        spec["width"] = width_override
    if heads_override:
        spec["heads"] = heads_override
    if layers is not None:
        spec["layers"] = layers
    w, L, P, E = spec["width"], spec["layers"], spec["patch"], spec["out_dim"]
    gh, gw = vit_grid(height, width, stride, P)
    scale = w ** -0.5
    attn_std = w ** -0.5
    proj_std = (w ** -0.5) * ((2 * L) ** -0.5) * resid_gain
    fc_std = (2 * w) ** -0.5
    sd = {}
    sd["conv1.weight"] = _normal("conv1.weight", (w, 3, P, P), (3 * P * P) ** -0.5, seed)
    sd["class_embedding"] = _normal("class_embedding", (w,), scale, seed)
    sd["positional_embedding"] = _normal("positional_embedding", (gh * gw + 1, w), scale, seed)
    for ln in ("ln_pre", "ln_post"):
        sd[f"{ln}.weight"] = _normal(f"{ln}.weight", (w,), 0.05, seed, mean=1.0)
        sd[f"{ln}.bias"] = _normal(f"{ln}.bias", (w,), 0.02, seed)
    for i in range(L):
        p = f"transformer.resblocks.{i}."
        sd[p + "attn.in_proj_weight"] = _normal(p + "attn.in_proj_weight", (3 * w, w), attn_std, seed)
        sd[p + "attn.in_proj_bias"] = _normal(p + "attn.in_proj_bias", (3 * w,), 0.02, seed)
        sd[p + "attn.out_proj.weight"] = _normal(p + "attn.out_proj.weight", (w, w), proj_std, seed)
        sd[p + "attn.out_proj.bias"] = _normal(p + "attn.out_proj.bias", (w,), 0.02, seed)
        for ln in ("ln_1", "ln_2"):
            sd[p + ln + ".weight"] = _normal(p + ln + ".weight", (w,), 0.05, seed, mean=1.0)
            sd[p + ln + ".bias"] = _normal(p + ln + ".bias", (w,), 0.02, seed)
        sd[p + "mlp.c_fc.weight"] = _normal(p + "mlp.c_fc.weight", (4 * w, w), fc_std, seed)
        sd[p + "mlp.c_fc.bias"] = _normal(p + "mlp.c_fc.bias", (4 * w,), 0.02, seed)
        sd[p + "mlp.c_proj.weight"] = _normal(p + "mlp.c_proj.weight", (w, 4 * w), proj_std, seed)
        sd[p + "mlp.c_proj.bias"] = _normal(p + "mlp.c_proj.bias", (w,), 0.02, seed)
        if vpt_ctx and i > 0:
            sd[p + "VPT_shallow"] = _normal(p + "VPT_shallow", (vpt_ctx, w), 0.02, seed)
    sd["proj"] = _normal("proj", (w, E), scale, seed)
    if vpt_ctx:
        sd["VPT"] = _normal("VPT", (vpt_ctx, w), 0.02, seed)
    return sd


def text_state_dict(seed=0, layers=None, vocab=None, text_ctx=0):
    """State dict (numpy fp32) for the CLIP text tower used by text_encoder.TextEncoder /
    CLIP.encode_text (maple.py:908-935, 971-984).  ``text_ctx>0`` adds IVLP per-block
    ``VPT_shallow`` (language_ctx, maple.py:604-608)."""
    s = dict(TEXT_SPEC)
    if layers is not None:
        s["layers"] = layers
    if vocab is not None:
        s["vocab"] = vocab
    w, L = s["width"], s["layers"]
    attn_std = w ** -0.5
    proj_std = (w ** -0.5) * ((2 * L) ** -0.5)
    fc_std = (2 * w) ** -0.5
    sd = {}
    sd["token_embedding.weight"] = _normal("token_embedding.weight", (s["vocab"], w), 0.02, seed)
    sd["positional_embedding"] = _normal("t.positional_embedding", (s["ctx"], w), 0.01, seed)
    for i in range(L):
        p = f"transformer.resblocks.{i}."
        q = "t." + p
        sd[p + "attn.in_proj_weight"] = _normal(q + "attn.in_proj_weight", (3 * w, w), attn_std, seed)
        sd[p + "attn.in_proj_bias"] = _normal(q + "attn.in_proj_bias", (3 * w,), 0.02, seed)
        sd[p + "attn.out_proj.weight"] = _normal(q + "attn.out_proj.weight", (w, w), proj_std, seed)
        sd[p + "attn.out_proj.bias"] = _normal(q + "attn.out_proj.bias", (w,), 0.02, seed)
        for ln in ("ln_1", "ln_2"):
            sd[p + ln + ".weight"] = _normal(q + ln + ".weight", (w,), 0.05, seed, mean=1.0)
            sd[p + ln + ".bias"] = _normal(q + ln + ".bias", (w,), 0.02, seed)
        sd[p + "mlp.c_fc.weight"] = _normal(q + "mlp.c_fc.weight", (4 * w, w), fc_std, seed)
        sd[p + "mlp.c_fc.bias"] = _normal(q + "mlp.c_fc.bias", (4 * w,), 0.02, seed)
        sd[p + "mlp.c_proj.weight"] = _normal(q + "mlp.c_proj.weight", (w, 4 * w), proj_std, seed)
        sd[p + "mlp.c_proj.bias"] = _normal(q + "mlp.c_proj.bias", (w,), 0.02, seed)
        if text_ctx and i > 0:
            sd[p + "VPT_shallow"] = _normal(q + "VPT_shallow", (text_ctx, w), 0.02, seed)
    sd["ln_final.weight"] = _normal("ln_final.weight", (w,), 0.05, seed, mean=1.0)
    sd["ln_final.bias"] = _normal("ln_final.bias", (w,), 0.02, seed)
    sd["text_projection"] = _normal("text_projection", (w, s["out_dim"]), w ** -0.5, seed)
    return sd


def images(n, height=256, width=128, seed=0, offset=0):
    """U(-1,1) float32 crops [n,3,H,W]; image k depends only on (seed, offset+k)."""
    out = np.empty((n, 3, height, width), np.float32)
    for k in range(n):
        out[k] = _rng(f"image{offset + k}", seed).uniform(-1.0, 1.0, (3, height, width)).astype(np.float32)
    return out


def tta_offsets(n, seed=0, offset=0):
    """Seeded RandomCrop offsets (top i in [0,10], left j in [0,20]) for the augmented
    loader (data_prepare.py:263-270: flip, Pad((10,5)), RandomCrop((H,W)))."""
    out = np.empty((n, 2), np.int32)
    for k in range(n):
        r = _rng(f"tta{offset + k}", seed)
        out[k, 0] = r.integers(0, 11)
        out[k, 1] = r.integers(0, 21)
    return out


def tta_images_np(imgs, offs):
    """Reference semantics of the augmented transform on an already-normalised crop:
    horizontal flip, zero-pad (10 left/right, 5 top/bottom) in pixel space == -1 after
    Normalize(0.5,0.5), crop at (i, j)."""
    n, c, h, w = imgs.shape
    flipped = imgs[..., ::-1]
    padded = np.full((n, c, h + 10, w + 20), -1.0, np.float32)
    padded[:, :, 5:5 + h, 10:10 + w] = flipped
    out = np.empty_like(imgs)
    for k in range(n):
        i, j = offs[k]
        out[k] = padded[k, :, i:i + h, j:j + w]
    return out


def labels(num_query, num_gallery, num_ids, num_cams, seed=0, distractor_frac=0.1, junk_frac=0.0):
    """pid/camid arrays shaped like a ReID test split.  Gallery: ids 1..num_ids plus
    distractor pid 0 (Market convention) and optional junk pid -1; queries use
    ids 1..num_ids only (queries never pid 0)."""
    r = _rng("labels", seed)
    n_dis = int(num_gallery * distractor_frac)
    n_junk = int(num_gallery * junk_frac)
    n_real = num_gallery - n_dis - n_junk
    g_pids = np.concatenate([1 + np.arange(n_real) % num_ids, np.zeros(n_dis, np.int64),
                             -np.ones(n_junk, np.int64)]).astype(np.int64)
    g_pids = g_pids[r.permutation(num_gallery)]
    g_cams = r.integers(0, num_cams, num_gallery).astype(np.int64)
    q_pids = (1 + r.integers(0, min(num_ids, max(n_real, 1)), num_query)).astype(np.int64)
    q_cams = r.integers(0, num_cams, num_query).astype(np.int64)
    return q_pids, g_pids, q_cams, g_cams


def features(q_pids, g_pids, dim=1280, seed=0, noise=4.0):
    """Identity-clustered Gaussian features (centre N(0,I), noise sigma), SURVEY.md §8d.
    pid <= 0 images get their own random centre."""
    r = _rng("features", seed)
    pids = np.concatenate([q_pids, g_pids])
    uniq = np.unique(pids[pids > 0])
    centres = {int(p): r.standard_normal(dim).astype(np.float32) for p in uniq}
    out = np.empty((len(pids), dim), np.float32)
    for k, p in enumerate(pids):
        c = centres[int(p)] if p > 0 else r.standard_normal(dim).astype(np.float32)
        out[k] = c + noise * r.standard_normal(dim).astype(np.float32)
    return out[:len(q_pids)], out[len(q_pids):]


def _upsample_rows_cols(a, H, W):
    """Separable linear interpolation (align_corners=True) of [..., h, w] to [..., H, W]."""
    h, w = a.shape[-2:]
    ys, xs = np.linspace(0, h - 1, H), np.linspace(0, w - 1, W)
    y0 = np.minimum(ys.astype(np.int64), h - 2)
    x0 = np.minimum(xs.astype(np.int64), w - 2)
    fy, fx = (ys - y0)[:, None], (xs - x0)[None, :]
    a = a.astype(np.float64)
    r = a[..., y0, :] * (1 - fy) + a[..., y0 + 1, :] * fy
    return r[..., x0] * (1 - fx) + r[..., x0 + 1] * fx


def identity_crops(pids, cams, seed=0, noise=0.6, detail=0.3, cast=0.02, shift=1, height=256, width=128,
                   offset=0):
    """Identity-structured synthetic crops for end-to-end accuracy parity: each pid > 0 has
    a smooth base image (a 16x8 U(-1,1) grid, linearly upsampled) plus a fixed high-frequency
    texture; each camera adds a colour cast and a horizontal shift; each image adds its own
    Gaussian noise.  pid <= 0 images (distractors / junk) get their own base.  Values are
    clipped to [-1, 1] (the post-Normalize range).  Image k depends only on
    (seed, pids[k], cams[k], offset + k)."""
    out = np.empty((len(pids), 3, height, width), np.float32)
    cache = {}

    def base(key):
        if key not in cache:
            r = _rng(f"idbase{key}", seed)
            b = _upsample_rows_cols(r.uniform(-1, 1, (3, 16, 8)), height, width)
            cache[key] = b + detail * r.uniform(-1, 1, (3, height, width))
        return cache[key]

    for k, (p, c) in enumerate(zip(pids, cams)):
        rk = _rng(f"idimg{offset + k}", seed)
        b = base(int(p)) if p > 0 else base(f"x{offset + k}")
        rc = _rng(f"idcam{int(c)}", seed)
        cc = cast * rc.standard_normal(3)[:, None, None]
        sh = int(rc.integers(-shift, shift + 1))
        img = np.roll(b, sh, axis=2) + cc + noise * rk.standard_normal((3, height, width))
        out[k] = np.clip(img, -1.0, 1.0).astype(np.float32)
    return out


def crop_rgb(h, w, seed=0, key=0, noise=12.0):
    """A decoded-photo-like RGB crop, uint8 [h][w][3]: a smooth random colour field (a coarse
    grid linearly upsampled), a few hard-edged rectangles and per-pixel noise."""
    r = _rng(f"crop{key}", seed)
    gh, gw = max(2, h // 24 + 2), max(2, w // 24 + 2)
    img = _upsample_rows_cols(r.uniform(0, 255, (3, gh, gw)), max(h, 2), max(w, 2))[:, :h, :w]
    for _ in range(3):
        y0, x0 = int(r.integers(0, h)), int(r.integers(0, w))
        img[:, y0:y0 + int(r.integers(1, h + 1)), x0:x0 + int(r.integers(1, w + 1))] = r.uniform(0, 255, (3, 1, 1))
    img = img + noise * r.standard_normal((3, h, w))
    return np.ascontiguousarray(np.clip(np.rint(img), 0, 255).astype(np.uint8).transpose(1, 2, 0))


def jpeg_files(n, h=128, w=64, seed=0, quality=90, subsampling=2, offset=0, **save_kw):
    """n JPEG files (bytes) of synthetic crops encoded by Pillow (libjpeg-turbo): Market-1501
    crops are 128 x 64 baseline JPEGs with 4:2:0 chroma (subsampling=2)."""
    import io

    from PIL import Image
    out = []
    for k in range(n):
        b = io.BytesIO()
        Image.fromarray(crop_rgb(h, w, seed, offset + k)).save(b, "JPEG", quality=quality, subsampling=subsampling,
                                                               **save_kw)
        out.append(b.getvalue())
    return out


def token_ids(n, ctx=77, vocab=49408, seed=0, min_len=4, max_len=20):
    """Synthetic CLIP token rows: SOT 49406, random body, EOT 49407 (the max id, so
    ``argmax`` finds it, text_encoder.py:23), zero padding."""
    r = _rng("tokens", seed)
    out = np.zeros((n, ctx), np.int64)
    for k in range(n):
        ln = int(r.integers(min_len, max_len + 1))
        out[k, 0] = vocab - 2
        out[k, 1:ln - 1] = r.integers(1, vocab - 2, ln - 2)
        out[k, ln - 1] = vocab - 1
    return out


def openai_state_dict(model="ViT-B/16", seed=0, vpt_ctx=0, text_ctx=0, input_res=224):
    """OpenAI-CLIP key layout (``visual.*`` + top-level text keys + ``logit_scale``) as
    maple.build_model (maple.py:1044-1098) consumes it: the vision tower at its
    pretraining resolution (square grid, e.g. 14x14 + 1 positional rows for ViT-B/16 at
    224), so build_model's bicubic resize to the stride-12 grid is exercised.  IVLP
    extras with ``vpt_ctx`` / ``text_ctx`` > 0 (``visual.VPT``,
    ``visual.transformer.resblocks.{i}.VPT_shallow``, ``transformer.resblocks.{i}.VPT_shallow``)."""
    P = VIT_SPECS[model]["patch"]
    vis = vit_state_dict(model, height=input_res, width=input_res, stride=P, seed=seed, vpt_ctx=vpt_ctx)
    sd = {"visual." + k: v for k, v in vis.items()}
    sd.update(text_state_dict(seed=seed, text_ctx=text_ctx))
    sd["logit_scale"] = np.array(np.log(1 / 0.07), np.float32)
    return sd


def clipreid_checkpoint(model="ViT-B/16", seed=0, height=256, width=128, stride=12, resid_gain=1.0):
    """CLIP-ReID checkpoint key layout that utils.model_adaptor reads (utils.py:184-221):
    ``image_encoder.*`` (the stride-12 vision tower), ``text_encoder.*`` (the text tower,
    zero_shot_learning.py:31-34) and the BNNeck ``bottleneck.*`` / ``bottleneck_proj.*``
    BatchNorm1d buffers (utils.py:128-142)."""
    vis = vit_state_dict(model, height=height, width=width, stride=stride, seed=seed, resid_gain=resid_gain)
    sd = {"image_encoder." + k: v for k, v in vis.items()}
    sd.update({"text_encoder." + k: v for k, v in text_state_dict(seed=seed).items()})
    W, E = VIT_SPECS[model]["width"], VIT_SPECS[model]["out_dim"]
    for name, n in (("bottleneck", W), ("bottleneck_proj", E)):
        sd[name + ".weight"] = _normal(name + ".weight", (n,), 0.05, seed, mean=1.0)
        sd[name + ".bias"] = np.zeros(n, np.float32)
        sd[name + ".running_mean"] = _normal(name + ".running_mean", (n,), 0.1, seed)
        sd[name + ".running_var"] = np.abs(_normal(name + ".running_var", (n,), 0.1, seed, mean=1.0))
        sd[name + ".num_batches_tracked"] = np.array(100, np.int64)
    return sd


_FP16_SUFFIXES = ("conv1.weight", "attn.in_proj_weight", "attn.in_proj_bias", "attn.out_proj.weight",
                  "attn.out_proj.bias", "mlp.c_fc.weight", "mlp.c_fc.bias", "mlp.c_proj.weight",
                  "mlp.c_proj.bias", "proj", "text_projection")


def round_like_convert_weights(sd):
    """The values convert_weights (utils.py:145-166, maple.py:992-1013) leaves in a model:
    Conv/Linear weights and biases, the MHA in_proj, ``proj`` and ``text_projection``
    rounded to fp16 (and back to fp32); LayerNorm, embeddings and prompts untouched."""
    out = {}
    for k, v in sd.items():
        if k.split(".")[-1] in ("proj", "text_projection") or k.endswith(_FP16_SUFFIXES[:-2]):
            v = np.asarray(v, np.float32).astype(np.float16).astype(np.float32)
        out[k] = v
    return out


def glue_cls_features(n, dim, seed=0):
    """[n, dim] fp32 stand-in CLS features for the inference() glue fixtures."""
    return _normal(f"glue{dim}", (n, dim), 1.0, seed)


# Synthetic token row standing in for clip.tokenize("A photo of X X X X X person.") (the BPE
# vocabulary is absent): SOT, 10 body ids, EOT (the row's maximum, argmax -> EOT), zero pad.
CTX_INIT_TOKENS = [49406, 320, 1125, 539, 343, 343, 343, 343, 343, 2533, 269, 49407]


def ctx_init_tokens(ctx=77):
    out = np.zeros((1, ctx), np.int64)
    out[0, :len(CTX_INIT_TOKENS)] = CTX_INIT_TOKENS
    return out


MARKET_ATTRIBUTE_FIELDS = (["age", "backpack", "bag", "handbag", "clothes", "down", "up", "hair", "hat", "gender"]
                           + ["up" + c for c in ("black", "white", "red", "purple", "yellow", "gray", "blue", "green")]
                           + ["down" + c for c in ("black", "white", "pink", "purple", "yellow", "gray", "blue",
                                                   "green", "brown")]
                           + ["image_index"])


def write_market_attribute_mat(path, n_ids=24, seed=0):
    """A synthetic Market-1501_Attribute/market_attribute.mat (the submodule is absent
    offline) with the layout data_prepare.get_prompts reads (data_prepare.py:296-309):
    market_attribute.{test,train} structs of 28 1 x n fields — age in 1..4, the other 26
    attributes in {1, 2}, image_index the identity strings."""
    import scipy.io as sio
    r = _rng("market_attribute", seed)
    d = {}
    for f in MARKET_ATTRIBUTE_FIELDS[:-1]:
        d[f] = r.integers(1, 5 if f == "age" else 3, (1, n_ids))
    idx = np.empty((1, n_ids), dtype=object)
    for i in range(n_ids):
        idx[0, i] = f"{i + 1:04d}"
    d["image_index"] = idx
    sio.savemat(path, {"market_attribute": {"test": d, "train": d}})
