"""Host side of the CLIP-ReID encoders: weight packing into the libreidmi C structs
and the reference's model duck types.

    VisionTransformer.encode_image(img) -> (x11, x12, xproj)   custom_clip_model.py:77-100
                                                               maple.py:754-785 (IVLP, n_ctx>0)
    VisionTransformer.encode_cls(img, tta=None) -> (x12[:,0], xproj[:,0])  (inference fast path)
    TextTransformer.encode_text(tokens) -> (N, E)              maple.py:971-984
    TextEncoder(text)(prompts, tokenized_prompts) -> (N, E)    text_encoder.py:14-24
    CLIP(visual, text): encode_image / encode_text / dtype      maple.py:964-984

Weights come from a state dict with the reference's key layout (numpy or torch, fp32/fp16):
the vision keys of custom_clip_model.VisionTransformer (``conv1.weight``,
``transformer.resblocks.{i}.attn.in_proj_weight``, ... ``proj``; plus ``VPT`` /
``VPT_shallow`` for IVLP) and the text keys of CLIP (``token_embedding.weight``,
``transformer.resblocks.{i}...``, ``ln_final.*``, ``text_projection``).  Matrices are
stored fp16 in HBM (the reference's GPU dtype, utils.py:145-166), vectors fp32.  The packing
itself (LayerNorm folds, fp16 casts, transposes) is libreidmi's C ABI
(reidmi_vit_weights_pack / reidmi_text_weights_pack, pack.hip): this module only moves the
checkpoint's fp32 tensors to the device in the reference's key layout and hands them over, so
a non-Python caller packs the same bytes.  All compute runs in libreidmi.so.
"""
import ctypes

import numpy as np
import torch

from . import _lib

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32


class BlockWeights(ctypes.Structure):
    _fields_ = [(n, _vp) for n in ("ln1_w", "ln1_b", "qkv_w", "qkv_b", "out_w", "out_b", "ln2_w", "ln2_b",
                                   "fc1_w", "fc1_b", "fc2_w", "fc2_b", "prompt", "qkv_s", "fc1_s")]


class VitWeights(ctypes.Structure):
    _fields_ = [(n, _i32) for n in ("width", "layers", "heads", "patch", "stride", "out_dim", "grid_h", "grid_w",
                                    "n_ctx", "kpad")] + \
               [(n, _vp) for n in ("conv_w", "class_emb", "pos_emb", "ln_pre_w", "ln_pre_b", "ln_post_w",
                                   "ln_post_b", "proj_t", "vpt")] + [("blocks", ctypes.POINTER(BlockWeights))]


class TextWeights(ctypes.Structure):
    _fields_ = [(n, _i32) for n in ("width", "layers", "heads", "ctx", "vocab", "out_dim", "n_ctx")] + \
               [(n, _vp) for n in ("tok_emb", "pos_emb", "ln_final_w", "ln_final_b", "proj_t")] + \
               [("blocks", ctypes.POINTER(BlockWeights))]


class BlockSrc(ctypes.Structure):  # reidmi_block_src
    _fields_ = [(n, _vp) for n in ("ln_1_w", "ln_1_b", "in_proj_w", "in_proj_b", "out_proj_w", "out_proj_b", "ln_2_w",
                                   "ln_2_b", "c_fc_w", "c_fc_b", "c_proj_w", "c_proj_b", "vpt_shallow")]


class VitSrc(ctypes.Structure):  # reidmi_vit_src
    _fields_ = [(n, _i32) for n in ("width", "layers", "patch", "stride", "out_dim", "grid_h", "grid_w", "n_ctx")] + \
               [(n, _vp) for n in ("conv1_w", "class_embedding", "positional_embedding", "ln_pre_w", "ln_pre_b",
                                   "ln_post_w", "ln_post_b", "proj", "vpt")] + [("blocks", ctypes.POINTER(BlockSrc))]


class TextSrc(ctypes.Structure):  # reidmi_text_src
    _fields_ = [(n, _i32) for n in ("width", "layers", "ctx", "vocab", "out_dim", "n_ctx")] + \
               [(n, _vp) for n in ("token_embedding", "positional_embedding", "ln_final_w", "ln_final_b",
                                   "text_projection")] + [("blocks", ctypes.POINTER(BlockSrc))]


_SIG = {
    "reidmi_vit_pack_bytes": ([ctypes.POINTER(VitSrc)], ctypes.c_int64),
    "reidmi_vit_weights_pack": ([ctypes.POINTER(VitSrc), _vp, ctypes.c_int64, ctypes.POINTER(VitWeights),
                                 ctypes.POINTER(BlockWeights), _vp], ctypes.c_int),
    "reidmi_text_pack_bytes": ([ctypes.POINTER(TextSrc)], ctypes.c_int64),
    "reidmi_text_weights_pack": ([ctypes.POINTER(TextSrc), _vp, ctypes.c_int64, ctypes.POINTER(TextWeights),
                                  ctypes.POINTER(BlockWeights), _vp], ctypes.c_int),
    "reidmi_vit_workspace_bytes": ([ctypes.POINTER(VitWeights), ctypes.c_int64, ctypes.c_int], ctypes.c_int64),
    "reidmi_vit_forward": ([ctypes.POINTER(VitWeights), _vp, ctypes.c_int, ctypes.c_int64, ctypes.c_int,
                            ctypes.c_int, _vp, ctypes.c_int, _vp, _vp, _vp, _vp, ctypes.c_int64, _vp], ctypes.c_int),
    "reidmi_text_workspace_bytes": ([ctypes.POINTER(TextWeights), ctypes.c_int64], ctypes.c_int64),
    "reidmi_text_forward": ([ctypes.POINTER(TextWeights), _vp, _vp, ctypes.c_int64, ctypes.c_int, _vp, _vp,
                             ctypes.c_int64, _vp], ctypes.c_int),
}


def _fn(name):
    L = _lib.load()
    f = getattr(L, name)
    if name in _SIG and getattr(f, "_reidmi_typed", None) is None:
        f.argtypes, f.restype = _SIG[name]
        f._reidmi_typed = True
    return f


def _t(a):
    if isinstance(a, torch.Tensor):
        return a.detach().float().cpu()
    return torch.from_numpy(np.asarray(a, dtype=np.float32))


class _Sources:
    """The checkpoint's tensors as contiguous device fp32 (the packer's inputs), kept alive
    until the packing calls are issued (stream-ordered: the caching allocator reuses a freed
    block only for later work on the same stream)."""

    def __init__(self, device):
        self.device = device
        self.keep = []

    def f32(self, a):
        t = _t(a).contiguous().to(self.device)
        self.keep.append(t)
        return t.data_ptr()


def fold_layernorm(w, b, gamma, beta):
    """Host restatement of the packer's LayerNorm fold (pack.hip fold_rows_kernel), for tests:
    LN(x) w^T + b = rstd (x w'^T - mean s) + b' with w' = fp16(fp32(w diag(gamma))) (torch's
    fp64 -> fp16 cast rounds through fp32), s_n = sum_k w'[n, k] (exact in fp64) and
    b' = fp32(b + w beta) with the fp64 products summed exactly (math.fsum).  Returns (w' fp16,
    s, b') as torch tensors."""
    import math
    w32, g32 = _t(w).numpy(), _t(gamma).numpy()
    wf = torch.from_numpy((w32 * g32[None, :]).astype(np.float16))
    s = torch.from_numpy(wf.numpy().astype(np.float64).sum(1).astype(np.float32))
    prod = w32.astype(np.float64) * _t(beta).numpy().astype(np.float64)[None, :]
    bb = _t(b).numpy().astype(np.float64)
    bf = np.array([math.fsum([bb[n], *prod[n]]) for n in range(len(bb))], np.float64).astype(np.float32)
    return wf, s, torch.from_numpy(bf)


def _block_sources(sd, layers, src):
    arr = (BlockSrc * layers)()
    names = {"ln_1_w": "ln_1.weight", "ln_1_b": "ln_1.bias", "in_proj_w": "attn.in_proj_weight",
             "in_proj_b": "attn.in_proj_bias", "out_proj_w": "attn.out_proj.weight",
             "out_proj_b": "attn.out_proj.bias", "ln_2_w": "ln_2.weight", "ln_2_b": "ln_2.bias",
             "c_fc_w": "mlp.c_fc.weight", "c_fc_b": "mlp.c_fc.bias", "c_proj_w": "mlp.c_proj.weight",
             "c_proj_b": "mlp.c_proj.bias"}
    for i in range(layers):
        p = f"transformer.resblocks.{i}."
        for field, key in names.items():
            setattr(arr[i], field, src.f32(sd[p + key]))
        arr[i].vpt_shallow = src.f32(sd[p + "VPT_shallow"]) if (p + "VPT_shallow") in sd else None
    return arr


def _pack(kind, src_struct, layers, weights, device):
    """reidmi_{vit,text}_weights_pack into one device buffer; returns (buffer, host block array)."""
    nbytes = _fn(f"reidmi_{kind}_pack_bytes")(ctypes.byref(src_struct))
    if nbytes < 0:
        raise _lib.ReidmiError(f"reidmi_{kind}_pack_bytes: {_lib.load().reidmi_last_error().decode()}")
    buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)
    blocks = (BlockWeights * layers)()
    rc = _fn(f"reidmi_{kind}_weights_pack")(ctypes.byref(src_struct), buf.data_ptr(), nbytes, ctypes.byref(weights),
                                             blocks, _lib.stream(device))
    if rc != 0:
        raise _lib.ReidmiError(f"reidmi_{kind}_weights_pack: {_lib.load().reidmi_last_error().decode()}")
    weights.blocks = blocks
    return buf, blocks


def resize_pos_embed(posemb, gh, gw):
    """utils.py:111-125 / maple.py:1027-1041: bicubic resize of the square grid of a
    pretrained positional embedding to (gh, gw) (load time, host side)."""
    posemb = _t(posemb)
    tok, grid = posemb[:1], posemb[1:]
    gs = int(round(len(grid) ** 0.5))
    grid = grid.reshape(1, gs, gs, -1).permute(0, 3, 1, 2)
    grid = torch.nn.functional.interpolate(grid, size=(gh, gw), mode="bicubic")
    grid = grid.permute(0, 2, 3, 1).reshape(gh * gw, -1)
    return torch.cat([tok, grid], 0)


class VisionTransformer:
    """libreidmi vision tower.  ``stride`` defaults to the CLIP-ReID value 12
    (utils.py:169).  ``height``/``width`` are the input crop size (256x128)."""

    def __init__(self, state_dict, height=256, width=128, stride=12, device=None, prefix=""):
        sd = {k[len(prefix):]: v for k, v in state_dict.items() if k.startswith(prefix)}
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        conv = _t(sd["conv1.weight"])
        W, _, P, _ = conv.shape
        layers = len([k for k in sd if k.endswith(".attn.in_proj_weight")])
        self.width, self.layers, self.heads, self.patch, self.stride = W, layers, W // 64, P, stride
        self.out_dim = _t(sd["proj"]).shape[1]
        self.height, self.img_width = height, width
        gh, gw = (height - P) // stride + 1, (width - P) // stride + 1
        self.grid = (gh, gw)
        self.n_ctx = int(_t(sd["VPT"]).shape[0]) if "VPT" in sd else 0
        self.seq_len = 1 + gh * gw + self.n_ctx
        pos = _t(sd["positional_embedding"])
        if pos.shape[0] != 1 + gh * gw:
            pos = resize_pos_embed(pos, gh, gw)
        src = _Sources(self.device)
        vs = VitSrc()
        vs.width, vs.layers, vs.patch, vs.stride, vs.out_dim = W, layers, P, stride, self.out_dim
        vs.grid_h, vs.grid_w, vs.n_ctx = gh, gw, self.n_ctx
        vs.conv1_w = src.f32(conv)
        vs.class_embedding = src.f32(sd["class_embedding"])
        vs.positional_embedding = src.f32(pos)
        vs.ln_pre_w, vs.ln_pre_b = src.f32(sd["ln_pre.weight"]), src.f32(sd["ln_pre.bias"])
        vs.ln_post_w, vs.ln_post_b = src.f32(sd["ln_post.weight"]), src.f32(sd["ln_post.bias"])
        vs.proj = src.f32(sd["proj"])
        vs.vpt = src.f32(sd["VPT"]) if self.n_ctx else None
        bsrc = _block_sources(sd, layers, src)
        vs.blocks = bsrc
        self.weights = VitWeights()
        self._packed, self._blocks = _pack("vit", vs, layers, self.weights, self.device)
        del src
        self._ws = {}

    @property
    def dtype(self):
        return torch.float32

    def _workspace(self, B, full):
        """Workspace of the current stream (one per stream, so batches on several streams run
        concurrently; the caching allocator keeps each on its stream)."""
        nbytes = _fn("reidmi_vit_workspace_bytes")(ctypes.byref(self.weights), B, int(full))
        if nbytes < 0:
            raise _lib.ReidmiError(_lib.load().reidmi_last_error().decode())
        key = torch.cuda.current_stream(self.device).cuda_stream
        ws = self._ws.get(key)
        if ws is None or ws.numel() < nbytes:
            self._ws.pop(key, None)
            ws = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
            self._ws[key] = ws
        return ws, nbytes

    def _images(self, img):
        if not isinstance(img, torch.Tensor):
            img = torch.from_numpy(np.asarray(img))
        img = img.to(self.device)
        if img.dtype not in (torch.float32, torch.float16):
            img = img.float()
        return img.contiguous()

    def _run(self, img, tta, full, x12, proj, x11):
        img = self._images(img)
        B, C, H, Wd = img.shape
        if C != 3:
            raise ValueError("expected (B,3,H,W) images")
        ws, nbytes = self._workspace(B, full)
        if tta is not None:
            tta = torch.as_tensor(tta, dtype=torch.int32).to(self.device).contiguous()
        rc = _fn("reidmi_vit_forward")(ctypes.byref(self.weights), img.data_ptr(), int(img.dtype == torch.float16),
                                       B, H, Wd, None if tta is None else tta.data_ptr(), int(full),
                                       x12.data_ptr(), proj.data_ptr(), None if x11 is None else x11.data_ptr(),
                                       ws.data_ptr(), nbytes, _lib.stream(self.device))
        if rc != 0:
            raise _lib.ReidmiError(f"reidmi_vit_forward: {_lib.load().reidmi_last_error().decode()}")

    def encode_image(self, img):
        """(x11, x12, xproj), each [B, L, *] fp32 — custom_clip_model.py:100."""
        B = img.shape[0]
        L, W, E = self.seq_len, self.width, self.out_dim
        kw = dict(device=self.device, dtype=torch.float32)
        x11, x12, xp = torch.empty(B, L, W, **kw), torch.empty(B, L, W, **kw), torch.empty(B, L, E, **kw)
        self._run(img, None, True, x12, xp, x11)
        return x11, x12, xp

    __call__ = encode_image

    def encode_cls(self, img, tta=None, out_x12=None, out_proj=None):
        """(x12[:,0], xproj[:,0]) of encode_image(img) (or of the augmented view when
        ``tta`` [B,2] crop offsets are given) — what zero_shot_learning.py:85-87 consumes."""
        B = img.shape[0]
        kw = dict(device=self.device, dtype=torch.float32)
        x12 = out_x12 if out_x12 is not None else torch.empty(B, self.width, **kw)
        xp = out_proj if out_proj is not None else torch.empty(B, self.out_dim, **kw)
        self._run(img, tta, False, x12, xp, None)
        return x12, xp


class TextTransformer:
    """libreidmi text tower (CLIP.encode_text, maple.py:971-984; TextEncoder,
    text_encoder.py:14-24)."""

    def __init__(self, state_dict, device=None, prefix=""):
        sd = {k[len(prefix):]: v for k, v in state_dict.items() if k.startswith(prefix)}
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        tok = _t(sd["token_embedding.weight"])
        pos = _t(sd["positional_embedding"])
        W = tok.shape[1]
        layers = len([k for k in sd if k.startswith("transformer.") and k.endswith(".attn.in_proj_weight")])
        self.width, self.layers, self.heads, self.ctx, self.vocab = W, layers, W // 64, pos.shape[0], tok.shape[0]
        self.out_dim = _t(sd["text_projection"]).shape[1]
        vp = [k for k in sd if k.endswith("VPT_shallow")]
        self.n_ctx = int(_t(sd[vp[0]]).shape[0]) if vp else 0
        # fp32 copies for the prompt learners' token lookups (prompts.py) and TextEncoder
        self.token_embedding_weight = _t(tok).contiguous().to(self.device)
        self.positional_embedding = _t(pos).contiguous().to(self.device)
        src = _Sources(self.device)
        ts = TextSrc()
        ts.width, ts.layers, ts.ctx, ts.vocab, ts.out_dim, ts.n_ctx = (W, layers, pos.shape[0], tok.shape[0],
                                                                       self.out_dim, self.n_ctx)
        ts.token_embedding = self.token_embedding_weight.data_ptr()
        ts.positional_embedding = self.positional_embedding.data_ptr()
        ts.ln_final_w, ts.ln_final_b = src.f32(sd["ln_final.weight"]), src.f32(sd["ln_final.bias"])
        ts.text_projection = src.f32(sd["text_projection"])
        bsrc = _block_sources(sd, layers, src)
        ts.blocks = bsrc
        self.weights = TextWeights()
        self._packed, self._blocks = _pack("text", ts, layers, self.weights, self.device)
        del src
        self._ws = None
        # run on the positions up to the last EOT of the batch only (exact: causal mask,
        # reidmi_text_forward's ctx_used); False = all ctx positions, as the reference does
        self.trim_context = True

    def token_embedding(self, tokens):
        """nn.Embedding lookup (device) — used by prompt learners to build prompts."""
        return self.token_embedding_weight[torch.as_tensor(tokens, device=self.device).long()]

    def ctx_used(self, tokens):
        """Positions the batch needs: 1 + the largest EOT position (tokens.argmax(-1), the
        row text_encoder.py:23 / maple.py:981 reads), and at least the IVLP prompt rows."""
        if not self.trim_context or tokens.shape[0] == 0:
            return 0
        last = int(tokens.argmax(-1).max())  # one host sync when tokens are on the device
        return max(last + 1, self.n_ctx + 1)

    def _forward(self, tokens, prompts):
        tokens = torch.as_tensor(tokens)
        if tokens.dim() != 2 or tokens.shape[1] != self.ctx:
            raise ValueError(f"tokens must be [N, {self.ctx}]")
        used = self.ctx_used(tokens)
        tokens = tokens.to(self.device, torch.int64).contiguous()
        N = tokens.shape[0]
        nbytes = _fn("reidmi_text_workspace_bytes")(ctypes.byref(self.weights), N)
        if self._ws is None or self._ws.numel() < nbytes:
            self._ws = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        out = torch.empty(N, self.out_dim, device=self.device, dtype=torch.float32)
        if prompts is not None:
            prompts = prompts.to(self.device, torch.float32).contiguous()
        rc = _fn("reidmi_text_forward")(ctypes.byref(self.weights), tokens.data_ptr(),
                                        None if prompts is None else prompts.data_ptr(), N, used, out.data_ptr(),
                                        self._ws.data_ptr(), nbytes, _lib.stream(self.device))
        if rc != 0:
            raise _lib.ReidmiError(f"reidmi_text_forward: {_lib.load().reidmi_last_error().decode()}")
        return out

    def encode_text(self, text):
        return self._forward(text, None)


class TextEncoder:
    """text_encoder.TextEncoder over a TextTransformer: forward(prompts, tokenized_prompts)."""

    def __init__(self, text_model):
        self.text = text_model
        self.positional_embedding = text_model.positional_embedding
        self.dtype = torch.float32

    def __call__(self, prompts, tokenized_prompts):
        tok = torch.as_tensor(tokenized_prompts)
        if tok.dim() == 2 and tok.shape[0] == 1 and prompts.shape[0] > 1:
            # one template's token row for every prompt: the reference's
            # x[arange(B), tokenized_prompts.argmax(-1)] broadcasts it (text_encoder.py:23)
            tok = tok.expand(prompts.shape[0], -1)
        return self.text._forward(tok, prompts)

    forward = __call__


class CLIP:
    """Minimal CLIP container with the reference's encode_image / encode_text."""

    def __init__(self, visual=None, text=None):
        self.visual = visual
        self.text = text

    @property
    def dtype(self):
        return torch.float32

    def encode_image(self, image):
        return self.visual.encode_image(image)

    def encode_text(self, text):
        return self.text.encode_text(text)

    def eval(self):
        return self
