"""Floating-point oracle for the encoders: a plain-torch fp32 restatement of
  custom_clip_model.VisionTransformer.forward (custom_clip_model.py:57-100),
  maple.VisionTransformer IVLP prompts (maple.py:617-644, 754-785),
  CLIP.encode_text / TextEncoder.forward (maple.py:971-984, text_encoder.py:14-24),
over the same state-dict layout libreidmi packs.

TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py cpu_baseline leg).

``f16=True`` rounds to float16 exactly where the HIP kernels do — the out_proj / c_proj /
patch / proj GEMM operands, q/k/v, softmax probabilities before P.V, the attention and
QuickGELU outputs, the residual stream x (patch/CLS rows, ln_pre output, every residual
add) — and folds ln_1 / ln_2 into the fp16 QKV / c_fc GEMMs on x (`_ln_linear`), so tests
can separate kernel bugs from the precision the MI355X path runs at (fp16 operands, fp32
accumulation: the reference's own GPU dtype, utils.py:145-166).  With f16=False it is the
reference's fp32 math, pinned to tests/golden/vit_b16.npz, text.npz and ivlp.npz (made by
the reference modules).
"""
import numpy as np
import torch
import torch.nn.functional as F


def _t(a):
    return a.detach().float() if isinstance(a, torch.Tensor) else torch.from_numpy(np.asarray(a, np.float32))


def _h(x, on):
    return x.half().float() if on else x


_r = _h  # every rounded GEMM / attention operand is fp16


def _ln(x, w, b):
    return F.layer_norm(x, (x.shape[-1],), _t(w), _t(b), 1e-5)


def _ln_linear(x, g, beta, w, b, emulate):
    """LayerNorm(g, beta) then Linear(w, b).  emulate: as the kernels compute it — LN folded
    into an fp16 GEMM on the fp16 residual x: rstd * (x @ w'^T) - mean * rstd * s + b' with
    w' = fp16(w * g), s = row sums of w', b' = b + w @ beta (model.fold_layernorm)."""
    if not emulate:
        return _ln(x, g, beta) @ _t(w).t() + _t(b)
    W = x.shape[-1]
    mean = x.sum(-1, keepdim=True) / W
    var = ((x - mean) ** 2).sum(-1, keepdim=True) / W
    rstd = 1.0 / torch.sqrt(var + 1e-5)
    w64 = _t(w).double()
    wf = (w64 * _t(g).double()[None, :]).half()
    s = wf.double().sum(1).float()
    bf = (_t(b).double() + w64 @ _t(beta).double()).float()
    return rstd * (x @ wf.float().t()) + (-mean * rstd) * s + bf


def block(x, sd, p, heads, causal=False, f16=False):
    """ResidualAttentionBlock.forward (custom_clip_model.py:26-29) on x [B, L, W]."""
    B, L, W = x.shape
    qkv = _ln_linear(x, sd[p + "ln_1.weight"], sd[p + "ln_1.bias"], sd[p + "attn.in_proj_weight"],
                     sd[p + "attn.in_proj_bias"], f16)
    qkv = _r(qkv, f16).reshape(B, L, 3, heads, 64).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0], qkv[1], qkv[2]
    s = (q @ k.transpose(-1, -2)) * 0.125
    if causal:
        s = s + torch.full((L, L), float("-inf")).triu(1)
    m = s.amax(-1, keepdim=True)
    e = torch.exp(s - m)
    den = e.sum(-1, keepdim=True)
    o = (_r(e, f16) @ v) / den
    o = _r(o.permute(0, 2, 1, 3).reshape(B, L, W), f16)
    x = _h(x + (o @ _r(_t(sd[p + "attn.out_proj.weight"]), f16).t() + _t(sd[p + "attn.out_proj.bias"])), f16)
    u = _ln_linear(x, sd[p + "ln_2.weight"], sd[p + "ln_2.bias"], sd[p + "mlp.c_fc.weight"],
                   sd[p + "mlp.c_fc.bias"], f16)
    u = _r(u * torch.sigmoid(1.702 * u), f16)
    return _h(x + (u @ _r(_t(sd[p + "mlp.c_proj.weight"]), f16).t() + _t(sd[p + "mlp.c_proj.bias"])), f16)


def tta_view(img, offs):
    """data_prepare.py:263-270 on a normalised crop: flip, Pad((10,5)) (-1 fill), crop."""
    B, C, H, W = img.shape
    padded = torch.full((B, C, H + 10, W + 20), -1.0)
    padded[:, :, 5:5 + H, 10:10 + W] = img.flip(-1)
    return torch.stack([padded[b, :, int(offs[b][0]):int(offs[b][0]) + H, int(offs[b][1]):int(offs[b][1]) + W]
                        for b in range(B)])


def vit_forward(sd, img, stride=12, f16=False, tta=None):
    """(x11, x12, xproj) of the vision tower; img [B,3,H,W] fp32."""
    img = _t(img)
    if tta is not None:
        img = tta_view(img, tta)
    conv = _t(sd["conv1.weight"])
    W, _, P, _ = conv.shape
    B, _, H, Wd = img.shape
    gh, gw = (H - P) // stride + 1, (Wd - P) // stride + 1
    heads = W // 64
    cols = F.unfold(_r(img, f16), P, stride=stride).transpose(1, 2)  # [B, NP, 3PP] (c,ky,kx)
    x = cols @ _r(conv.reshape(W, -1), f16).t()
    pos = _t(sd["positional_embedding"])
    cls = (_t(sd["class_embedding"]) + pos[0]).expand(B, 1, W)
    x = _h(torch.cat([cls, x + pos[1:1 + gh * gw]], 1), f16)
    n_ctx = 0
    if "VPT" in sd:
        vpt = _t(sd["VPT"]).half().float()
        n_ctx = vpt.shape[0]
        x = torch.cat([x, vpt.expand(B, -1, -1)], 1)
    x = _h(_ln(x, sd["ln_pre.weight"], sd["ln_pre.bias"]), f16)
    L = x.shape[1]
    x11 = None
    for i in range(12):
        p = f"transformer.resblocks.{i}."
        if i > 0 and (p + "VPT_shallow") in sd:
            x = torch.cat([x[:, :L - n_ctx], _t(sd[p + "VPT_shallow"]).half().float().expand(B, -1, -1)], 1)
        x = block(x, sd, p, heads, False, f16)
        if i == 10:
            x11 = x
    x12 = _ln(x, sd["ln_post.weight"], sd["ln_post.bias"])
    xp = _r(x12, f16) @ _r(_t(sd["proj"]), f16)
    return x11, x12, xp


def text_forward(sd, tokens, prompts=None, f16=False):
    """CLIP.encode_text(tokens) or TextEncoder(prompts, tokens): [N, E]."""
    tokens = torch.as_tensor(np.asarray(tokens)).long()
    W = _t(sd["ln_final.weight"]).shape[0]
    heads = W // 64
    x = _t(sd["token_embedding.weight"])[tokens] if prompts is None else _t(prompts)
    x = _h(x + _t(sd["positional_embedding"]), f16)
    N, L, _ = x.shape
    layers = len([k for k in sd if k.startswith("transformer.") and k.endswith(".attn.in_proj_weight")])
    for i in range(layers):
        p = f"transformer.resblocks.{i}."
        if i > 0 and (p + "VPT_shallow") in sd:
            ctx = _t(sd[p + "VPT_shallow"]).half().float()
            x = torch.cat([x[:, :1], ctx.expand(N, -1, -1), x[:, 1 + ctx.shape[0]:]], 1)
        x = block(x, sd, p, heads, True, f16)
    x = _ln(x[torch.arange(N), tokens.argmax(-1)], sd["ln_final.weight"], sd["ln_final.bias"])
    return _r(x, f16) @ _r(_t(sd["text_projection"]), f16)


class FastVit:
    """The same fp32 math as vit_forward(f16=False) laid out the way the reference's modules run
    it on the CPU (custom_clip_model.py:57-100: Conv2d, nn.MultiheadAttention -> in_proj linear,
    scaled_dot_product_attention, out_proj; LayerNorm; QuickGELU), with the weights converted
    once to contiguous fp32 tensors.  bench.py's cpu_baseline times this: the CPU reference
    path's speed, not the emulation's (vit_forward re-reads the numpy state dict per op and
    runs the attention as explicit matmul/softmax)."""

    def __init__(self, sd, stride=12):
        self.w = {k: torch.from_numpy(np.ascontiguousarray(np.asarray(v, np.float32))) for k, v in sd.items()}
        self.stride = stride
        self.width = self.w["conv1.weight"].shape[0]
        self.heads = self.width // 64
        self.layers = len([k for k in sd if k.startswith("transformer.") and k.endswith(".attn.in_proj_weight")])

    @torch.inference_mode()
    def __call__(self, img, tta=None):
        w = self.w
        img = _t(img)
        if tta is not None:
            img = tta_view(img, tta)
        B = img.shape[0]
        x = F.conv2d(img, w["conv1.weight"], stride=self.stride)
        x = x.reshape(B, self.width, -1).permute(0, 2, 1)
        x = torch.cat([w["class_embedding"].expand(B, 1, -1), x], 1) + w["positional_embedding"]
        x = F.layer_norm(x, (self.width,), w["ln_pre.weight"], w["ln_pre.bias"], 1e-5)
        L, H = x.shape[1], self.heads
        x11 = None
        for i in range(12):
            p = f"transformer.resblocks.{i}."
            h = F.layer_norm(x, (self.width,), w[p + "ln_1.weight"], w[p + "ln_1.bias"], 1e-5)
            qkv = F.linear(h, w[p + "attn.in_proj_weight"], w[p + "attn.in_proj_bias"])
            q, k, v = qkv.reshape(B, L, 3, H, 64).permute(2, 0, 3, 1, 4)
            o = F.scaled_dot_product_attention(q, k, v).permute(0, 2, 1, 3).reshape(B, L, self.width)
            x = x + F.linear(o, w[p + "attn.out_proj.weight"], w[p + "attn.out_proj.bias"])
            h = F.layer_norm(x, (self.width,), w[p + "ln_2.weight"], w[p + "ln_2.bias"], 1e-5)
            u = F.linear(h, w[p + "mlp.c_fc.weight"], w[p + "mlp.c_fc.bias"])
            u = u * torch.sigmoid(1.702 * u)
            x = x + F.linear(u, w[p + "mlp.c_proj.weight"], w[p + "mlp.c_proj.bias"])
            if i == 10:
                x11 = x
        x12 = F.layer_norm(x, (self.width,), w["ln_post.weight"], w["ln_post.bias"], 1e-5)
        return x11, x12, x12 @ w["proj"]
