"""GPU parity of the encoder kernels and towers (libreidmi) against the fp32 torch
restatement (oracle/vit_ref.py, itself pinned to the reference's outputs) and the
reference-generated fixtures.

Tolerances (fp16 MFMA operands, fp32 accumulation — the reference's own GPU dtype):
  * kernels vs a torch fp32 reference on the same fp16 operands: rel 2e-3 (fp16 outputs)
  * towers vs oracle with fp16 rounding at the same points: cosine >= 0.99999
  * towers vs the reference's fp32 outputs: max |err| <= 1.5 x the reference's own fp16-vs-fp32
    deviation on the same inputs (conftest.close_to_reference), cosine >= 0.99995
    (the reference's own fp16 GPU dtype deviates 0.007 on the same inputs)
"""
import numpy as np
import pytest
import torch

from multimodal_reid_amd import synthetic as syn
from oracle import vit_ref
from conftest import close_to_reference, golden

pytestmark = pytest.mark.gpu


def _lib():
    from multimodal_reid_amd import _lib
    return _lib


def _cos(a, b):
    a = np.asarray(a, np.float64).reshape(len(a), -1)
    b = np.asarray(b, np.float64).reshape(len(b), -1)
    return (a * b).sum(1) / np.linalg.norm(a, axis=1) / np.linalg.norm(b, axis=1)


def _gemm(L, epi, A, W, bias, out, rowstat=None, colsum=None, tile=None, walk=0):
    M, K = A.shape
    N = W.shape[0]
    if tile is None:
        L.call("reidmi_gemm_f16", epi, L.ptr(A), K, L.ptr(W), K, M, N, K, L.ptr(bias), L.ptr(rowstat), L.ptr(colsum),
               L.ptr(out), out.shape[1], L.stream())
    else:  # per-call tiling (every choice bit-identical)
        L.call_tools("reidmi_gemm_f16_tiled", epi, L.ptr(A), K, L.ptr(W), K, M, N, K, L.ptr(bias), L.ptr(rowstat),
               L.ptr(colsum), L.ptr(out), out.shape[1], tile, walk, L.stream())


@pytest.mark.parametrize("epi", [0, 1, 5, 6])
@pytest.mark.parametrize("M,N,K", [(300, 256, 192), (1, 128, 64), (1000, 768, 768)])
def test_gemm_epilogues(gpu, epi, M, N, K):
    """fp16 operands, fp32 accumulation: against torch fp32 on the same fp16 values."""
    L = _lib()
    g = torch.Generator().manual_seed(M + N + K + epi)
    A = torch.randn(M, K, generator=g).half()
    W = (torch.randn(N, K, generator=g) / K ** 0.5).half()
    bias = torch.randn(N, generator=g)
    ref = A.float() @ W.float().t() + bias
    base = torch.randn(M, N, generator=g).half()
    if epi == 6:
        out = base.clone().cuda()
    else:
        out = torch.empty(M, N, dtype=torch.float32 if epi == 5 else torch.float16, device="cuda")
    _gemm(L, epi, A.cuda(), W.cuda(), bias.cuda(), out)
    got = out.float().cpu()
    if epi == 1:
        ref = ref * torch.sigmoid(1.702 * ref)
    if epi == 6:
        ref = ref + base.float()
    tol = 1e-5 if epi == 5 else 2e-3  # fp16 outputs carry their own rounding
    assert (got - ref).abs().max() <= tol * (ref.abs().max() + 1)


@pytest.mark.parametrize("epi", [0, 1, 5, 6])
@pytest.mark.parametrize("M,N,K", [(54016, 768, 768), (1000, 2304, 768), (700, 512, 3072), (70000, 256, 192),
                                   (40000, 3072, 768)])
def test_gemm_tiles_and_walks_bitexact(gpu, epi, M, N, K):
    """The 128x128 register-staged tile and the persistent 256x256 LDS-DMA tile (every
    XCD tile walk: 1, 2, 4, 8 N-groups; odd K-step counts cross tiles with the stage parity
    flipped) run the same MFMA chain per output element, so they agree bit for bit; rows
    past M (clamped source rows) must not leak into the result."""
    L = _lib()
    g = torch.Generator().manual_seed(M + N + K + epi)
    A = torch.randn(M, K, generator=g).half().cuda()
    W = (torch.randn(N, K, generator=g) / K ** 0.5).half().cuda()
    bias = torch.randn(N, generator=g).cuda()
    outs = []
    for tile, walk in ((1, 1), (2, 1), (2, 2), (2, 4), (2, 8)):
        if epi == 6:
            out = torch.ones(M, N, dtype=torch.float16, device="cuda")
        else:
            out = torch.zeros(M, N, dtype=torch.float32 if epi == 5 else torch.float16, device="cuda")
        _gemm(L, epi, A, W, bias, out, tile=tile, walk=walk)
        outs.append(out)
    for o in outs[1:]:
        assert torch.equal(outs[0], o)
    rows = torch.arange(0, M, max(1, M // 97), device="cuda")
    ref = A[rows].float() @ W.float().t() + bias
    if epi == 1:
        ref = ref * torch.sigmoid(1.702 * ref)
    if epi == 6:
        ref = ref + 1
    assert (outs[1][rows].float() - ref).abs().max() <= 2e-3 * (ref.abs().max() + 1)


@pytest.mark.parametrize("epi", [0, 1])
@pytest.mark.parametrize("M,N,K", [(300, 256, 768), (70000, 768, 768), (5000, 3072, 1024)])
def test_gemm_f16_layernorm_fold(gpu, epi, M, N, K):
    """ln_1 / ln_2 folded into the fp16 QKV / c_fc GEMM (model.fold_layernorm + row statistics):
    epi(LN(x) W^T + b) against fp64 torch on the same fp16 x, rows with large means (the
    cancellation the fold must survive); both tilings and the grouped walk bit-identical."""
    from multimodal_reid_amd.model import fold_layernorm
    L = _lib()
    g = torch.Generator().manual_seed(M + N + K)
    x = (torch.randn(M, K, generator=g) * (0.5 + torch.rand(M, 1, generator=g) * 3)
         + torch.randn(M, 1, generator=g) * 8).half()
    gam, bet = 1 + 0.3 * torch.randn(K, generator=g), 0.2 * torch.randn(K, generator=g)
    W, b = torch.randn(N, K, generator=g) / K ** 0.5, 0.1 * torch.randn(N, generator=g)
    wf, cs, bf = fold_layernorm(W, b, gam, bet)
    xd = x.double()
    mean = xd.mean(1, keepdim=True)
    rstd = 1 / torch.sqrt(((xd - mean) ** 2).mean(1, keepdim=True) + 1e-5)
    rs = torch.cat([rstd, -mean * rstd], 1).float()
    rs = torch.cat([rs, torch.full((256, 2), float("nan"))]).contiguous()  # padded to whole tiles
    ref = ((xd - mean) * rstd * gam.double() + bet.double()) @ W.double().t() + b.double()
    if epi == 1:
        ref = ref * torch.sigmoid(1.702 * ref)
    dx, dw, dcs, dbf, drs = (t.cuda() for t in (x, wf, cs, bf, rs))
    outs = []
    for tile, walk in ((1, 1), (2, 1), (2, 4)):
        out = torch.zeros(M, N, dtype=torch.float16, device="cuda")
        _gemm(L, epi, dx, dw, dbf, out, drs, dcs, tile=tile, walk=walk)
        outs.append(out)
    for o in outs[1:]:
        assert torch.equal(outs[0], o)
    got = outs[0].double().cpu()
    assert (got - ref).abs().max() <= 2e-3 * (ref.abs().max() + 1)
    assert _cos(got.numpy(), ref.numpy()).min() >= 0.99999


@pytest.mark.parametrize("W", [512, 768, 1024])
@pytest.mark.parametrize("M,K_mult", [(300, 1), (1037, 4), (13, 1)])
def test_residual_partials_rowstats(gpu, W, M, K_mult):
    """The residual epilogue's 64-column LayerNorm partials (EpiArgs::pstat) combined by
    rowstat_combine_kernel (run_block's ln_1 / ln_2 statistics) equal a statistics pass over
    the same fp16 rows within a few ulp, for every width and ragged M."""
    L = _lib()
    g = torch.Generator(device="cuda").manual_seed(W + M)
    K = W * K_mult
    A = (torch.randn(M, K, device="cuda", generator=g) * 0.5).half()
    Wt = (torch.randn(W, K, device="cuda", generator=g) * K ** -0.5).half()
    bias = torch.randn(W, device="cuda", generator=g) * 0.1
    x = (torch.randn(M, W, device="cuda", generator=g) * 3 + 0.7).half()
    pst = torch.full((W // 64, M, 2), float("nan"), device="cuda")
    L.call("reidmi_gemm_f16_resid_partials", L.ptr(A), K, L.ptr(Wt), K, M, W, K, L.ptr(bias), L.ptr(x), W,
           L.ptr(pst), L.stream())
    st_p = torch.empty(M, 2, device="cuda")
    st_x = torch.empty(M + 256, 2, device="cuda")
    L.call("reidmi_row_stats_f16", None, M, W, W, L.ptr(pst), L.ptr(st_p), L.stream())
    L.call("reidmi_row_stats_f16", L.ptr(x), M, W, W, None, L.ptr(st_x), L.stream())
    torch.cuda.synchronize()
    assert torch.isfinite(pst).all()
    xf = x.double()  # the rows the residual GEMM updated in place
    mean, var = xf.mean(1), xf.var(1, unbiased=False)
    rstd = (var + 1e-5).rsqrt()
    want = torch.stack([rstd, -mean * rstd], 1).float()
    assert torch.allclose(st_p, st_x[:M], rtol=1e-5, atol=1e-6)
    assert torch.allclose(st_p, want, rtol=2e-5, atol=2e-6)
    # the partials themselves: per 64-column block sum and centred sum of squares
    blk = xf.view(M, W // 64, 64)
    s = blk.sum(2)
    m2 = ((blk - blk.mean(2, keepdim=True)) ** 2).sum(2)
    assert torch.allclose(pst[..., 0].double(), s.t(), rtol=1e-5, atol=1e-3)
    assert torch.allclose(pst[..., 1].double(), m2.t(), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("W", [512, 768, 1024])
def test_layernorm(gpu, W):
    L = _lib()
    x = torch.randn(333, W) * 3 + 1
    g, b = torch.randn(W), torch.randn(W)
    ref = torch.nn.functional.layer_norm(x, (W,), g, b, 1e-5)
    dx, dg, dbb = x.cuda(), g.cuda(), b.cuda()
    y32 = torch.empty(333, W, device="cuda")
    y16 = torch.empty(333, W, device="cuda", dtype=torch.float16)
    L.call("reidmi_layernorm", L.ptr(dx), 333, W, None, W, L.ptr(dg), L.ptr(dbb), 1e-5, L.ptr(y32), W, L.ptr(y16), W,
           L.stream())
    assert (y32.cpu() - ref).abs().max() < 1e-4 * ref.abs().max()
    assert (y16.float().cpu() - ref).abs().max() < 1e-3 * ref.abs().max()


@pytest.mark.parametrize("L,causal", [(211, False), (213, False), (77, True), (50, False), (256, True), (128, False),
                                      (193, False), (208, False), (209, False), (224, False)])
def test_mhsa(gpu, L, causal):
    lib = _lib()
    nseq, H = 3, 4
    lp = lib.load().reidmi_attn_lpad(L)
    g = torch.Generator().manual_seed(L)
    q = (torch.randn(nseq * H, L, 64, generator=g) * 2).half()
    k = (torch.randn(nseq * H, L, 64, generator=g) * 2).half()
    v = torch.randn(nseq * H, L, 64, generator=g).half()
    vt = torch.zeros(nseq * H, 64, lp, dtype=torch.float16)
    vt[:, :, :L] = v.transpose(1, 2)
    vt[:, :, L:] = float("nan")  # padding must never be read into the result
    o = torch.empty(nseq * L, H * 64, dtype=torch.float16, device="cuda")
    dq, dk, dvt = q.cuda(), k.cuda(), vt.cuda()
    lib.call("reidmi_mhsa_f16", lib.ptr(dq), lib.ptr(dk), lib.ptr(dvt), lib.ptr(o), nseq, L, H, int(causal),
             lib.stream())
    s = (q.float() @ k.float().transpose(1, 2)) * 0.125
    if causal:
        s = s + torch.full((L, L), float("-inf")).triu(1)
    p = torch.softmax(s, -1)
    ref = (p @ v.float()).reshape(nseq, H, L, 64).permute(0, 2, 1, 3).reshape(nseq * L, H * 64)
    got = o.float().cpu()
    assert torch.isfinite(got).all()
    assert (got - ref).abs().max() < 5e-3  # fp16 P and O (bf16 needed 3e-2)


@pytest.mark.parametrize("L,nseq,H", [(211, 300, 12), (211, 1, 12), (211, 21, 12), (211, 23, 12), (205, 40, 12),
                                      (208, 3, 4), (209, 100, 12), (212, 64, 16)])
def test_mhsa_rr_bitexact_vs_two_stage_kernel(gpu, L, nseq, H):
    """The round-robin vision kernel of the tools library (mhsa_rr_kernel: 8 waves walk (head,
    32-query block) units over three LDS slots, V^T rows of 212; reidmi_mhsa_f16_rr — round 6's
    A/B, measured no faster) against the product's two-stage kernel (reidmi_mhsa_f16,
    V^T rows of reidmi_attn_lpad(L)): the same bits for every output.  Head counts below, at and
    above one per CU and workgroup sequences of 1-15 heads, so every load path of its schedule
    runs (the prologue's two heads, the shared prefetch, wave 0's refill of a slot its own last
    unit just read, idle waves in a partial last round); NaN in every V^T padding column."""
    from multimodal_reid_amd import _lib as L_
    lp = L_.load().reidmi_attn_lpad(L)
    g = torch.Generator(device="cuda").manual_seed(L * 7 + nseq)
    n = nseq * H
    q = (torch.randn(n, L, 64, generator=g, device="cuda") * 2).half()
    k = (torch.randn(n, L, 64, generator=g, device="cuda") * 2).half()
    v = torch.randn(n, L, 64, generator=g, device="cuda").half()
    vt_rr = torch.full((n, 64, 212), float("nan"), dtype=torch.float16, device="cuda")
    vt_rr[:, :, :L] = v.transpose(1, 2)
    vt = torch.full((n, 64, lp), float("nan"), dtype=torch.float16, device="cuda")
    vt[:, :, :L] = v.transpose(1, 2)
    o_rr = torch.full((nseq * L, H * 64), float("nan"), dtype=torch.float16, device="cuda")
    o = torch.full((nseq * L, H * 64), float("nan"), dtype=torch.float16, device="cuda")
    L_.call_tools("reidmi_mhsa_f16_rr", L_.ptr(q), L_.ptr(k), L_.ptr(vt_rr), L_.ptr(o_rr), nseq, L, H, L_.stream())
    L_.call("reidmi_mhsa_f16", L_.ptr(q), L_.ptr(k), L_.ptr(vt), L_.ptr(o), nseq, L, H, 0, L_.stream())
    torch.cuda.synchronize()
    assert torch.isfinite(o).all()
    assert torch.equal(o_rr.view(torch.int16), o.view(torch.int16))


@pytest.mark.parametrize("M,N,K", [(3000, 768, 3072), (513, 2304, 768), (256, 256, 128)])
def test_gemm_w4_prototype_bitexact(gpu, M, N, K):
    """The one-wave-per-SIMD GEMM prototype of the tools library gives the shipped
    persistent kernel's bits (same MFMA chain per element), partial last row tiles included."""
    from multimodal_reid_amd import _lib as L
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    A = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).half()
    W = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) / K ** 0.5).half()
    b = torch.rand(N, device="cuda", generator=g)
    o1 = torch.empty(M, N, device="cuda", dtype=torch.float16)
    o2 = torch.full((M, N), float("nan"), device="cuda", dtype=torch.float16)
    L.call_tools("reidmi_gemm_f16_tiled", 0, L.ptr(A), K, L.ptr(W), K, M, N, K, L.ptr(b), None, None, L.ptr(o1), N, 2,
                 0, L.stream())
    L.call_tools("reidmi_gemm_f16_w4", L.ptr(A), K, L.ptr(W), K, M, N, K, L.ptr(b), L.ptr(o2), N, 0, L.stream())
    assert torch.equal(o1, o2)


@pytest.mark.parametrize("L,causal,nseq,H", [(20, True, 700, 8), (50, True, 700, 8), (77, True, 500, 8),
                                            (128, True, 300, 8), (211, False, 300, 12)])
def test_mhsa_many_heads(gpu, L, causal, nseq, H):
    """More (sequence, head) pairs than the persistent grid has workgroups, so every workgroup
    walks several heads: the prefetch rings (three LDS stages for the causal text shapes,
    NKB 1-4; the pipelined two-stage vision kernel) rotate and their counted waits are
    exercised.  Reference: torch fp32 softmax attention on the device, same bound as test_mhsa."""
    lib = _lib()
    lp = lib.load().reidmi_attn_lpad(L)
    g = torch.Generator(device="cuda").manual_seed(1000 + L)
    n = nseq * H
    q = (torch.randn(n, L, 64, generator=g, device="cuda") * 2).half()
    k = (torch.randn(n, L, 64, generator=g, device="cuda") * 2).half()
    v = torch.randn(n, L, 64, generator=g, device="cuda").half()
    vt = torch.full((n, 64, lp), float("nan"), dtype=torch.float16, device="cuda")
    vt[:, :, :L] = v.transpose(1, 2)
    o = torch.empty(nseq * L, H * 64, dtype=torch.float16, device="cuda")
    lib.call("reidmi_mhsa_f16", lib.ptr(q), lib.ptr(k), lib.ptr(vt), lib.ptr(o), nseq, L, H, int(causal),
             lib.stream())
    worst = 0.0
    for a in range(0, n, 512):  # reference in slices (fp32 scores of 512 heads at a time)
        z = min(n, a + 512)
        s = (q[a:z].float() @ k[a:z].float().transpose(1, 2)) * 0.125
        if causal:
            s = s + torch.full((L, L), float("-inf"), device="cuda").triu(1)
        ref = torch.softmax(s, -1) @ v[a:z].float()  # [heads, L, 64], head index = b * H + h
        b0, b1 = a // H, (z + H - 1) // H
        got = o.view(nseq, L, H, 64)[b0:b1].permute(0, 2, 1, 3).reshape(-1, L, 64)[a - b0 * H:z - b0 * H]
        assert torch.isfinite(got).all()
        worst = max(worst, float((got.float() - ref).abs().max()))
    assert worst < 5e-3, worst


@pytest.fixture(scope="module")
def vit_b16(gpu):
    from multimodal_reid_amd.model import VisionTransformer
    sd = syn.vit_state_dict("ViT-B/16", seed=0)
    return sd, VisionTransformer(sd)


def test_vit_b16_encode_image_vs_reference(vit_b16):
    sd, m = vit_b16
    g = golden("vit_b16.npz")
    imgs = syn.images(3, seed=0)
    x11, x12, xp = (t.cpu().numpy() for t in m.encode_image(torch.from_numpy(imgs)))
    assert x12.shape == (3, 211, 768) and xp.shape == (3, 211, 512) and x11.shape == (3, 211, 768)
    # bounded by the reference's own fp16 deviation on these inputs (x12cls 0.0071, projcls 0.0047;
    # the token rows and x11 against the x12cls deviation)
    close_to_reference(x12[:, 0], g, "x12cls")
    close_to_reference(xp[:, 0], g, "projcls")
    close_to_reference(x11[:, 0], g, "x11cls", via="x12cls")
    close_to_reference(x12[0, :8], g, "x12_tok", via="x12cls")
    close_to_reference(xp[0, 100:104], g, "proj_tok", via="projcls")
    with torch.no_grad():
        b11, b12, bp = vit_ref.vit_forward(sd, imgs, f16=True)
    assert _cos(x12[:, 0], b12[:, 0].numpy()).min() >= 0.99999
    assert _cos(xp[:, 0], bp[:, 0].numpy()).min() >= 0.99999


def test_vit_l14_encode_image_vs_reference(gpu):
    """ViT-L/14 (configs[4]): width 1024, 16 heads, patch 14 (im2col K 588 -> 640), the 12
    blocks the reference executes; same tolerances as ViT-B/16."""
    from multimodal_reid_amd.model import VisionTransformer
    g = golden("vit_l14.npz")
    sd = syn.vit_state_dict("ViT-L/14", seed=0, layers=12)
    m = VisionTransformer(sd)
    assert m.seq_len == 211 and m.width == 1024 and m.heads == 16
    imgs = syn.images(2, seed=4)
    x11, x12, xp = (t.cpu().numpy() for t in m.encode_image(torch.from_numpy(imgs)))
    # the reference's own fp16 deviation: x12cls 0.0105, projcls 0.0039
    close_to_reference(x12[:, 0], g, "x12cls")
    close_to_reference(xp[:, 0], g, "projcls")
    close_to_reference(x11[:, 0], g, "x11cls", via="x12cls")
    close_to_reference(x12[1, 200:204], g, "x12_tok", via="x12cls")
    c12, cp = m.encode_cls(torch.from_numpy(imgs))
    close_to_reference(c12.cpu().numpy(), g, "x12cls")
    close_to_reference(cp.cpu().numpy(), g, "projcls")
    with torch.no_grad():
        _, b12, bp = vit_ref.vit_forward(sd, imgs, f16=True)
    assert _cos(x12[:, 0], b12[:, 0].numpy()).min() >= 0.99999
    assert _cos(xp[:, 0], bp[:, 0].numpy()).min() >= 0.99999


def test_vit_cls_path_and_tta(vit_b16):
    sd, m = vit_b16
    g = golden("vit_b16.npz")
    imgs = torch.from_numpy(syn.images(3, seed=0))
    _, x12, xp = m.encode_image(imgs)
    c12, cp = m.encode_cls(imgs)
    # CLS path: the last block's Q / attention / MLP for the CLS row only, its attention
    # reassociated through the folded in_proj (no K / V: cls_attn_nokv) with fp32-exact
    # products: equal to the full path up to the fp16 roundings of K / V it skips.
    assert _cos(c12.cpu().numpy(), x12[:, 0].cpu().numpy()).min() >= 0.999999
    assert _cos(cp.cpu().numpy(), xp[:, 0].cpu().numpy()).min() >= 0.999999
    assert (c12 - x12[:, 0]).abs().max() < 5e-3 and (cp - xp[:, 0]).abs().max() < 5e-3
    close_to_reference(c12.cpu().numpy(), g, "x12cls")
    close_to_reference(cp.cpu().numpy(), g, "projcls")
    t12, tp = m.encode_cls(imgs, tta=g["tta_offsets"])  # augmented view built inside im2col
    close_to_reference(t12.cpu().numpy(), g, "tta_x12cls", via="x12cls")
    close_to_reference(tp.cpu().numpy(), g, "tta_projcls", via="projcls")
    aug = syn.tta_images_np(imgs.numpy(), g["tta_offsets"])
    a12, ap = m.encode_cls(torch.from_numpy(aug))
    assert torch.equal(a12, t12) and torch.equal(ap, tp)


@pytest.mark.parametrize("arch,gain,vpt", [("ViT-B/16", 1.0, 0), ("ViT-B/16", 4.0, 0), ("ViT-B/16", 1.0, 2),
                                            ("ViT-L/14", 1.0, 0)])
def test_cls_attention_without_kv_matches_kv_path(gpu, monkeypatch, arch, gain, vpt):
    """The last block's CLS attention reassociated through the folded in_proj (cls_attn_nokv:
    K and V never formed) against the K / V GEMM + single-query kernel path it replaced
    (REIDMI_CLS_KV=1): the same function, differing by the fp16 roundings of K and V the new path
    skips.  37 images (a partial last group of 16), ViT-B/16 at CLIP's init and the spread
    network, IVLP prompts (L = 213), ViT-L/14 (width 1024, 16 heads)."""
    from multimodal_reid_amd.model import VisionTransformer
    sd = syn.vit_state_dict(arch, seed=3, layers=12, resid_gain=gain, **({"vpt_ctx": vpt} if vpt else {}))
    m = VisionTransformer(sd)
    imgs = torch.from_numpy(syn.images(37, seed=9))
    assert m.seq_len == 211 + vpt
    monkeypatch.delenv("REIDMI_CLS_KV", raising=False)
    n12, np_ = (t.cpu().numpy() for t in m.encode_cls(imgs))
    monkeypatch.setenv("REIDMI_CLS_KV", "1")
    k12, kp = (t.cpu().numpy() for t in m.encode_cls(imgs))
    assert np.isfinite(n12).all() and np.isfinite(np_).all()
    assert _cos(n12, k12).min() >= 0.999995 and _cos(np_, kp).min() >= 0.999995
    scale = np.abs(k12).max()
    assert np.abs(n12 - k12).max() <= 2e-3 * scale, (np.abs(n12 - k12).max(), scale)


def test_vit_batch_invariance(vit_b16):
    """Each image's features are bit-identical whatever batch it is computed in."""
    sd, m = vit_b16
    imgs = torch.from_numpy(syn.images(70, seed=5))
    big12, bigp = m.encode_cls(imgs)
    for i in (0, 33, 69):
        s12, sp = m.encode_cls(imgs[i:i + 1])
        assert torch.equal(s12[0], big12[i]) and torch.equal(sp[0], bigp[i])


def test_vit_ivlp_prompts(gpu):
    """IVLP tower (maple.py:617-644,754-785): 2 VPT tokens, per-block overwrite."""
    from multimodal_reid_amd.model import VisionTransformer
    sd = syn.vit_state_dict("ViT-B/16", seed=4, vpt_ctx=2)
    m = VisionTransformer(sd)
    assert m.seq_len == 213
    imgs = syn.images(2, seed=4)
    _, x12, xp = m.encode_image(torch.from_numpy(imgs))
    with torch.no_grad():
        _, r12, rp = vit_ref.vit_forward(sd, imgs, f16=True)
    assert _cos(x12[:, 0].cpu().numpy(), r12[:, 0].numpy()).min() >= 0.99999
    assert _cos(xp.cpu().numpy().reshape(-1, 512), rp.numpy().reshape(-1, 512)).min() >= 0.9999


def test_text_encoder_vs_reference(gpu):
    from multimodal_reid_amd.model import TextTransformer, TextEncoder
    sd = syn.text_state_dict(seed=0)
    g = golden("text.npz")
    tm = TextTransformer(sd)
    out = tm.encode_text(torch.from_numpy(g["tokens"])).cpu().numpy()
    close_to_reference(out, g, "text_feat")  # the reference's fp16 deviation: 0.0056
    with torch.no_grad():
        ref = vit_ref.text_forward(sd, g["tokens"], f16=True).numpy()
    assert _cos(out, ref).min() >= 0.99995  # 12 causal blocks: bf16 rounding flips compound
    # TextEncoder(prompts, tokenized) == encode_text when prompts = token_embedding(tokens)
    te = TextEncoder(tm)
    prompts = tm.token_embedding(g["tokens"])
    out2 = te(prompts, torch.from_numpy(g["tokens"])).cpu().numpy()
    assert np.array_equal(out, out2)


@pytest.mark.parametrize("text_ctx", [0, 4])
def test_text_trimmed_context_bitexact(gpu, text_ctx):
    """ctx_used (the causal-mask trim to 1 + the batch's last EOT position) changes no bit of
    encode_text / TextEncoder, for token rows and for IVLP text prompts (maple.py:630-640);
    a row encoded alone (its own, shorter trim) equals the same row inside the batch."""
    from multimodal_reid_amd.model import TextTransformer, TextEncoder
    sd = syn.text_state_dict(seed=3, layers=4, text_ctx=text_ctx)
    tm = TextTransformer(sd)
    tok = syn.token_ids(24, seed=3, min_len=8, max_len=60)
    assert tm.ctx_used(torch.from_numpy(tok)) == int(tok.argmax(-1).max()) + 1 < 77
    trimmed = tm.encode_text(tok)
    tm.trim_context = False
    full = tm.encode_text(tok)
    assert torch.equal(trimmed, full)
    prompts = tm.token_embedding(tok)
    te = TextEncoder(tm)
    pf = te(prompts, torch.from_numpy(tok))
    tm.trim_context = True
    pt = te(prompts, torch.from_numpy(tok))
    assert torch.equal(pf, pt) and torch.equal(pt, trimmed)
    for i in (0, 5, 17):
        assert torch.equal(tm.encode_text(tok[i:i + 1])[0], trimmed[i])


def test_inference_glue(vit_b16):
    """zero_shot_learning.inference feature epilogue, non-mm and --mm (zero_shot_learning.py:85-128)."""
    from multimodal_reid_amd import zero_shot_learning as zsl
    sd, m = vit_b16
    imgs = torch.from_numpy(syn.images(5, seed=9))
    offs = syn.tta_offsets(5, seed=9)
    emb = zsl.embed_pair(m, imgs, tta=offs).cpu()
    a12, ap = m.encode_cls(imgs)
    b12, bp = m.encode_cls(imgs, tta=offs)
    ref = (torch.cat([a12, ap], 1) + torch.cat([b12, bp], 1)).cpu() / 2
    assert torch.allclose(emb, ref, atol=1e-6)
    zs = torch.nn.functional.normalize(torch.randn(37, 512), dim=1)
    emb_mm = zsl.embed_pair(m, imgs, tta=offs, zeroshot_weights=zs, multimodal=True).cpu()
    p = (ap + bp).cpu() / 2
    p = p / p.norm(dim=-1, keepdim=True)
    logits = (1.0 / 0.07 * p @ zs.T).softmax(-1)
    ref_mm = torch.cat([(a12 + b12).cpu() / 2, logits], 1)
    assert emb_mm.shape == (5, 768 + 37)
    assert torch.allclose(emb_mm, ref_mm, atol=1e-5)


def _qkv_attention(L, nseq, W, fused, x, wq, bias, cs, rs):
    from multimodal_reid_amd import _lib as lib
    H = W // 64
    lp = lib.load().reidmi_attn_lpad(L)
    q = k = vt = None
    if not fused:
        q = torch.empty(nseq * H * L * 64, dtype=torch.float16, device="cuda")
        k = torch.empty_like(q)
        vt = torch.zeros(nseq * H * 64 * lp, dtype=torch.float16, device="cuda")
    o = torch.full((nseq * L, W), float("nan"), dtype=torch.float16, device="cuda")
    lib.call_tools("reidmi_qkv_attention_f16", lib.ptr(x), W, lib.ptr(wq), W, lib.ptr(bias), lib.ptr(cs), lib.ptr(rs), nseq,
             L, H, W, lib.ptr(q), lib.ptr(k), lib.ptr(vt), lib.ptr(o), int(fused), lib.stream())
    return o


@pytest.mark.parametrize("L,nseq,W", [(211, 37, 768), (213, 300, 768), (211, 23, 1024), (224, 5, 768), (193, 9, 768)])
def test_qkv_attention_fused_bitexact(gpu, L, nseq, W):
    """The fused QKV GEMM + attention kernel (q / k / v never leave the CU) equals the QKV
    GEMM (head-split epilogue) followed by the attention kernel bit for bit: the same MFMA
    chain per q / k / v element, the same fold / bias / RNE epilogue, the same attention code
    on the same operands.  Vision lengths (211, IVLP 213, ViT-L width 1024) and the ends of the
    fused kernel's range (193 and 224 tokens); unit counts that do not divide over the XCDs."""
    from multimodal_reid_amd.model import fold_layernorm
    g = torch.Generator().manual_seed(L * 7 + nseq + W)
    M = nseq * L
    x = (torch.randn(M, W, generator=g) * (0.5 + torch.rand(M, 1, generator=g)) + torch.randn(M, 1, generator=g)).half()
    gam, bet = 1 + 0.3 * torch.randn(W, generator=g), 0.2 * torch.randn(W, generator=g)
    Wi, bi = torch.randn(3 * W, W, generator=g) / W ** 0.5, 0.1 * torch.randn(3 * W, generator=g)
    wf, cs, bf = fold_layernorm(Wi, bi, gam, bet)
    xd = x.double()
    mean = xd.mean(1, keepdim=True)
    rstd = 1 / torch.sqrt(((xd - mean) ** 2).mean(1, keepdim=True) + 1e-5)
    rs = torch.cat([torch.cat([rstd, -mean * rstd], 1).float(), torch.zeros(256, 2)]).contiguous()
    args = [t.cuda() for t in (x, wf, bf, cs, rs)]
    fused = _qkv_attention(L, nseq, W, True, *args)
    ref = _qkv_attention(L, nseq, W, False, *args)
    assert torch.isfinite(ref).all()
    bad = (fused.view(torch.int16) != ref.view(torch.int16)).cpu()
    if bad.any():
        r, c = bad.nonzero(as_tuple=True)
        t = r % L
        diff = (fused.float() - ref.float()).abs().cpu()
        msg = (f"{int(bad.sum())}/{bad.numel()} differ, max |d| {float(diff.max()):.3g}; "
               f"tokens {sorted(set(t.tolist()))[:12]}, seqs {sorted(set((r // L).tolist()))[:8]}, "
               f"heads {sorted(set((c // 64).tolist()))[:12]}, dims {sorted(set((c % 64).tolist()))[:16]}")
        pytest.fail(msg)
