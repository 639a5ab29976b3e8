"""GPU parity of the retrieval back end (libreidmi) against the oracle and the
reference-generated fixtures.  Integer/index outputs and exact-fp32 distances are
compared bit-for-bit."""
import numpy as np
import pytest
import torch

import oracle
from multimodal_reid_amd import synthetic as syn
from conftest import golden

pytestmark = pytest.mark.gpu


def _ev():
    from multimodal_reid_amd import evaluate
    return evaluate


def _inputs(seed=1, Q=100, G=500, D=1280, junk=0.04):
    qp, gp, qc, gc = syn.labels(Q, G, num_ids=60, num_cams=6, seed=seed, distractor_frac=0.1, junk_frac=junk)
    qf, gf = syn.features(qp, gp, dim=D, seed=seed, noise=4.0)
    return qf, gf, qp, gp, qc, gc


def test_l2norm_bitexact(gpu):
    qf, gf, *_ = _inputs()
    x = np.concatenate([qf, gf])
    y = _ev().l2_normalize_device(torch.from_numpy(x)).cpu().numpy()
    assert np.array_equal(y.view(np.uint32), oracle.l2norm(x).view(np.uint32))


@pytest.mark.parametrize("Q,G,D", [(100, 500, 1280), (37, 259, 768), (1, 1, 2), (130, 129, 1792), (5, 300, 513),
                                   (300, 700, 100), (1200, 257, 36)])  # row-norm tails; banded walk, partial band
def test_distmat_bitexact(gpu, Q, G, D):
    r = np.random.default_rng(Q * 7 + G)
    q = r.standard_normal((Q, D)).astype(np.float32)
    g = r.standard_normal((G, D)).astype(np.float32)
    ref = oracle.distmat(q, g).view(np.uint32)
    from multimodal_reid_amd import _lib
    d = _ev().euclidean_distance(torch.from_numpy(q), torch.from_numpy(g))
    assert isinstance(d, np.ndarray) and d.dtype == np.float32
    assert np.array_equal(d.view(np.uint32), ref)
    # per-call kernel choice: the pipelined K-step-32 kernel (D % 4 == 0) and the single-stage one
    qd, gd = torch.from_numpy(q).cuda(), torch.from_numpy(g).cuda()
    for v in (0, 1):
        out = torch.empty(Q, G, device="cuda")
        ws = torch.empty(Q + G, device="cuda")
        _lib.call_tools("reidmi_distmat_f32_variant", _lib.ptr(qd), Q, D, _lib.ptr(gd), G, D, D, _lib.ptr(out), G,
                  _lib.ptr(ws), v, _lib.stream())
        assert np.array_equal(out.cpu().numpy().view(np.uint32), ref), v


@pytest.mark.parametrize("Q,G,D", [(100, 500, 1280), (37, 259, 768), (1, 1, 2), (130, 129, 1792), (5, 300, 513),
                                   (700, 3000, 1280)])
def test_distmat_f16_mode_bound(gpu, Q, G, D):
    """The §8b reduced-precision mode (reidmi_distmat_f16): every entry within
    2^-8 ||q|| ||g|| of the exact distance (fp16 operands: 2^-11 relative per element, the
    dot's error <= 2^-10 ||q|| ||g|| by Cauchy-Schwarz, doubled by the -2 q.g term, plus fp32
    accumulation), on unnormalised and on L2-normalised rows; padding of D to the GEMM's K step
    and of G to its tile never leaks into the result."""
    r = np.random.default_rng(Q * 11 + G)
    q = r.standard_normal((Q, D)).astype(np.float32)
    g = r.standard_normal((G, D)).astype(np.float32)
    ev = _ev()
    for norm in (False, True):
        qd, gd = torch.from_numpy(q).cuda(), torch.from_numpy(g).cuda()
        if norm:
            qd, gd = ev.l2_normalize_device(qd), ev.l2_normalize_device(gd)
        exact = ev.euclidean_distance_device(qd, gd)
        low = ev.euclidean_distance_device(qd, gd, precision="fp16")
        bound = 2.0 ** -8 * qd.norm(dim=1)[:, None] * gd.norm(dim=1)[None, :] + 1e-6
        assert torch.isfinite(low).all()
        assert bool(((low - exact).abs() <= bound).all()), float(((low - exact).abs() / bound).max())
    with pytest.raises(ValueError):
        ev.euclidean_distance_device(qd, gd, precision="bf16")


@pytest.mark.parametrize("Q,G,D,pad", [(37, 259, 768, 0), (130, 1001, 1280, 3), (3000, 6007, 1280, 0)])
def test_distmat_f16_fused_equals_products_pass(gpu, Q, G, D, pad):
    """The fp16 mode's distances come out of the GEMM's epilogue: bit-identical to the plain
    fp32 products of the same GEMM (reidmi_gemm_f16, EPI_F32) finished as (||q||^2 + ||g||^2)
    - 2 dot in fp32 (the separate pass the epilogue replaced), for unaligned row pitches, ragged
    columns, partial tiles and the persistent tile (3000 x 6007); columns past G untouched."""
    from multimodal_reid_amd import _lib
    r = np.random.default_rng(Q + G)
    q = torch.from_numpy(r.standard_normal((Q, D)).astype(np.float32)).cuda()
    g = torch.from_numpy(r.standard_normal((G, D)).astype(np.float32)).cuda()
    out = torch.full((Q, G + pad), float("nan"), device="cuda")
    ws = torch.empty(_lib.load().reidmi_distmat_f16_workspace_bytes(Q, G, D), device="cuda", dtype=torch.uint8)
    _lib.call("reidmi_distmat_f16", _lib.ptr(q), Q, D, _lib.ptr(g), G, D, D, _lib.ptr(out), G + pad, _lib.ptr(ws),
              ws.numel(), _lib.stream())
    Dp, Gp = (D + 63) // 64 * 64, (G + 255) // 256 * 256
    qh = torch.zeros(Q, Dp, dtype=torch.float16, device="cuda")
    gh = torch.zeros(Gp, Dp, dtype=torch.float16, device="cuda")
    qh[:, :D], gh[:G, :D] = q.half(), g.half()
    dot = torch.empty(Q, Gp, device="cuda")
    _lib.call("reidmi_gemm_f16", 5, _lib.ptr(qh), Dp, _lib.ptr(gh), Dp, Q, Gp, Dp, None, None, None, _lib.ptr(dot),
              Gp, _lib.stream())
    qq, gg = torch.empty(Q, device="cuda"), torch.empty(G, device="cuda")
    _lib.call("reidmi_row_sqnorm_f32", _lib.ptr(q), Q, D, D, _lib.ptr(qq), _lib.stream())
    _lib.call("reidmi_row_sqnorm_f32", _lib.ptr(g), G, D, D, _lib.ptr(gg), _lib.stream())
    ref = (qq[:, None] + gg[None, :]) - 2.0 * dot[:, :G]
    assert torch.equal(out[:, :G].contiguous().view(torch.int32), ref.view(torch.int32))
    if pad:
        assert bool(torch.isnan(out[:, G:]).all())


def test_distmat_f16_mode_ranking(gpu):
    """mAP / rank-1 through the reduced-precision mode against the exact one on identity-clustered
    features of 800 q x 6000 g (normalised, as R1_mAP_eval feeds the distance): the retrieval
    metrics agree to 2e-3 (measured: profiles/r04/distmat_f16_mode.txt)."""
    ev = _ev()
    qf, gf, qp, gp, qc, gc = _inputs(seed=9, Q=800, G=6000, junk=0.02)
    qn = ev.l2_normalize_device(torch.from_numpy(qf).cuda())
    gn = ev.l2_normalize_device(torch.from_numpy(gf).cuda())
    res = {}
    for prec in ("fp32", "fp16"):
        d = ev.euclidean_distance_device(qn, gn, precision=prec)
        valid, first, ap, nkept, _ = ev.eval_rows_device(d, qp, gp, qc, gc)
        cmc, mAP = ev.aggregate_cmc_map(valid.cpu().numpy(), first.cpu().numpy(), ap.cpu().numpy(),
                                        nkept.cpu().numpy(), len(gp), 50)
        res[prec] = (float(cmc[0]), float(mAP))
    print("distmat modes (rank-1, mAP):", res)
    assert abs(res["fp16"][1] - res["fp32"][1]) <= 2e-3
    assert abs(res["fp16"][0] - res["fp32"][0]) <= 2e-3


def test_distmat_matches_reference_fixture(gpu):
    g = golden("backend_small.npz")
    qf, gf, *_ = _inputs()
    feats = torch.nn.functional.normalize(torch.from_numpy(np.concatenate([qf, gf])), dim=1, p=2)
    d = _ev().euclidean_distance(feats[:100], feats[100:])
    assert np.abs(d - g["distmat"]).max() < 1e-5


@pytest.mark.parametrize("name,k", [("backend_small.npz", 50), ("backend_ties.npz", 20)])
def test_topk_rank_lists_bitexact(gpu, name, k):
    g = golden(name)
    idx = _ev().topk_rows_device(torch.from_numpy(g["distmat"]), k).cpu().numpy()
    assert np.array_equal(idx, g[f"rank{k}_stable"])


def test_topk_long_rows_and_divisor(gpu):
    r = np.random.default_rng(5)
    x = np.round(r.random((40, 20000)) * 512).astype(np.float32)  # heavy ties
    div = (1 + r.random(40)).astype(np.float32)
    idx, val = _ev().topk_rows_device(torch.from_numpy(x), 51, row_div=torch.from_numpy(div).cuda(),
                                      with_values=True)
    ref = oracle.topk_rows(x / div[:, None], 51)
    assert np.array_equal(idx.cpu().numpy(), ref)


def _eval_rows_np(dist, qp, gp, qc, gc):
    v, f, a, n, o = _ev().eval_rows_device(torch.from_numpy(dist), qp, gp, qc, gc)
    return v.cpu().numpy(), f.cpu().numpy(), a.cpu().numpy(), n.cpu().numpy()


@pytest.mark.parametrize("name,max_rank", [("backend_small.npz", 50), ("backend_ties.npz", 20)])
def test_eval_bitexact(gpu, name, max_rank):
    g = golden(name)
    args = (g["q_pids"], g["g_pids"], g["q_cams"], g["g_cams"])
    rows = _eval_rows_np(g["distmat"], *args)
    ref = oracle.eval_rows(g["distmat"], *args)
    for a, b in zip(rows, ref):
        assert np.array_equal(a.astype(b.dtype), b)
    cmc, mAP = _ev().eval_func(g["distmat"], *args, max_rank=max_rank)
    assert np.array_equal(cmc, g["cmc_stable"]) and cmc.dtype == np.float32
    assert mAP == g["map_stable"]


def test_r1_map_eval_end_to_end(gpu):
    g = golden("backend_small.npz")
    qf, gf, qp, gp, qc, gc = _inputs()
    ev = _ev().R1_mAP_eval(100, max_rank=50, feat_norm=True)
    ev.reset()
    ev.update((torch.from_numpy(np.concatenate([qf, gf])), np.concatenate([qp, gp]), np.concatenate([qc, gc])))
    cmc, mAP = ev.compute()
    assert abs(mAP - g["map_r1map"]) < 1e-6
    assert np.abs(cmc - g["cmc_r1map"]).max() <= 1.0 / 100 + 1e-7  # at most one query flips on a near-tie


@pytest.mark.parametrize("max_rank", [10, 20, 50])
def test_r1_map_eval_max_rank_is_not_forwarded(gpu, max_rank):
    """The reference's compute() calls eval_func with its default max_rank=50
    (evaluate.py:132) whatever R1_mAP_eval was constructed with (prompt_learning.py:636
    passes 10): the CMC is 50 long and equal to the max_rank=50 result."""
    g = golden("backend_small.npz")
    qf, gf, qp, gp, qc, gc = _inputs()
    ev = _ev().R1_mAP_eval(100, max_rank=max_rank, feat_norm=True)
    ev.reset()
    ev.update((torch.from_numpy(np.concatenate([qf, gf])), np.concatenate([qp, gp]), np.concatenate([qc, gc])))
    cmc, mAP = ev.compute()
    assert cmc.shape == (50,)
    assert abs(mAP - g["map_r1map"]) < 1e-6
    assert np.abs(cmc - g["cmc_r1map"]).max() <= 1.0 / 100 + 1e-7


def test_eval_market_scale_rows_vs_oracle(gpu):
    sp = syn.DATASET_SPLITS["market1501"]
    qp, gp, qc, gc = syn.labels(sp["num_query"], sp["num_gallery"], sp["num_ids"], sp["num_cams"], seed=7,
                                junk_frac=0.02)
    r = np.random.default_rng(7)
    dev = torch.device("cuda")
    q = torch.from_numpy(r.standard_normal((sp["num_query"], 256)).astype(np.float32)).to(dev)
    gf = torch.from_numpy(r.standard_normal((sp["num_gallery"], 256)).astype(np.float32)).to(dev)
    ev = _ev()
    dist = ev.euclidean_distance_device(q, gf)
    v, f, a, n, o = ev.eval_rows_device(dist, qp, gp, qc, gc)
    sel = np.arange(0, sp["num_query"], 97)
    dsub = dist[sel].cpu().numpy()
    assert np.array_equal(dsub.view(np.uint32), oracle.distmat(q[sel].cpu().numpy(), gf.cpu().numpy()).view(np.uint32))
    ref = oracle.eval_rows(dsub, qp[sel], gp, qc[sel], gc)
    for a_, b_ in zip((v, f, a, n), ref):
        assert np.array_equal(a_.cpu().numpy()[sel].astype(b_.dtype), b_)
    idx = ev.topk_rows_device(dist[sel], 50).cpu().numpy()
    assert np.array_equal(idx, oracle.topk_rows(dsub, 50))


@pytest.mark.parametrize("G,pid_shift,pid_scale", [(3001, 0, 1), (4099, 0, 1), (3001, -(1 << 40), 1),
                                                   (2053, (1 << 62) - 9, 1), (3001, 0, 100003), (4099, -5, 1 << 40),
                                                   (3001, 5, 1800), (3001, 5, 7000)])  # wide 16-bit key ranges
def test_eval_many_positives_and_junk_vs_oracle(gpu, G, pid_shift, pid_scale):
    """Queries whose positives (> 512) or junk items (> 256) exceed the main kernel's LDS
    lists go to the large-list kernel; ragged row starts (ld = G) exercise the 16-byte
    alignment head; quantised distances give exact ties.  Bit-exact against the oracle."""
    r = np.random.default_rng(G)
    Q = 9
    gp = r.integers(1, 4, G).astype(np.int64)  # pids 1..3: ~G/3 positives per query
    gc = r.integers(0, 3, G).astype(np.int64)
    qp = np.array([1, 2, 3, 1, 2, 3, 7, 1, 2], np.int64)
    qc = np.array([0, 1, 2, 5, 5, 5, 0, 1, 2], np.int64)
    gp[::7] = 9  # some negatives for everyone
    qp[7:], gp[:40] = 8, 8  # two queries with 40 items of their pid (wave kernel path)
    gc[:40] = np.arange(40) % 3
    # arbitrary int64 pids: packed 16-bit labels when the gallery's pid range allows, else int64
    qp, gp = qp * pid_scale + pid_shift, gp * pid_scale + pid_shift
    dist = (np.round(r.random((Q, G)) * 64) / 64).astype(np.float32)
    rows = _eval_rows_np(dist, qp, gp, qc, gc)
    ref = oracle.eval_rows(dist, qp, gp, qc, gc)
    for a, b in zip(rows, ref):
        assert np.array_equal(a.astype(b.dtype), b)


@pytest.mark.parametrize("steps", [0, 16, 1024])
def test_eval_bucket_paths_vs_oracle(gpu, steps):
    """The main kernel's bucket binning (every query within its LDS lists): 1..300 positives
    per query, distances continuous (steps 0) or quantised to 1/16 or 1/1024 (items tied with
    positives, several positives per bucket: the exact (value, index) walk), with negative
    values and +-inf mixed in.  Bit-exact against the oracle.  (NaN distances are outside the
    contract: the oracle's comparator, like the kernel's, does not order them.)"""
    r = np.random.default_rng(100 + steps)
    Q, G = 48, 5003
    gp = r.integers(1, 60, G).astype(np.int64)
    gc = r.integers(0, 4, G).astype(np.int64)
    gp[:300], gc[:300] = 77, np.arange(300) % 4     # query 0's identity: ~225 positives
    qp = np.concatenate([[77], r.integers(1, 60, Q - 1)]).astype(np.int64)
    qc = r.integers(0, 4, Q).astype(np.int64)
    dist = (r.random((Q, G)) * 4 - 1).astype(np.float32)
    if steps:
        dist = (np.round(dist * steps) / steps).astype(np.float32)
    dist[1::5, r.integers(0, G, 40)] = np.inf
    dist[2::5, r.integers(0, G, 40)] = -np.inf
    dist[3::5, r.integers(0, G, 40)] = dist[3::5, :1]  # more exact ties with a row's first item
    dist[4] = 0.5                                    # one row of equal values: every compare a tie
    rows = _eval_rows_np(dist, qp, gp, qc, gc)
    ref = oracle.eval_rows(dist, qp, gp, qc, gc)
    for a, b in zip(rows, ref):
        assert np.array_equal(a.astype(b.dtype), b)


@pytest.mark.parametrize("G,pid_shift", [(6007, 0), (9001, -(1 << 40))])
def test_eval_beyond_lds_lists_vs_oracle(gpu, G, pid_shift):
    """Queries with more positives than the large-list kernel's LDS holds (> 2048) are
    evaluated by its last workgroup on workspace scratch: no capacity limit, as in the
    reference (evaluate.py:40-80).  Bit-exact against the oracle, overflow stays 0."""
    r = np.random.default_rng(G)
    Q = 5
    gp = r.integers(1, 3, G).astype(np.int64)  # pids 1..2: ~G/2 items each
    gc = r.integers(0, 2, G).astype(np.int64)
    gp[::11] = 9
    qp = (np.array([1, 2, 1, 9, 4], np.int64) + pid_shift)
    gp = gp + pid_shift
    qc = np.array([0, 1, 3, 0, 0], np.int64)
    dist = (np.round(r.random((Q, G)) * 256) / 256).astype(np.float32)
    ev = _ev()
    d = torch.from_numpy(dist).cuda()
    v, f, a, n, o = ev.eval_rows_device(d, qp, gp, qc, gc)
    assert int(o.cpu()[0]) == 0
    ref = oracle.eval_rows(dist, qp, gp, qc, gc)
    for a_, b_ in zip((v, f, a, n), ref):
        assert np.array_equal(a_.cpu().numpy().astype(b_.dtype), b_)
    cmc, mAP = ev.eval_func(dist, qp, gp, qc, gc, max_rank=50)
    ocmc, omap = oracle.eval_func(dist, qp, gp, qc, gc, 50)
    assert np.array_equal(cmc, ocmc) and mAP == omap


def test_eval_edge_cases(gpu):
    ev = _ev()
    r = np.random.default_rng(3)
    # gallery smaller than max_rank: max_rank shrinks to num_g (evaluate.py:37-39)
    dist = r.random((4, 10)).astype(np.float32)
    qp = np.array([1, 2, 3, 9]); gp = np.array([1, 1, 2, 2, 3, 3, 4, 4, 5, 5])
    qc = np.zeros(4, np.int64); gc = np.ones(10, np.int64)
    cmc, mAP = ev.eval_func(dist, qp, gp, qc, gc, max_rank=50)
    ocmc, omap = oracle.eval_func(dist, qp, gp, qc, gc, max_rank=50)
    assert cmc.shape == (10,) and np.array_equal(cmc, ocmc) and mAP == omap
    # no query identity in the gallery -> AssertionError (evaluate.py:82)
    with pytest.raises(AssertionError):
        ev.eval_func(dist, np.array([7, 8, 9, 9]), gp, qc, gc)
    # ragged kept lengths below max_rank -> ValueError like np.asarray(all_cmc) (evaluate.py:84)
    gp2 = np.array([1, 1, 1, 2, 2, 3, 3, 4, 4, 5])
    gc2 = np.array([0, 0, 1, 0, 1, 0, 1, 0, 1, 0])
    with pytest.raises(ValueError):
        oracle.eval_func(dist, qp, gp2, qc, gc2, max_rank=50)
    with pytest.raises(ValueError):
        ev.eval_func(dist, qp, gp2, qc, gc2, max_rank=50)
