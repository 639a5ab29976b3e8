"""GPU parity of the staged / sharded re-ranking (reidmi_rr_*, reranking.staged_rerank):
bit-identical to the one-call kernels (reidmi_rerank) and to the oracle, with the distance
rows processed in several chunks, and across 2 ranks sharing cuda:0 (gloo, host-staged)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402

reidmi_boot.load()

import oracle  # noqa: E402
from multimodal_reid_amd import synthetic as syn  # noqa: E402

pytestmark = pytest.mark.gpu


def _feats(Q, G, seed, dim=256, ids=400, noise=3.0):
    qp, gp, _, _ = syn.labels(Q, G, num_ids=ids, num_cams=6, seed=seed)
    qf, gf = syn.features(qp, gp, dim=dim, seed=seed, noise=noise)
    return oracle.l2norm(np.concatenate([qf, gf]))


@pytest.mark.parametrize("Q,G,k1,k2", [(100, 500, 50, 15), (100, 500, 20, 6), (64, 700, 20, 1), (300, 2200, 50, 15)])
def test_staged_bitexact_vs_one_call_and_oracle(gpu, Q, G, k1, k2):
    from multimodal_reid_amd import reranking
    feats = _feats(Q, G, seed=Q + k1)
    f = torch.from_numpy(feats).to(gpu)
    N = Q + G
    staged = reranking.re_ranking_sharded(f[:Q], f[Q:], k1, k2, 0.3, chunk_bytes=4 * N * 97).cpu().numpy()
    one = reranking.re_ranking_device(f[:Q], f[Q:], k1, k2, 0.3).cpu().numpy()
    assert np.array_equal(staged.view(np.uint32), one.view(np.uint32))
    if N <= 800:
        ref = oracle.re_ranking(feats[:Q], feats[Q:], k1, k2, 0.3)
        assert np.array_equal(staged.view(np.uint32), ref.view(np.uint32))


def test_staged_duke_scale_bitexact_vs_one_call(gpu):
    from multimodal_reid_amd import evaluate, reranking
    sp = syn.DATASET_SPLITS["dukemtmc"]
    Q, G = sp["num_query"], sp["num_gallery"]
    qp, gp, _, _ = syn.labels(Q, G, sp["num_ids"], sp["num_cams"], seed=0, distractor_frac=0.1, junk_frac=0.02)
    qf, gf = syn.features(qp, gp)
    qn = evaluate.l2_normalize_device(torch.from_numpy(qf).to(gpu))
    gn = evaluate.l2_normalize_device(torch.from_numpy(gf).to(gpu))
    staged = reranking.re_ranking_sharded(qn, gn, 50, 15, 0.3, chunk_bytes=1 << 30)
    one = reranking.re_ranking_device(qn, gn, 50, 15, 0.3)
    assert torch.equal(staged.view(torch.int32), one.view(torch.int32))


def _worker(rank, world, port, out):
    import torch.distributed as dist
    from multimodal_reid_amd import distributed as rd, reranking
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    feats = _feats(120, 900, seed=5)
    f = torch.from_numpy(feats).cuda()
    part = reranking.re_ranking_sharded(f[:120], f[120:], 50, 15, 0.3, chunk_bytes=4 * 1020 * 200)
    out[rank] = rd.gather_rows(part, 120).cpu().numpy()
    dist.destroy_process_group()


def test_sharded_two_ranks_one_gpu(gpu):
    import torch.multiprocessing as mp
    from multimodal_reid_amd import reranking
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
    f = torch.from_numpy(_feats(120, 900, seed=5)).to(gpu)
    one = reranking.re_ranking_device(f[:120], f[120:], 50, 15, 0.3).cpu().numpy()
    for r in range(2):
        assert np.array_equal(out[r].view(np.uint32), one.view(np.uint32))


def _rank_rows(f, Q, prefilter, chunk_bytes):
    from multimodal_reid_amd import reranking
    old = reranking.RANK_PREFILTER
    reranking.RANK_PREFILTER = prefilter
    try:
        st = reranking.HipStages(f, Q, 50, 15, 0.3, chunk_bytes=chunk_bytes)
        R, rmax = st.rank_rows(0, f.shape[0])
        return R.cpu().numpy(), rmax.cpu().numpy(), st
    finally:
        reranking.RANK_PREFILTER = old


@pytest.mark.parametrize("case", ["clustered", "near_dup", "exact_dup", "large_norm", "gaussian_1792", "fp16_range",
                                  "concentrated"])
def test_rank_prefilter_bitexact(gpu, case):
    """R2 through the fp16 pre-filter (reidmi_rr_rank_rows_f16) equals the exact rows
    (reidmi_rr_rank_rows) bit for bit: initial_rank and the row maxima, on inputs that stress
    the error bound — near-duplicates and exact duplicates (dense ties at the K-th distance,
    candidate overflow -> the exact path), unnormalised features, concentrated high-dimensional
    distances, a random network's concentrated embeddings (every row to the exact rows) — and
    features beyond fp16's range (the pre-filter is then not used)."""
    r = np.random.default_rng(len(case))
    if case == "clustered":
        f = _feats(200, 1800, seed=3)
    elif case == "near_dup":
        base = r.standard_normal((40, 256)).astype(np.float32)
        f = np.repeat(base, 50, axis=0) + 1e-4 * r.standard_normal((2000, 256)).astype(np.float32)
        f = oracle.l2norm(f)
    elif case == "exact_dup":
        base = oracle.l2norm(r.standard_normal((30, 128)).astype(np.float32))
        f = np.repeat(base, 70, axis=0)
    elif case == "large_norm":
        f = (r.standard_normal((1500, 320)) * 40).astype(np.float32)
    elif case == "gaussian_1792":
        f = oracle.l2norm(r.standard_normal((1300, 1792)).astype(np.float32))
    elif case == "fp16_range":
        f = r.standard_normal((900, 256)).astype(np.float32)
        f[7, 3] = 40000.0
    else:
        # a random network's embeddings: every distance inside the bound -> the exact rows
        f = oracle.l2norm(np.ones((1200, 512), np.float32) + 1e-3 * r.standard_normal((1200, 512)).astype(np.float32))
    f = torch.from_numpy(np.ascontiguousarray(f)).to(gpu)
    N = f.shape[0]
    Rf, mf, st = _rank_rows(f, 100, True, 4 * N * 300)
    Re, me, _ = _rank_rows(f, 100, False, 4 * N * 300)
    assert st._f16[4] == (case != "fp16_range")
    assert np.array_equal(Rf, Re)
    assert np.array_equal(mf.view(np.uint32), me.view(np.uint32))


def _rank_rows_f16_direct(f, K, stride, chunk_rows):
    """reidmi_rr_rank_rows_f16_ex over all rows with a given sample stride (0: the dense form):
    (rank [N][K], rowmax [N], need [N]) as numpy; rows with need = 1 carry no output."""
    from multimodal_reid_amd import _lib
    N, D = f.shape
    Np, Dp = (N + 255) // 256 * 256, (D + 63) // 64 * 64
    sqn = torch.empty(N, device=f.device)  # the exact rows' squared norms (reranking.HipStages)
    _lib.call("reidmi_row_sqnorm_f32", _lib.ptr(f), N, D, D, _lib.ptr(sqn), _lib.stream())
    nrm = torch.sqrt(sqn)
    x16 = torch.zeros((Np, Dp), dtype=torch.float16, device=f.device)
    ok = torch.ones(1, dtype=torch.int32, device=f.device)
    _lib.call("reidmi_rr_feat16", _lib.ptr(f), N, D, D, _lib.ptr(x16), Np, Dp, _lib.ptr(ok), _lib.stream())
    nmax2 = torch.empty(2, device=f.device)
    _lib.call("reidmi_rr_norm_max", _lib.ptr(sqn), _lib.ptr(nrm), N, _lib.ptr(nmax2), _lib.stream())
    R = torch.full((N, K), -1, dtype=torch.int32, device=f.device)
    rmax = torch.zeros(N, device=f.device)
    need = torch.zeros(N, dtype=torch.int32, device=f.device)
    chunk = torch.empty(chunk_rows * Np, device=f.device)
    _lib.call("reidmi_rr_rank_rows_f16_ex", _lib.ptr(f), N, D, D, _lib.ptr(sqn), _lib.ptr(nrm), _lib.ptr(nmax2),
              _lib.ptr(x16), Np, Dp, 0, N, K, _lib.ptr(R), _lib.ptr(rmax), _lib.ptr(need), _lib.ptr(chunk), chunk_rows,
              stride, _lib.stream())
    return R.cpu().numpy(), rmax.cpu().numpy(), need.cpu().numpy()


@pytest.mark.parametrize("case", ["clustered", "sorted_ids", "near_dup", "tracklets", "large_norm", "gaussian_1792",
                                  "concentrated"])
def test_rank_prefilter_in_epilogue_bitexact(gpu, case):
    """The in-epilogue selection (1/16 sample -> per-row thresholds -> EPI_RRSV survivor lists ->
    rank_select_sv), in row passes (rectangular) and in one call over the symmetric product's
    upper triangle (each pair tested for both its rows), equals the dense form (bounds written
    and streamed) and the exact rows bit for bit on every row it decides, at N = 12 000-16 000
    (the sampled form applies from N ~ 4 096); 'sorted_ids' orders the items by identity so the
    sample misses whole clusters (loose thresholds), 'near_dup' / 'tracklets' make long survivor
    lists and dense ties, 'concentrated' sends every row to the exact path."""
    from multimodal_reid_amd import _lib
    r = np.random.default_rng(len(case) + 7)
    if case in ("clustered", "sorted_ids"):
        f = _feats(400, 11600, seed=9, ids=900)
        if case == "sorted_ids":
            qp, gp, _, _ = syn.labels(400, 11600, num_ids=900, num_cams=6, seed=9)
            f = f[np.argsort(np.concatenate([qp, gp]), kind="stable")]
    elif case == "near_dup":
        base = r.standard_normal((300, 384)).astype(np.float32)
        f = oracle.l2norm(np.repeat(base, 40, axis=0) + 1e-4 * r.standard_normal((12000, 384)).astype(np.float32))
    elif case == "tracklets":
        f = _feats(500, 13500, seed=11, dim=512, ids=1200, noise=2.0)
        f = oracle.l2norm(f[::24].repeat(24, axis=0)[:14000] + 1e-3 * r.standard_normal((14000, 512)).astype(np.float32))
    elif case == "large_norm":
        f = (r.standard_normal((12500, 320)) * 40).astype(np.float32)
    elif case == "gaussian_1792":
        f = oracle.l2norm(r.standard_normal((16000, 1792)).astype(np.float32))
    else:
        f = oracle.l2norm(np.ones((12000, 512), np.float32) + 1e-3 * r.standard_normal((12000, 512)).astype(np.float32))
    f = torch.from_numpy(np.ascontiguousarray(f)).to(gpu)
    N, K = f.shape[0], 51
    pass_rows = _lib.load().reidmi_rr_rank_rows_f16_pass_rows
    Np = (N + 255) // 256 * 256
    assert 256 <= int(pass_rows(N, Np, 256, K, 16)) < N  # rectangular: row passes (whole 256-row tiles)
    assert int(pass_rows(N, Np, 4096, K, 16)) == N  # the triangle form: all rows in one call
    assert int(pass_rows(N, Np, 256, K, 0)) == 256  # the dense form: chunk_rows
    Rs, ms, ns = _rank_rows_f16_direct(f, K, 16, 256)
    Rt, mt, nt = _rank_rows_f16_direct(f, K, 16, 4096)
    Rd, md, nd = _rank_rows_f16_direct(f, K, 0, 256)
    Re, me, _ = _rank_rows(f, 100, False, 4 * N * 300)
    for R, m, need in ((Rs, ms, ns), (Rt, mt, nt), (Rd, md, nd)):
        ok = need == 0
        assert np.array_equal(R[ok], Re[ok, :K])
        assert np.array_equal(m[ok].view(np.uint32), me[ok].view(np.uint32))
    if case == "concentrated":
        assert ns.all() and nt.all() and nd.all()
    elif case in ("clustered", "sorted_ids", "gaussian_1792", "large_norm"):
        assert ns.mean() < 0.05 and nt.mean() < 0.05, (ns.mean(), nt.mean())  # the sampled forms decide the rows
    print(f"{case}: sampled form decides {1 - ns.mean():.3f} of the rows (triangle {1 - nt.mean():.3f}), "
          f"dense form {1 - nd.mean():.3f}")


def test_rank_prefilter_triangle_list_overflow(gpu):
    """The triangle form with a chunk that leaves 1 024 survivor slots per row, on 8 clusters of
    1 500 near-duplicates (every cluster member survives for every row): the rows whose lists
    overflow come back marked in need[] (the 1M run marks a few), the others bit-exact; through
    the Python driver (HipStages.rank_rows: marked rows go through the exact rows) initial_rank
    and the row maxima equal the exact rows for every row."""
    from multimodal_reid_amd import _lib
    r = np.random.default_rng(5)
    base = r.standard_normal((8, 384)).astype(np.float32)
    f = oracle.l2norm(np.repeat(base, 1500, axis=0) + 1e-4 * r.standard_normal((12000, 384)).astype(np.float32))
    f = torch.from_numpy(np.ascontiguousarray(f)).to(gpu)
    N, K = f.shape[0], 51
    Np = (N + 255) // 256 * 256
    cr = 2060  # chunk rows of Np floats: a 1 024-pair list per row
    assert int(_lib.load().reidmi_rr_rank_rows_f16_pass_rows(N, Np, cr, K, 16)) == N
    Rt, mt, nt = _rank_rows_f16_direct(f, K, 16, cr)
    Re, me, _ = _rank_rows(f, 100, False, 4 * N * 300)
    assert nt.sum() > N // 2  # the lists overflowed
    ok = nt == 0
    assert np.array_equal(Rt[ok], Re[ok, :K]) and np.array_equal(mt[ok].view(np.uint32), me[ok].view(np.uint32))
    Rp, mp, _ = _rank_rows(f, 100, True, 4 * N * 2304)
    assert np.array_equal(Rp, Re) and np.array_equal(mp.view(np.uint32), me.view(np.uint32))


def _one_call(feat, Q, k1, k2, lam):
    """reidmi_rerank itself (N x N fp32 distance materialised), whatever N."""
    from multimodal_reid_amd import _lib, reranking
    N, D = feat.shape
    G = N - Q
    L = _lib.load()
    nbytes = L.reidmi_rerank_workspace_bytes(Q, G, k1, k2, 0, 0)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=feat.device)
    out = torch.empty((Q, G), device=feat.device)
    flags = torch.zeros(1, dtype=torch.int32, device=feat.device)
    lh, lf = reranking._lam(lam)
    _lib.call("reidmi_rerank", _lib.ptr(feat), Q, G, D, D, k1, k2, lh, lf, _lib.ptr(out), G, _lib.ptr(ws), nbytes,
              _lib.ptr(flags), _lib.stream())
    reranking._check(flags)
    del ws
    return out


@pytest.mark.parametrize("case", ["clustered", "tracklets"])
def test_staged_prefilter_above_min_n_bitexact(gpu, case):
    """Where the staged path is actually used: N = 33 000 >= STAGED_MIN_N, D = 1280, so
    re_ranking_device takes the row-chunked stages with the fp16 R2 pre-filter (and
    R1_mAP_eval(reranking=True) too).  Both must equal the one-call reidmi_rerank (its N x N
    fp32 distance, 4.4 GB, still fits) bit for bit, and the CMC/mAP must be identical.
    'tracklets': the gallery is groups of 24 near-identical crops (MSMT17-style tracklets),
    dense exact-distance ties and duplicate-heavy neighbourhoods."""
    from multimodal_reid_amd import evaluate, reranking
    Q, G, D = 1500, 31500, 1280
    assert Q + G >= reranking.STAGED_MIN_N
    qp, gp, qc, gc = syn.labels(Q, G, num_ids=1300, num_cams=15, seed=41, distractor_frac=0.1, junk_frac=0.02)
    if case == "clustered":
        qf, gf = syn.features(qp, gp, dim=D, seed=41)
    else:
        r = np.random.default_rng(41)
        qf, gf = syn.features(qp, gp, dim=D, seed=41, noise=2.0)
        base = gf[::24].repeat(24, axis=0)[:G]
        gf = (base + 1e-3 * r.standard_normal(base.shape)).astype(np.float32)
        gp = gp[::24].repeat(24)[:G]
    qn = evaluate.l2_normalize_device(torch.from_numpy(qf).to(gpu))
    gn = evaluate.l2_normalize_device(torch.from_numpy(gf).to(gpu))
    auto = reranking.re_ranking_device(qn, gn, 50, 15, 0.3)
    one = _one_call(torch.cat([qn, gn]).contiguous(), Q, 50, 15, 0.3)
    assert torch.equal(auto.view(torch.int32), one.view(torch.int32))
    cmc1, map1 = evaluate.eval_func_device(one, qp, gp, qc, gc)
    del auto, one
    torch.cuda.empty_cache()
    ev = evaluate.R1_mAP_eval(Q, max_rank=50, feat_norm=True, reranking=True)
    ev.reset()
    ev.update((torch.cat([torch.from_numpy(qf), torch.from_numpy(gf)]), np.concatenate([qp, gp]),
               np.concatenate([qc, gc])))
    cmc2, map2 = ev.compute()
    assert np.array_equal(cmc1, cmc2) and map1 == map2


def _tri_case(case):
    r = np.random.default_rng(77)
    if case == "clustered":
        return _feats(400, 11800, seed=13, dim=384, ids=900)
    # tracklets: groups of 24 near-identical items (dense ties, long survivor lists)
    f = _feats(400, 12000, seed=14, dim=384, ids=1000, noise=2.0)
    return oracle.l2norm(f[::24].repeat(24, axis=0)[:12400] + 1e-3 * r.standard_normal((12400, 384)).astype(np.float32))


def _tri_chunk(N):
    return 4 * N * 4608  # chunk rows >= 4 096 at this N: the triangle form applies


def _tri_worker(rank, world, port, out, case):
    import torch.distributed as dist
    from multimodal_reid_amd import distributed as rd, reranking
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        f = torch.from_numpy(_tri_case(case)).cuda()
        N, Q = f.shape[0], 400
        st = reranking.HipStages(f, Q, 50, 15, 0.3, chunk_bytes=_tri_chunk(N))
        part = reranking.staged_rerank(st, N, Q)
        out[rank] = (rd.gather_rows(part, Q).cpu().numpy(), st.stats["form"], st.stats["exact_rows"])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", ["clustered", "tracklets"])
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_triangle_r2_equals_one_gpu(gpu, case, world):
    """R2's triangle form split over ranks (HipStages.rank_rows_tri_sharded: each rank runs a
    contiguous 1/W of the upper-triangle tiles over all rows, the partial survivor lists go to
    their rows' owners all-to-all) on >= 12 000 items: the re-ranked distances of gloo world 2 / 3
    (sharing cuda:0) equal the one-process run (the one-call triangle form) bit for bit, and
    every rank took the sharded triangle (not the rectangular row passes)."""
    import torch.multiprocessing as mp
    from multimodal_reid_amd import reranking
    feats = _tri_case(case)
    f = torch.from_numpy(feats).to(gpu)
    N, Q = f.shape[0], 400
    st = reranking.HipStages(f, Q, 50, 15, 0.3, chunk_bytes=_tri_chunk(N))
    one = reranking.staged_rerank(st, N, Q).cpu().numpy()
    assert st.stats["form"] == "triangle"
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_tri_worker, args=(world, port, out, case), nprocs=world, join=True)
    for r in range(world):
        got, form, exact = out[r]
        assert form == "triangle (sharded)", (r, form)
        assert np.array_equal(got.view(np.uint32), one.view(np.uint32)), r
    print(f"{case} world {world}: exact-fallback rows per rank {[out[r][2] for r in range(world)]} "
          f"(one GPU: {st.stats['exact_rows']})")
