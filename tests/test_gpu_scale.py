"""configs[3] and configs[4] at their workload sizes (BASELINE.json; VERDICT r3 asked for both):

* MSMT17, 11 659 q x 82 161 g, D = 1280 (configs[3]): the staged re-rank re_ranking_device takes
  (row-chunked stages, R2 through the in-epilogue triangle pre-filter) equals the one-call
  reidmi_rerank with its N x N fp32 distance materialised (35 GB, fits one MI355X) bit for bit,
  on identity-clustered features and on a tracklet gallery (groups of 24 near-identical crops:
  dense ties, long survivor lists); R1_mAP_eval(reranking=True) gives the identical CMC/mAP.
  Reference: reranking.py:29-100, evaluate.py:124-132.
* 1 010 000 items at D = 1792 (configs[4]'s ViT-L/14 gallery + 10 000 queries): R2 over every
  row through HipStages.rank_rows (the triangle form over the whole symmetric product, rows
  it marks sent to the exact rows) equals reidmi_rr_rank_rows (the exact fp32 rows) on 1 024
  sampled rows and on every marked row, bit for bit.  Reference: reranking.py:36-48.
* configs[4] end to end at 10 000 q x 1 000 000 g, D = 1792 (VERDICT r4 Next #2): the exact
  distance + eval rows of 256 sampled queries bit-exact against the C oracle on those rows
  (evaluate.py:7-13,29-88); the whole staged re-rank R1-R7 at N = 1.01 M bit-identical for two
  distance-chunk sizes (different R2 pass shapes); R1_mAP_eval(reranking=True) from the raw
  features gives the identical CMC/mAP (evaluate.py:91-135, reranking.py:29-100).
Features are generated on the device (identity-clustered Gaussians)."""
import os

import numpy as np
import pytest
import torch

from multimodal_reid_amd import synthetic as syn

pytestmark = pytest.mark.gpu


def _clustered(pids, D, seed, dev, noise=4.0):
    """Identity-clustered features on the device: centre N(0, I) per pid > 0 (own centre for
    pid <= 0) + noise N(0, sigma^2 I) (not normalised)."""
    g = torch.Generator(device=dev).manual_seed(seed)
    p = torch.from_numpy(np.asarray(pids)).to(dev)
    n_ids = int(p.max().item()) + 1
    centres = torch.randn((n_ids, D), generator=g, device=dev)
    idx = torch.where(p > 0, p, 0)
    f = torch.empty((len(pids), D), device=dev)
    for a in range(0, len(pids), 65536):
        z = min(len(pids), a + 65536)
        own = torch.randn((z - a, D), generator=g, device=dev)
        c = torch.where((p[a:z] > 0)[:, None], centres[idx[a:z]], own)
        f[a:z] = c + noise * torch.randn((z - a, D), generator=g, device=dev)
    return f


def _one_call(feat, Q, k1, k2, lam):
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
def test_msmt17_size_staged_equals_one_call(gpu, case):
    from multimodal_reid_amd import evaluate, reranking
    sp = syn.DATASET_SPLITS["msmt17"]
    Q, G, D = sp["num_query"], sp["num_gallery"], 1280
    qp, gp, qc, gc = syn.labels(Q, G, sp["num_ids"], sp["num_cams"], seed=17, distractor_frac=0.1, junk_frac=0.02)
    if case == "tracklets":
        gp = gp[::24].repeat(24)[:G]
        gc = gc[::24].repeat(24)[:G]
    raw = _clustered(np.concatenate([qp, gp]), D, 17, gpu, noise=4.0 if case == "clustered" else 2.0)
    if case == "tracklets":
        base = raw[Q:][::24].repeat_interleave(24, 0)[:G]
        gen = torch.Generator(device=gpu).manual_seed(18)
        raw = torch.cat([raw[:Q], base + 1e-3 * base.norm(dim=1, keepdim=True) / D ** 0.5 *
                         torch.randn(base.shape, generator=gen, device=gpu)])
    f = evaluate.l2_normalize_device(raw)  # R1_mAP_eval's feat_norm (evaluate.py:114)
    qn, gn = f[:Q].contiguous(), f[Q:].contiguous()
    stats = {}
    staged = reranking.re_ranking_sharded(qn, gn, 50, 15, 0.3, stats=stats)
    auto = reranking.re_ranking_device(qn, gn, 50, 15, 0.3)  # Q + G >= STAGED_MIN_N: the staged path
    assert torch.equal(staged.view(torch.int32), auto.view(torch.int32))
    del auto
    assert stats["form"] == "triangle" and stats["rows"] == Q + G
    assert stats["exact_rows"] < 0.05 * (Q + G), stats["exact_rows"]  # the pre-filter decides the rows
    one = _one_call(f, Q, 50, 15, 0.3)
    assert torch.equal(staged.view(torch.int32), one.view(torch.int32))
    cmc1, map1 = evaluate.eval_func_device(one, qp, gp, qc, gc)
    del one, staged
    torch.cuda.empty_cache()
    ev = evaluate.R1_mAP_eval(Q, max_rank=50, feat_norm=True, reranking=True)
    ev.reset()
    ev.update((raw, np.concatenate([qp, gp]), np.concatenate([qc, gc])))
    cmc2, map2 = ev.compute()
    assert np.array_equal(cmc1, cmc2) and map1 == map2
    print(f"MSMT17 {case}: R2 exact-fallback rows {stats['exact_rows']} of {Q + G}; mAP(rerank) {map2:.4f}")


def test_1m_gallery_rank_rows_bitexact_sample(gpu):
    from multimodal_reid_amd import _lib, reranking
    Q, G, D = 10000, 1000000, 1792
    N = Q + G
    qp, gp, _, _ = syn.labels(Q, G, num_ids=50000, num_cams=15, seed=23, distractor_frac=0.1)
    from multimodal_reid_amd import evaluate
    f = evaluate.l2_normalize_device(_clustered(np.concatenate([qp, gp]), D, 23, gpu))
    st = reranking.HipStages(f, Q, 50, 15, 0.3)
    R, rmax = st.rank_rows(0, N)
    assert st.stats["form"] == "triangle" and st.stats["rows"] == N
    marked = np.concatenate(st.stats["exact_idx"]) if st.stats["exact_idx"] else np.zeros(0, np.int64)
    assert len(marked) == st.stats["exact_rows"] < 0.01 * N
    K = st.K
    rng = np.random.default_rng(23)
    ranges = [(int(a), int(a) + 256) for a in rng.integers(0, N - 256, 4)]
    ranges += [(int(r), int(r) + 1) for r in marked[:64]]
    chunk = torch.empty(256 * N, device=gpu)
    for lo, hi in ranges:
        Re = torch.empty((hi - lo, K), dtype=torch.int32, device=gpu)
        me = torch.empty(hi - lo, device=gpu)
        _lib.call("reidmi_rr_rank_rows", _lib.ptr(st.feat), N, D, D, _lib.ptr(st.sqn), lo, hi, K, _lib.ptr(Re),
                  _lib.ptr(me), _lib.ptr(chunk), 256, _lib.stream())
        assert torch.equal(R[lo:hi], Re), (lo, hi)
        assert torch.equal(rmax[lo:hi].view(torch.int32), me.view(torch.int32)), (lo, hi)
    print(f"1M x {D}: R2 triangle form, {len(marked)} rows marked for the exact rows; "
          f"{sum(h - l for l, h in ranges)} rows checked against reidmi_rr_rank_rows")


def test_1m_gallery_eval_and_rerank_end_to_end(gpu):
    import time
    import oracle
    from multimodal_reid_amd import evaluate, reranking
    Q, G, D = 10000, 1000000, 1792
    qp, gp, qc, gc = syn.labels(Q, G, num_ids=50000, num_cams=15, seed=29, distractor_frac=0.1)
    raw = _clustered(np.concatenate([qp, gp]), D, 29, gpu)
    f = evaluate.l2_normalize_device(raw)
    qn, gn = f[:Q].contiguous(), f[Q:].contiguous()
    t0 = time.perf_counter()
    # (1) exact distance + eval rows (one launch each over the 10 000 x 1 000 000 problem)
    d = evaluate.euclidean_distance_device(qn, gn)
    valid, first, ap, nkept, ovf = evaluate.eval_rows_device(d, qp, gp, qc, gc)
    assert int(ovf.reshape(-1)[0].item()) == 0
    rows = np.sort(np.random.default_rng(29).choice(Q, 256, replace=False))
    ridx = torch.from_numpy(rows).to(gpu)
    d_s = d[ridx].cpu().numpy()
    got = [t[ridx].cpu().numpy() for t in (valid, first, ap, nkept)]
    cmc, mAP = evaluate.aggregate_cmc_map(valid.cpu().numpy(), first.cpu().numpy(), ap.cpu().numpy(),
                                          nkept.cpu().numpy(), G, 50)
    del d, valid, first, ap, nkept
    torch.cuda.empty_cache()
    t1 = time.perf_counter()
    oracle.set_threads(min(16, os.cpu_count() or 1))
    od = oracle.distmat(qn[ridx].cpu().numpy(), gn.cpu().numpy())
    assert np.array_equal(d_s.view(np.uint32), od.view(np.uint32))
    ov, of, oa, on = oracle.eval_rows(od, qp[rows], gp, qc[rows], gc)
    assert np.array_equal(got[0].astype(np.int64), ov.astype(np.int64))
    assert np.array_equal(got[1], of) and np.array_equal(got[3], on)
    assert np.array_equal(got[2].view(np.uint64), oa.view(np.uint64))
    del od
    t2 = time.perf_counter()
    # (2) the staged re-rank at N = 1.01 M, two distance-chunk sizes
    s1, s2 = {}, {}
    fin = reranking.re_ranking_sharded(qn, gn, 50, 15, 0.3, stats=s1)
    cmc_r, map_r = evaluate.eval_func_device(fin, qp, gp, qc, gc)
    fin2 = reranking.re_ranking_sharded(qn, gn, 50, 15, 0.3, chunk_bytes=3 << 30, stats=s2)
    assert torch.equal(fin.view(torch.int32), fin2.view(torch.int32))  # 2 x 40 GB resident
    del fin, fin2
    torch.cuda.empty_cache()
    t3 = time.perf_counter()
    # (3) the drop-in surface from the raw features
    ev = evaluate.R1_mAP_eval(Q, max_rank=50, feat_norm=True, reranking=True)
    ev.reset()
    ev.update((raw, np.concatenate([qp, gp]), np.concatenate([qc, gc])))
    del raw, f, qn, gn
    torch.cuda.empty_cache()
    cmc_e, map_e = ev.compute()
    assert np.array_equal(cmc_e, cmc_r) and map_e == map_r
    t4 = time.perf_counter()
    print(f"1M: plain mAP {mAP:.5f} rank-1 {cmc[0]:.5f}; re-ranked mAP {map_r:.5f} rank-1 {cmc_r[0]:.5f}; "
          f"R2 forms {s1['form']} / {s2['form']} (exact-fallback rows {s1['exact_rows']} / {s2['exact_rows']}); "
          f"s: eval {t1 - t0:.1f}, oracle {t2 - t1:.1f}, re-rank x2 {t3 - t2:.1f}, R1_mAP_eval {t4 - t3:.1f}")
