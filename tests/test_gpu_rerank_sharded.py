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
