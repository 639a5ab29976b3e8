"""GPU parity of k-reciprocal re-ranking (rerank.hip) — bit-exact against the fixtures
the reference produced (reranking.py only_local path) and against the oracle."""
import numpy as np
import pytest
import torch

import oracle
from multimodal_reid_amd import synthetic as syn
from conftest import golden

pytestmark = pytest.mark.gpu


def _rr():
    from multimodal_reid_amd import reranking
    return reranking


@pytest.mark.parametrize("k1,k2", [(50, 15), (20, 6)])
def test_rerank_only_local_bitexact_vs_reference(gpu, k1, k2):
    g = golden("rerank_small.npz")
    q = torch.zeros(100, 4)
    gl = torch.zeros(500, 4)
    final = _rr().re_ranking(q, gl, k1, k2, 0.3, local_distmat=g["dist_all"], only_local=True)
    ref = g[f"final_k{k1}_{k2}"]
    assert final.dtype == np.float32 and final.shape == ref.shape
    assert np.array_equal(final.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("k1,k2", [(50, 15), (20, 6), (20, 1)])
def test_rerank_from_features_bitexact_vs_oracle(gpu, k1, k2):
    g = golden("rerank_small.npz")
    qf, gf = syn.features(g["q_pids"], g["g_pids"], dim=1280, seed=3, noise=4.0)
    feats = oracle.l2norm(np.concatenate([qf, gf]))
    final = _rr().re_ranking(torch.from_numpy(feats[:100]), torch.from_numpy(feats[100:]), k1, k2, 0.3)
    ref = oracle.re_ranking(feats[:100], feats[100:], k1, k2, 0.3)
    assert np.array_equal(final.view(np.uint32), ref.view(np.uint32))
    if k2 == 15:  # and mAP-level parity with the reference's full path (its torch distance)
        args = (g["q_pids"], g["g_pids"], g["q_cams"], g["g_cams"], 50)
        assert abs(oracle.eval_func(final, *args)[1] - g["map_k50_15"]) <= 1e-3


def test_rerank_local_distmat_added(gpu):
    r = np.random.default_rng(8)
    qp, gp, qc, gc = syn.labels(40, 260, num_ids=30, num_cams=4, seed=8)
    qf, gf = syn.features(qp, gp, dim=256, seed=8)
    feats = oracle.l2norm(np.concatenate([qf, gf]))
    local = (r.random((300, 300)) * 0.2).astype(np.float32)  # not symmetric
    final = _rr().re_ranking(torch.from_numpy(feats[:40]), torch.from_numpy(feats[40:]), 20, 6, 0.3,
                             local_distmat=local)
    D = oracle.distmat(feats, feats) + local
    ref = oracle.rerank_from_dist(D, 40, 20, 6, 0.3)
    assert np.array_equal(final.view(np.uint32), ref.view(np.uint32))


def test_rerank_medium_bitexact_vs_oracle(gpu):
    qp, gp, qc, gc = syn.labels(300, 2200, num_ids=400, num_cams=6, seed=12)
    qf, gf = syn.features(qp, gp, dim=256, seed=12, noise=3.0)
    feats = oracle.l2norm(np.concatenate([qf, gf]))
    final = _rr().re_ranking(torch.from_numpy(feats[:300]), torch.from_numpy(feats[300:]), 50, 15, 0.3)
    ref = oracle.re_ranking(feats[:300], feats[300:], 50, 15, 0.3)
    assert np.array_equal(final.view(np.uint32), ref.view(np.uint32))


def test_rerank_duke_scale_properties(gpu):
    """Duke-size (2228 x 17661) run: completes within capacity, distances bounded, and the
    re-ranked eval runs end to end (R1_mAP_eval(reranking=True), evaluate.py:124-127)."""
    from multimodal_reid_amd import evaluate
    sp = syn.DATASET_SPLITS["dukemtmc"]
    qp, gp, qc, gc = syn.labels(sp["num_query"], sp["num_gallery"], sp["num_ids"], sp["num_cams"], seed=13)
    r = np.random.default_rng(13)
    cent = r.standard_normal((sp["num_ids"] + 1, 512)).astype(np.float32)
    pids = np.concatenate([qp, gp])
    feats = cent[np.clip(pids, 0, None)] + 1.5 * r.standard_normal((len(pids), 512)).astype(np.float32)
    ev = evaluate.R1_mAP_eval(sp["num_query"], max_rank=50, feat_norm=True, reranking=True)
    ev.reset()
    ev.update((torch.from_numpy(feats), pids, np.concatenate([qc, gc])))
    cmc, mAP = ev.compute()
    assert 0.0 < mAP <= 1.0 and cmc[0] <= cmc[-1]
    fn = evaluate.l2_normalize_device(torch.from_numpy(feats))
    final = _rr().re_ranking_device(fn[:sp["num_query"]], fn[sp["num_query"]:], 50, 15, 0.3)
    assert torch.isfinite(final).all() and float(final.min()) >= 0.0 and float(final.max()) <= 1.001  # fp16(0.7) = 0.7002
