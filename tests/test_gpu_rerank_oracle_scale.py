"""The re-rank the product runs at benchmark size, pinned to the oracle (VERDICT r5 Next #1).

From N >= reranking.STAGED_MIN_N (16 384) `re_ranking_device` and `R1_mAP_eval(reranking=True)`
take the staged path (reidmi_rr_*) with R2 through the fp16 pre-filter in the GEMM epilogue.
Until round 5 that path was compared with the oracle only below N ~ 2 500 and, at DukeMTMC size,
only with the GPU one-call kernels.  Here it is compared with `oracle.re_ranking` (the C
restatement of reranking.py:29-100, pinned to the reference's own fixtures by
tests/test_oracle.py) on the SAME normalised features at configs[2]'s size, 2228 q x 17661 g
(N = 19 889), D = 1280 — bit for bit on every one of the 39.3 M re-ranked distances — and the
re-ranked CMC/mAP of the drop-in `R1_mAP_eval` (evaluate.py:124-132) equal `oracle.eval_func`
(evaluate.py:29-88) on the oracle's own distances.

The oracle's full Duke re-rank takes ~7 s on 16 host threads (bench.py's rerank cpu_port)."""
import os

import numpy as np
import pytest
import torch

import oracle
from multimodal_reid_amd import synthetic as syn

pytestmark = pytest.mark.gpu


def _duke(case):
    sp = syn.DATASET_SPLITS["dukemtmc"]
    Q, G = sp["num_query"], sp["num_gallery"]
    qp, gp, qc, gc = syn.labels(Q, G, sp["num_ids"], sp["num_cams"], seed=0, distractor_frac=0.1, junk_frac=0.02)
    if case == "clustered":  # bench.py rerank_leg's features
        qf, gf = syn.features(qp, gp)
    else:
        # tracklets: the gallery is groups of 24 near-identical crops of one identity (MSMT17 /
        # Duke video-style), i.e. dense near-ties and duplicate-heavy k-reciprocal neighbourhoods
        r = np.random.default_rng(23)
        qf, gf = syn.features(qp, gp, seed=23, noise=2.0)
        base = gf[::24].repeat(24, axis=0)[:G]
        gf = (base + 1e-3 * r.standard_normal(base.shape)).astype(np.float32)
        gp = np.ascontiguousarray(gp[::24].repeat(24)[:G])
        gc = np.ascontiguousarray(gc[::24].repeat(24)[:G])
    return Q, G, qp, gp, qc, gc, qf, gf


_ORACLE_CACHE = {}


def _oracle_final(key, qn, gn, k1, k2):
    if key not in _ORACLE_CACHE:
        oracle.set_threads(min(16, os.cpu_count() or 1))
        _ORACLE_CACHE[key] = oracle.re_ranking(qn, gn, k1, k2, 0.3)
    return _ORACLE_CACHE[key]


@pytest.mark.parametrize("case,k1,k2", [("clustered", 50, 15), ("clustered", 20, 6), ("tracklets", 50, 15)])
def test_staged_rerank_duke_size_bitexact_vs_oracle(gpu, case, k1, k2):
    from multimodal_reid_amd import evaluate, reranking
    Q, G, qp, gp, qc, gc, qf, gf = _duke(case)
    assert Q + G >= reranking.STAGED_MIN_N  # the drop-in takes the staged path here
    qn = evaluate.l2_normalize_device(torch.from_numpy(qf).to(gpu))
    gn = evaluate.l2_normalize_device(torch.from_numpy(gf).to(gpu))
    # the normalisation itself is the oracle's (F.normalize, evaluate.py:114) bit for bit
    qn_h, gn_h = qn.cpu().numpy(), gn.cpu().numpy()
    assert np.array_equal(qn_h.view(np.uint32), oracle.l2norm(qf).view(np.uint32))
    got = reranking.re_ranking_device(qn, gn, k1, k2, 0.3).cpu().numpy()
    stats = {}
    staged = reranking.re_ranking_sharded(qn, gn, k1, k2, 0.3, stats=stats).cpu().numpy()
    assert np.array_equal(staged.view(np.uint32), got.view(np.uint32))
    # the rows were decided by the fp16 pre-filter (in-epilogue selection), not the exact fallback
    assert stats["form"] in ("triangle", "row passes") and stats["exact_rows"] < 0.05 * stats["rows"], stats
    ref = _oracle_final((case, k1, k2), qn_h, gn_h, k1, k2)
    assert got.shape == ref.shape == (Q, G)
    diff = got.view(np.uint32) != ref.view(np.uint32)
    assert not diff.any(), f"{int(diff.sum())} of {diff.size} re-ranked distances differ from the oracle " \
                           f"(first at {np.argwhere(diff)[0].tolist()}); bisect with tools/rr_stages.py"
    print(f"[duke {case} k1={k1} k2={k2}] {Q}x{G}: bit-exact vs oracle; R2 form {stats['form']}, "
          f"exact-fallback rows {stats['exact_rows']} of {stats['rows']}")


@pytest.mark.parametrize("case", ["clustered", "tracklets"])
def test_r1_map_eval_reranking_duke_size_vs_oracle(gpu, case):
    """evaluate.py:124-132 (feat_norm -> re_ranking(50, 15, 0.3) -> eval_func) through the drop-in
    R1_mAP_eval from raw features: CMC and mAP equal the oracle's eval_func on the oracle's
    re-ranked distances, to the last bit."""
    from multimodal_reid_amd import evaluate
    Q, G, qp, gp, qc, gc, qf, gf = _duke(case)
    ev = evaluate.R1_mAP_eval(Q, max_rank=50, feat_norm=True, reranking=True)
    ev.reset()
    ev.update((torch.cat([torch.from_numpy(qf), torch.from_numpy(gf)]).to(gpu), np.concatenate([qp, gp]),
               np.concatenate([qc, gc])))
    cmc, mAP = ev.compute()
    ref = _oracle_final((case, 50, 15), oracle.l2norm(qf), oracle.l2norm(gf), 50, 15)
    cmc_o, map_o = oracle.eval_func(ref, qp, gp, qc, gc, 50)
    assert cmc.dtype == cmc_o.dtype and np.array_equal(cmc, cmc_o), np.abs(cmc - cmc_o).max()
    assert float(mAP) == float(map_o), (mAP, map_o)
    print(f"[duke {case}] R1_mAP_eval(reranking=True): mAP {mAP:.6f} rank-1 {cmc[0]:.6f} == oracle")
