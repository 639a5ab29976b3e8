"""The staged re-rank the drop-in runs at MSMT17 size (configs[3]: 11 659 q x 82 161 g, N = 93 820,
D = 1280, bench.py msmt17 leg's SURVEY §8d features and labels) against the C oracle's dense
re_ranking (oracle/reid_oracle.c, reranking.py:29-100) bit for bit, plus eval_func's CMC / mAP on
both.  A one-off record, not a -m gpu test: the oracle's dense N x N formulation needs ~110 GB of
host memory and minutes on 16 threads at this size (tests/test_gpu_rerank_oracle_scale.py pins the
same path at DukeMTMC size inside the suite).

    python tools/rerank_scale_oracle.py [msmt17|dukemtmc|market1501] [THREADS]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
import oracle  # noqa: E402
from multimodal_reid_amd import evaluate, reranking, synthetic as syn  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "msmt17"
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    sp = syn.DATASET_SPLITS[name]
    Q, G = sp["num_query"], sp["num_gallery"]
    qp, gp, qc, gc = syn.labels(Q, G, sp["num_ids"], sp["num_cams"], seed=0, distractor_frac=0.1, junk_frac=0.02)
    qf, gf = syn.features(qp, gp, dim=1280, seed=0)
    dev = torch.device("cuda")
    qn = evaluate.l2_normalize_device(torch.from_numpy(qf).to(dev))
    gn = evaluate.l2_normalize_device(torch.from_numpy(gf).to(dev))
    qn_h, gn_h = qn.cpu().numpy(), gn.cpu().numpy()
    assert np.array_equal(qn_h.view(np.uint32), oracle.l2norm(qf).view(np.uint32))
    reranking.re_ranking_device(qn[:200], gn[:16384], 50, 15, 0.3)  # kernel loads
    torch.cuda.synchronize()
    t = time.perf_counter()
    got_d = reranking.re_ranking_device(qn, gn, 50, 15, 0.3)
    torch.cuda.synchronize()
    t_gpu = time.perf_counter() - t
    stats = {}
    reranking.re_ranking_sharded(qn, gn, 50, 15, 0.3, stats=stats)
    cmc_g, map_g = evaluate.eval_func_device(got_d, qp, gp, qc, gc)
    got = got_d.cpu().numpy()
    del got_d
    torch.cuda.empty_cache()
    print(f"[{name}] GPU staged re-rank {t_gpu:.3f} s (R2 form {stats.get('form')}, exact-fallback rows "
          f"{stats.get('exact_rows')} of {stats.get('rows')}); oracle on {threads} threads ...", flush=True)
    oracle.set_threads(threads)
    t = time.perf_counter()
    ref = oracle.re_ranking(qn_h, gn_h, 50, 15, 0.3)
    t_cpu = time.perf_counter() - t
    diff = got.view(np.uint32) != ref.view(np.uint32)
    cmc_o, map_o = oracle.eval_func(ref, qp, gp, qc, gc, 50)
    out = {"config": f"{name} {Q}q x {G}g (N={Q + G}), D=1280 SURVEY §8d features, k1=50 k2=15 lambda=0.3",
           "distances": int(diff.size), "distances_differing": int(diff.sum()),
           "cmc_equal": bool(np.array_equal(cmc_g, cmc_o)), "map_gpu": float(map_g), "map_oracle": float(map_o),
           "map_equal": float(map_g) == float(map_o), "gpu_s": round(t_gpu, 3), "oracle_s": round(t_cpu, 1),
           "oracle_threads": threads, "r2_form": stats.get("form"), "r2_exact_rows": stats.get("exact_rows")}
    print(json.dumps(out), flush=True)
    sys.exit(0 if out["distances_differing"] == 0 and out["cmc_equal"] and out["map_equal"] else 1)


if __name__ == "__main__":
    main()
