"""Per-stage wall times of the staged k-reciprocal re-rank (reranking.staged_rerank, one
process) on bench.py's MSMT17 features: the embedded identity-structured crops (default) or
the §8d Gaussian features (--gaussian).  Each stage is synchronised on its own, so the sum is
a little above the unsynchronised call; the whole call is timed too.

    python tools/rr_stages.py [--gaussian] [--reps 3]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from multimodal_reid_amd import evaluate, reranking, synthetic as syn  # noqa: E402
from multimodal_reid_amd.model import VisionTransformer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gaussian", action="store_true")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.cuda.set_device(0)
    if a.gaussian:
        Q, G = 11659, 82161
        qp, gp, _, _ = syn.labels(Q, G, 3060, 15, seed=3, distractor_frac=0.1)
        qf, gf = syn.features(qp, gp, dim=1280, seed=0)
        qn = evaluate.l2_normalize_device(torch.from_numpy(qf).to(dev))
        gn = evaluate.l2_normalize_device(torch.from_numpy(gf).to(dev))
    else:
        sd = syn.vit_state_dict("ViT-B/16", seed=0, resid_gain=bench.MSMT17_RESID_GAIN)
        model = VisionTransformer(sd, device=dev)
        wl = bench.Workload(dev, 0, 1, 20480, dataset="msmt17", model=model, crops="identity")
        wl.embed()
        qn, gn = evaluate.l2_normalize_device(wl.q_emb), evaluate.l2_normalize_device(wl.g_emb)
        del wl, model
        torch.cuda.empty_cache()
    Q = qn.shape[0]
    feat = torch.cat([qn, gn]).contiguous()
    N = feat.shape[0]
    for r in range(a.reps):
        st = reranking.HipStages(feat, Q, 50, 15, 0.3)
        t = {}

        def lap(name, t0):
            torch.cuda.synchronize()
            t[name] = round(time.perf_counter() - t0, 4)
            return time.perf_counter()

        torch.cuda.synchronize()
        t0 = t_all = time.perf_counter()
        R, rmax = st.rank_rows(0, N)
        t0 = lap("R1_R2_rank_rows", t0)
        V = st.v_rows(R, rmax, 0, N)
        V = st.offsets(V[0]), V[1], V[2]
        t0 = lap("R3_v_rows", t0)
        Vq = st.qe_rows(R, V, 0, N)
        Vq = st.offsets(Vq[0]), Vq[1], Vq[2]
        t0 = lap("R4_qe_rows", t0)
        out = st.jaccard_rows(rmax, Vq, 0, Q)
        t0 = lap("R5_R7_jaccard_rows", t0)
        st.check()
        t["sum"] = round(time.perf_counter() - t_all, 4)
        t["nnz_V"] = int(V[0][-1].item())
        t["nnz_Vqe"] = int(Vq[0][-1].item())
        t["exact_rows"] = st.stats["exact_rows"]
        t["form"] = st.stats["form"]
        del out, R, rmax, V, Vq, st
        torch.cuda.synchronize()
        tw = time.perf_counter()
        out = reranking.re_ranking_sharded(qn, gn, 50, 15, 0.3)
        torch.cuda.synchronize()
        t["whole_call"] = round(time.perf_counter() - tw, 4)
        del out
        print(json.dumps({"features": "gaussian" if a.gaussian else "embedded", "N": N, "rep": r, **t}), flush=True)


if __name__ == "__main__":
    main()
