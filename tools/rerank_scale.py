"""Time the staged re-ranking (re_ranking_sharded, one process) at DukeMTMC and MSMT17
sizes on identity-clustered synthetic features, per stage; and the one-call path at Duke.

    python tools/rerank_scale.py [duke|msmt17 ...]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import evaluate, reranking, synthetic as syn  # noqa: E402


class Timed(reranking.HipStages):
    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.t = {}

    def _time(self, name, fn, *a):
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = fn(*a)
        torch.cuda.synchronize()
        self.t[name] = round(time.perf_counter() - t, 4)
        return r

    def rank_rows(self, lo, hi):
        return self._time("rank_rows", super().rank_rows, lo, hi)

    def v_rows(self, *a):
        return self._time("v_rows", super().v_rows, *a)

    def qe_rows(self, *a):
        return self._time("qe_rows", super().qe_rows, *a)

    def jaccard_rows(self, *a):
        return self._time("csc+jaccard", super().jaccard_rows, *a)


def main():
    dev = torch.device("cuda")
    for name in sys.argv[1:] or ["duke", "msmt17"]:
        sp = syn.DATASET_SPLITS["dukemtmc" if name == "duke" else name]
        Q, G = sp["num_query"], sp["num_gallery"]
        qp, gp, qc, gc = syn.labels(Q, G, sp["num_ids"], sp["num_cams"], seed=0, distractor_frac=0.1, junk_frac=0.02)
        qf, gf = syn.features(qp, gp)
        qn = evaluate.l2_normalize_device(torch.from_numpy(qf).to(dev))
        gn = evaluate.l2_normalize_device(torch.from_numpy(gf).to(dev))
        feat = torch.cat([qn, gn]).contiguous()
        for rep in range(2):
            st = Timed(feat, Q, 50, 15, 0.3)
            torch.cuda.synchronize()
            t = time.perf_counter()
            out = reranking.staged_rerank(st, Q + G, Q)
            torch.cuda.synchronize()
            wall = time.perf_counter() - t
        print(f"{name} Q={Q} G={G} staged wall {wall:.3f} s  stages {st.t}  "
              f"peak mem {torch.cuda.max_memory_allocated() / 2**30:.1f} GiB", flush=True)
        if name == "duke":
            for rep in range(2):
                torch.cuda.synchronize()
                t = time.perf_counter()
                one = reranking.re_ranking_device(qn, gn, 50, 15, 0.3)
                torch.cuda.synchronize()
                wall1 = time.perf_counter() - t
            print(f"duke one-call wall {wall1:.3f} s  equal {torch.equal(one.view(torch.int32), out.view(torch.int32))}",
                  flush=True)
        del out, st, feat


if __name__ == "__main__":
    main()
