"""bench.py's MSMT17 leg alone (configs[3] on one GPU: sharded embed of the random-weight
ViT-B/16, exact distmat + CMC/mAP, staged re-rank + CMC/mAP), then the staged re-rank of the
same features with the R2 fp16 pre-filter on / off, interleaved:  python tools/msmt17_leg.py"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from multimodal_reid_amd import evaluate, reranking, synthetic as syn  # noqa: E402
from multimodal_reid_amd.model import VisionTransformer  # noqa: E402

dev = torch.device("cuda")
torch.cuda.set_device(0)
model = VisionTransformer(syn.vit_state_dict("ViT-B/16", seed=0), device=dev)
print(json.dumps(bench.msmt17_leg(model, dev, 0, 1, 1024)), flush=True)
wl = bench.Workload(dev, 0, 1, 1024, dataset="msmt17", model=model)
wl.embed()
qn, gn = evaluate.l2_normalize_device(wl.q_emb), evaluate.l2_normalize_device(wl.g_emb)
ref = None
for r in range(2):
    for pf in (True, False):
        reranking.RANK_PREFILTER = pf
        torch.cuda.synchronize()
        t = time.perf_counter()
        out = reranking.re_ranking_sharded(qn, gn, 50, 15, 0.3)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        same = "" if ref is None else (" bit-identical" if torch.equal(ref.view(torch.int32), out.view(torch.int32))
                                       else " DIFFERENT")
        ref = out if ref is None else ref
        print(f"r{r} staged re-rank of the random-network features, prefilter={pf}: {dt:.3f} s{same}", flush=True)
