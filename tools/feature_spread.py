"""How concentrated are the synthetic network's embeddings?  For residual-branch gains of the
synthetic CLIP-ReID checkpoint (synthetic.vit_state_dict resid_gain) and per-image crop noise:
embed identity-structured crops (2 TTA passes), CMC/mAP, the spread of the normalised features
(mean pairwise cosine to the feature mean), and the staged re-rank's R2 statistics (rows sent
to the exact fallback).

    python tools/feature_spread.py [Q G IDS] [--gains 1,2,4] [--noise 0.6,0.3]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import evaluate, reranking, utils  # noqa: E402
from multimodal_reid_amd import synthetic as syn  # noqa: E402
from multimodal_reid_amd import zero_shot_learning as zsl  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("Q", type=int, nargs="?", default=2000)
    ap.add_argument("G", type=int, nargs="?", default=16000)
    ap.add_argument("ids", type=int, nargs="?", default=800)
    ap.add_argument("--gains", default="1,2,4")
    ap.add_argument("--noise", default="0.6,0.3")
    a = ap.parse_args()
    qp, gp, qc, gc = syn.labels(a.Q, a.G, num_ids=a.ids, num_cams=6, seed=5, distractor_frac=0.1)
    pids, cams = np.concatenate([qp, gp]), np.concatenate([qc, gc])
    offs = syn.tta_offsets(a.Q + a.G, seed=5)
    for noise in (float(x) for x in a.noise.split(",")):
        t0 = time.time()
        imgs = syn.identity_crops(pids, cams, seed=5, noise=noise)
        print(f"crops noise {noise}: {time.time() - t0:.1f} s", flush=True)
        for gain in (float(x) for x in a.gains.split(",")):
            model, _, _ = utils.model_adaptor(None, 256, 128, syn.clipreid_checkpoint("ViT-B/16", seed=20,
                                                                                     resid_gain=gain))
            feats = []
            for s in range(0, len(imgs), 512):
                feats.append(zsl.embed_pair(model, torch.from_numpy(imgs[s:s + 512]), tta=offs[s:s + 512]))
            f = torch.cat(feats)
            n = evaluate.l2_normalize_device(f)
            mu = n.mean(0)
            spread = float((n @ (mu / mu.norm())).mean())
            args = (f[a.Q:], f[:a.Q], torch.from_numpy(gp), torch.from_numpy(qp), torch.from_numpy(gc),
                    torch.from_numpy(qc))
            cmc, mAP = zsl.get_cmc_map(*args)
            st = {}
            torch.cuda.synchronize()
            t0 = time.time()
            fin = reranking.re_ranking_sharded(n[:a.Q], n[a.Q:], 50, 15, 0.3, stats=st)
            torch.cuda.synchronize()
            dt = time.time() - t0
            valid, first, ap_, nk, ovf = evaluate.eval_rows_device(fin, torch.from_numpy(qp).cuda(),
                                                                   torch.from_numpy(gp).cuda(),
                                                                   torch.from_numpy(qc).cuda(),
                                                                   torch.from_numpy(gc).cuda())
            rows = torch.stack([valid.double(), first.double(), ap_, nk.double()], 1).cpu().numpy()
            rcmc, rmap = evaluate.aggregate_cmc_map(rows[:, 0].astype(np.int64), rows[:, 1].astype(np.int64),
                                                    rows[:, 2], rows[:, 3].astype(np.int64), a.G, 50)
            print(f"noise {noise} gain {gain}: mAP {mAP:.4f} r1 {cmc[0]:.4f}; cos to mean {spread:.4f}; "
                  f"re-rank mAP {rmap:.4f} r1 {rcmc[0]:.4f} in {dt:.3f} s, R2 {st.get('form')} "
                  f"exact rows {st.get('exact_rows')}/{st.get('rows')}", flush=True)
            del model, f, n, fin
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
