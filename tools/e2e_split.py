"""Split the end-to-end mAP error (tests/test_gpu_pipeline.py test_end_to_end_accuracy_vs_reference):
our re-rank / eval on the REFERENCE's own features (tools/diag/e2e_ref_feats.npz, written by
tests/golden/make_goldens.py --only e2e; not committed) against the reference's mAPs, and the
per-row error of our features against the reference's fp32 features next to its fp16 run's.
    python tools/e2e_split.py"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import synthetic as syn, utils, zero_shot_learning as zsl  # noqa: E402

g = np.load(os.path.join(REPO, "tests", "golden", "e2e.npz"))
ref = np.load(os.path.join(REPO, "tools", "diag", "e2e_ref_feats.npz"))
qp, gp, qc, gc = g["q_pids"], g["g_pids"], g["q_cams"], g["g_cams"]
Q = len(qp)
lab = (torch.from_numpy(gp), torch.from_numpy(qp), torch.from_numpy(gc), torch.from_numpy(qc))


def maps(f):
    f = torch.from_numpy(f).cuda() if isinstance(f, np.ndarray) else f
    return zsl.get_cmc_map(f[Q:], f[:Q], *lab)[1], zsl.get_cmc_map(f[Q:], f[:Q], *lab, reranking=True)[1]


for tag in ("fp32", "fp16"):
    m, r = maps(ref[tag])
    print(f"reference {tag} features through our eval: mAP {m:.6f} (ref {float(g['map_' + tag]):.6f}), "
          f"re-ranked {r:.6f} (ref {float(g['map_rr_' + tag]):.6f})")
imgs = syn.identity_crops(np.concatenate([qp, gp]), np.concatenate([qc, gc]), seed=21)
model, _, _ = utils.model_adaptor(None, 256, 128, syn.clipreid_checkpoint("ViT-B/16", seed=20))
out = []
for s in range(0, len(imgs), 64):
    out.append(zsl.embed_pair(model, torch.from_numpy(imgs[s:s + 64]), tta=g["tta_offsets"][s:s + 64]))
ours = torch.cat(out)
m, r = maps(ours)
print(f"ours: mAP {m:.6f} (d {m - float(g['map_fp32']):+.2e}), re-ranked {r:.6f} (d {r - float(g['map_rr_fp32']):+.2e})")
o = ours.cpu().numpy().astype(np.float64)
f32, f16 = ref["fp32"].astype(np.float64), ref["fp16"].astype(np.float64)
eo, e16 = np.abs(o - f32).max(1), np.abs(f16 - f32).max(1)
print(f"per-row max|err| vs ref fp32: ours median {np.median(eo):.3g} max {eo.max():.3g}; "
      f"ref fp16 median {np.median(e16):.3g} max {e16.max():.3g}; rows where ours > ref fp16: {(eo > e16).mean():.3f}")
