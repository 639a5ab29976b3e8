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
imgs = syn.identity_crops(np.concatenate([qp, gp]), np.concatenate([qc, gc]), seed=21, noise=float(g["noise"]))
model, _, _ = utils.model_adaptor(None, 256, 128, syn.clipreid_checkpoint("ViT-B/16", seed=20, resid_gain=float(g["resid_gain"])))
out = []
for s in range(0, len(imgs), 64):
    out.append(zsl.embed_pair(model, torch.from_numpy(imgs[s:s + 64]), tta=g["tta_offsets"][s:s + 64]))
ours = torch.cat(out)
m, r = maps(ours)
print(f"ours: mAP {m:.6f} (d {m - float(g['map_fp32']):+.2e}), re-ranked {r:.6f} (d {r - float(g['map_rr_fp32']):+.2e})")
o = ours.cpu().numpy().astype(np.float64)
if os.environ.get("E2E_DUMP"):
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    np.save(os.path.join(REPO, "gpurun_out", "e2e_ours_feats.npy"), ours.cpu().numpy())
f32, f16 = ref["fp32"].astype(np.float64), ref["fp16"].astype(np.float64)
eo, e16 = np.abs(o - f32).max(1), np.abs(f16 - f32).max(1)
print(f"per-row max|err| vs ref fp32: ours median {np.median(eo):.3g} max {eo.max():.3g}; "
      f"ref fp16 median {np.median(e16):.3g} max {e16.max():.3g}; rows where ours > ref fp16: {(eo > e16).mean():.3f}")

# Sensitivity of the metrics to feature error of the reference fp16 run's size: the reference's
# fp32 features plus its own fp16-minus-fp32 error, row-permuted (same magnitudes, other rows), in
# 8 seeded draws; rank-1 / mAP spread, plain and re-ranked.
dlt = (f16 - f32)
res = []
for s in range(8):
    perm = np.random.default_rng(s).permutation(len(dlt))
    f = torch.from_numpy((f32 + dlt[perm]).astype(np.float32)).cuda()
    c, m = zsl.get_cmc_map(f[Q:], f[:Q], *lab)
    rc, rm = zsl.get_cmc_map(f[Q:], f[:Q], *lab, reranking=True)
    res.append((c[0], m, rc[0], rm))
res = np.array(res, np.float64)
c_ref = (float(g["cmc_fp32"][0]), float(g["map_fp32"]), float(g["cmc_rr_fp32"][0]), float(g["map_rr_fp32"]))
for j, name in enumerate(("rank-1", "mAP", "re-ranked rank-1", "re-ranked mAP")):
    d = res[:, j] - c_ref[j]
    print(f"perturbed ref fp32 ({len(res)} draws): {name} - ref: min {d.min():+.2e} max {d.max():+.2e} "
          f"std {d.std():.2e}")
