"""A/B of the end-to-end accuracy check (tests/test_gpu_pipeline.py
test_end_to_end_accuracy_vs_reference) across library builds: prints plain and re-ranked
mAP / rank-1 and top-10 agreement with the reference's fp32 run for each build.

    python tools/e2e_ab.py LIB.so[,LIB2.so,...]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import _lib, evaluate, synthetic as syn, utils  # noqa: E402
from multimodal_reid_amd import zero_shot_learning as zsl  # noqa: E402
from lib_ab import open_lib  # noqa: E402


def main():
    g = np.load(os.path.join(ROOT, "tests", "golden", "e2e.npz"))
    qp, gp, qc, gc = g["q_pids"], g["g_pids"], g["q_cams"], g["g_cams"]
    Q = len(qp)
    imgs = syn.identity_crops(np.concatenate([qp, gp]), np.concatenate([qc, gc]), seed=21)
    offs = g["tta_offsets"]
    for path in sys.argv[1].split(","):
        _lib._LIB = open_lib(path)
        model, _, _ = utils.model_adaptor(None, 256, 128, syn.clipreid_checkpoint("ViT-B/16", seed=20))
        feats = torch.cat([zsl.embed_pair(model, torch.from_numpy(imgs[s:s + 64]), tta=offs[s:s + 64])
                           for s in range(0, len(imgs), 64)])
        f = torch.cat([feats[:16], feats[Q:Q + 16]]).cpu().numpy().astype(np.float64)
        dev = np.abs(f - g["feat32_fp32"]).max()
        args = (feats[Q:], feats[:Q], torch.from_numpy(gp), torch.from_numpy(qp), torch.from_numpy(gc),
                torch.from_numpy(qc))
        cmc, mAP = zsl.get_cmc_map(*args)
        rcmc, rmap = zsl.get_cmc_map(*args, reranking=True)
        n = evaluate.l2_normalize_device(feats)
        ours = evaluate.topk_rows_device(evaluate.euclidean_distance_device(n[:Q], n[Q:]), 50).cpu().numpy()
        agree = float(np.mean([np.array_equal(a[:10], b[:10]) for a, b in zip(ours, g["rank50_fp32"])]))
        print(f"{os.path.basename(path):28s} max|f - f32| {dev:.5f}  mAP {mAP:.5f} (ref32 {float(g['map_fp32']):.5f} "
              f"ref16 {float(g['map_fp16']):.5f})  rr mAP {rmap:.5f} (ref32 {float(g['map_rr_fp32']):.5f} "
              f"ref16 {float(g['map_rr_fp16']):.5f})  r1 {cmc[0]:.4f}  top10 agree {agree:.3f}", flush=True)


if __name__ == "__main__":
    main()
