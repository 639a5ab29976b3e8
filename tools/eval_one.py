"""Time reidmi_eval_rows on a Market- or MSMT17-size distance matrix (random distances,
synthetic labels):  python tools/eval_one.py [market1501|msmt17] [REPS]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import evaluate, synthetic as syn  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "market1501"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    sp = syn.DATASET_SPLITS[name]
    Q, G = sp["num_query"], sp["num_gallery"]
    qp, gp, qc, gc = syn.labels(Q, G, sp["num_ids"], sp["num_cams"], seed=0, junk_frac=0.02)
    dev = torch.device("cuda")
    d = torch.rand(Q, G, device=dev)
    args = [torch.from_numpy(a).to(dev) for a in (qp, gp, qc, gc)]
    evaluate.eval_rows_device(d, *args)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        evaluate.eval_rows_device(d, *args)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    nb = 4.0 * Q * G + 16.0 * G
    print(f"eval_rows {name} {Q}x{G}: {ms * 1e3:.1f} us  {nb / ms / 1e6:.1f} GB/s ({nb / ms / 1e6 / 8000:.3f} of 8 TB/s)")


if __name__ == "__main__":
    main()
