"""Run the exact-fp32 distance kernel on one shape REPS times (rocprofv3 --pmc passes):
    python tools/distmat_one.py [Q G D] [REPS]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import evaluate  # noqa: E402


def main():
    a = [int(x) for x in sys.argv[1:]]
    Q, G, D = a[:3] if len(a) >= 3 else (11659, 82161, 1280)
    reps = a[3] if len(a) >= 4 else 3
    dev = torch.device("cuda")
    q, g = torch.randn(Q, D, device=dev), torch.randn(G, D, device=dev)
    out = torch.empty(Q, G, device=dev)
    evaluate.euclidean_distance_device(q, g, out=out)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        evaluate.euclidean_distance_device(q, g, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"distmat {Q}x{G}x{D}: {ms:.3f} ms  {2.0 * Q * G * D / ms / 1e9:.1f} TF/s")


if __name__ == "__main__":
    main()
