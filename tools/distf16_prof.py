"""The fp16 distance mode (reidmi_distmat_f16) at Market size, for a rocprofv3 kernel trace:
casts, squared norms, the GEMM with its distance epilogue.

    rocprofv3 --kernel-trace --stats -d DIR -- python tools/distf16_prof.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import evaluate  # noqa: E402

Q, G, D = 3368, 15913, 1280
q = evaluate.l2_normalize_device(torch.randn(Q, D, device="cuda"))
g = evaluate.l2_normalize_device(torch.randn(G, D, device="cuda"))
out = torch.empty(Q, G, device="cuda")
for _ in range(10):
    evaluate.euclidean_distance_device(q, g, out=out, precision="fp16")
torch.cuda.synchronize()
print("ok")
