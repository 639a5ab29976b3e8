"""The QKV GEMM's head-split epilogue (q, k token-major rows; v^T scattered 2-byte stores)
against a plain fp16 output of the same M x 2304 x 768 product, ln_1 folded in both
(libreidmi_tools.so), interleaved rounds:  python tools/qkv_epi_ab.py [B] [ROUNDS]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import _lib as L  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
R = int(sys.argv[2]) if len(sys.argv) > 2 else 3
Lt, H, W = 211, 12, 768
M, N = B * Lt, 3 * W
dev = torch.device("cuda")
A = (torch.rand(M, W, device=dev) * 2 - 1).half()
Wt = ((torch.rand(N, W, device=dev) * 2 - 1) / W ** 0.5).half()
b = torch.rand(N, device=dev)
rs = torch.stack([torch.rand(M + 256, device=dev) + 0.5, torch.rand(M + 256, device=dev) - 0.5], 1)
cs = torch.rand(N, device=dev)
lp = L.load().reidmi_attn_lpad(Lt)
q = torch.empty(B * H * Lt * 64, dtype=torch.float16, device=dev)
k = torch.empty_like(q)
vt = torch.empty(B * H * 64 * lp, dtype=torch.float16, device=dev)
out = torch.empty(M, N, dtype=torch.float16, device=dev)
runs = {
    "EPI_QKV (head split)": lambda: L.call_tools("reidmi_gemm_f16_qkv", L.ptr(A), W, L.ptr(Wt), W, B, Lt, H, L.ptr(b),
                                                  L.ptr(rs), L.ptr(cs), L.ptr(q), L.ptr(k), L.ptr(vt), lp, L.stream()),
    "EPI_H16 (plain rows)": lambda: L.call_tools("reidmi_gemm_f16_tiled", 0, L.ptr(A), W, L.ptr(Wt), W, M, N, W,
                                                  L.ptr(b), L.ptr(rs), L.ptr(cs), L.ptr(out), N, 0, 0, L.stream()),
}
for r in range(R):
    for name, fn in runs.items():
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        print(f"r{r} B={B} {name}: {ms * 1e3:.1f} us {2.0 * M * N * W / ms / 1e9:.1f} TF/s", flush=True)
