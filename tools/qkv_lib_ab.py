"""The QKV GEMM (ln_1 fold + head split, EPI_QKV) across library builds (tools/build_variant.py
gemm.hip variants, which carry the tools entry reidmi_gemm_f16_qkv), interleaved rounds at a
batch of B sequences; q / k / v^T outputs checked bit-identical across the builds.

    python tools/qkv_lib_ab.py LIB.so,LIB2.so [B] [ROUNDS]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import _lib as L  # noqa: E402

libs = [(os.path.basename(p), ctypes.CDLL(os.path.abspath(p))) for p in sys.argv[1].split(",")]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 19281
R = int(sys.argv[3]) if len(sys.argv) > 3 else 3
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
vt = torch.zeros(B * H * 64 * lp, dtype=torch.float16, device=dev)
vp = ctypes.c_void_p
args = [vp(A.data_ptr()), ctypes.c_int64(W), vp(Wt.data_ptr()), ctypes.c_int64(W), ctypes.c_int64(B), ctypes.c_int(Lt),
        ctypes.c_int(H), vp(b.data_ptr()), vp(rs.data_ptr()), vp(cs.data_ptr()), vp(q.data_ptr()), vp(k.data_ptr()),
        vp(vt.data_ptr()), ctypes.c_int(lp), vp(torch.cuda.current_stream().cuda_stream)]
ref = None
for r in range(R):
    for name, lib in libs:
        assert lib.reidmi_gemm_f16_qkv(*args) == 0
        torch.cuda.synchronize()
        same = ""
        outs = [t.view(torch.int16).clone() for t in (q, k, vt)] if r == 0 else None
        if outs is not None:
            if ref is None:
                ref = outs
            else:
                same = " bit-identical" if all(torch.equal(x, y) for x, y in zip(outs, ref)) else " DIFFERENT"
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            lib.reidmi_gemm_f16_qkv(*args)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        print(f"r{r} B={B} {name:24s}: {ms * 1e3:.1f} us {2.0 * M * N * W / ms / 1e9:.1f} TF/s{same}", flush=True)
