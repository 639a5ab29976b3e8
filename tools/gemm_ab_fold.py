"""Interleaved A/B of GEMM variants on the encoder's fp16 LayerNorm-folded shapes (QKV head
split is timed with the bf16 store epilogue) and the residual shapes, one process:
    python tools/gemm_ab_fold.py M v1,v2,... [rounds]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import _lib as L  # noqa: E402


def main():
    M = int(sys.argv[1])
    vs = [int(v) for v in sys.argv[2].split(",")]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    dev = torch.device("cuda")
    shapes = [("qkv", 2304, 768, 0, True), ("c_fc", 3072, 768, 1, True), ("out_proj", 768, 768, 6, False),
              ("c_proj", 768, 3072, 6, False)]
    bufs = {}
    for name, N, K, epi, fold in shapes:
        A = (torch.rand(M, K, device=dev) * 2 - 1)
        W = (torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5
        b = torch.rand(N, device=dev)
        if fold:
            rs = torch.stack([torch.rand(M + 256, device=dev) + 0.5, torch.rand(M + 256, device=dev) - 0.5], 1)
            cs = torch.rand(N, device=dev)
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            bufs[name] = ("reidmi_gemm_f16", (A.half(), W.half(), b, rs, cs, out))
        else:
            out = torch.zeros(M, N, device=dev, dtype=torch.float16)
            bufs[name] = ("reidmi_gemm_bf16", (A.bfloat16(), W.bfloat16(), b, out))
    res = {}
    for _ in range(rounds):
        for name, N, K, epi, fold in shapes:
            fn, t = bufs[name]
            if fold:
                A, W, b, rs, cs, out = t
                args = (epi, L.ptr(A), K, L.ptr(W), K, M, N, K, L.ptr(b), L.ptr(rs), L.ptr(cs), L.ptr(out), N,
                        L.stream())
            else:
                A, W, b, out = t
                args = (epi, L.ptr(A), K, L.ptr(W), K, M, N, K, L.ptr(b), L.ptr(out), N, L.stream())
            for v in vs:
                L.call("reidmi_gemm_set_variant", v)
                L.call(fn, *args)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    L.call(fn, *args)
                e1.record()
                torch.cuda.synchronize()
                res.setdefault((name, v), []).append(2.0 * M * N * K / (e0.elapsed_time(e1) / 10) / 1e9)
    L.call("reidmi_gemm_set_variant", 0)
    for name, N, K, epi, fold in shapes:
        line = [f"{name:9s} M={M} N={N} K={K}"]
        for v in vs:
            xs = sorted(res[(name, v)])
            line.append(f"v{v}: {xs[len(xs) // 2]:7.1f}")
        print("  ".join(line), "TF/s (median)")


if __name__ == "__main__":
    main()
