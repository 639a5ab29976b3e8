"""A/B timing of the GEMM tile variants on the encoder's shapes, interleaved in one
process (cdna_hip_programming.md rule 24).  Prints TFLOP/s per (shape, variant)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import _lib as L  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 512 * 211
SHAPES = [("qkv", 2304, 768, 3), ("out_proj", 768, 768, 6), ("c_fc", 3072, 768, 1), ("c_proj", 768, 3072, 6)]
VARIANTS = [int(v) for v in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["2", "3"])]
ROUNDS = 5


def main():
    dev = torch.device("cuda")
    res = {}
    bufs = {}
    for name, N, K, epi in SHAPES:
        A = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        W = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).bfloat16()
        b = torch.rand(N, device=dev)
        if epi in (2,):
            out = torch.zeros(M, N, device=dev)
        elif epi == 6:
            out = torch.zeros(M, N, device=dev, dtype=torch.float16)
        elif epi == 3:
            out = None
        else:
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        bufs[name] = (A, W, b, out)
    qkv_out = [torch.empty(M * 768, device=dev, dtype=torch.bfloat16) for _ in range(3)]
    for r in range(ROUNDS):
        for name, N, K, epi in SHAPES:
            A, W, b, out = bufs[name]
            for v in VARIANTS:
                L.call("reidmi_gemm_set_variant", v)
                if epi == 3:  # head-split epilogue is not exposed; time the bf16 store epilogue instead
                    o = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                    args = (0, L.ptr(A), K, L.ptr(W), K, M, N, K, L.ptr(b), L.ptr(o), N, L.stream())
                else:
                    args = (epi, L.ptr(A), K, L.ptr(W), K, M, N, K, L.ptr(b), L.ptr(out), N, L.stream())
                L.call("reidmi_gemm_bf16", *args)  # warm
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                n = 10
                for _ in range(n):
                    L.call("reidmi_gemm_bf16", *args)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / n
                res.setdefault((name, v), []).append(2.0 * M * N * K / ms / 1e9)
    L.call("reidmi_gemm_set_variant", 0)
    for name, N, K, epi in SHAPES:
        line = [f"{name:9s} M={M} N={N} K={K}"]
        for v in VARIANTS:
            xs = sorted(res[(name, v)])
            line.append(f"v{v}: med {xs[len(xs) // 2]:7.1f} min {xs[0]:7.1f} TF/s")
        print("  ".join(line))


if __name__ == "__main__":
    main()
