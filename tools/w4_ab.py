"""The one-wave-per-SIMD GEMM prototype (reidmi_gemm_f16_w4) against the shipped persistent
kernel (reidmi_gemm_f16_tiled, tile 2) with the same plain fp16 + bias epilogue, on the
encoder's shapes at the bench batch; outputs compared bit for bit.  Also both without stores
(w4 nostore vs the shipped kernel's mainloop ceiling from the GEMM_VAR_* builds is recorded
separately).
    python tools/w4_ab.py [M] [ROUNDS]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import _lib as L  # noqa: E402

SHAPES = [("cfc", 3072, 768), ("outp", 768, 768), ("projp", 768, 3072), ("qkv", 2304, 768)]


def timeit(fn, reps=5):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 864256
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    dev = torch.device("cuda")
    for r in range(rounds):
        for name, N, K in SHAPES:
            A = (torch.rand(M, K, device=dev) * 2 - 1).half()
            W = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).half()
            b = torch.rand(N, device=dev)
            o1 = torch.empty(M, N, device=dev, dtype=torch.float16)
            o2 = torch.empty(M, N, device=dev, dtype=torch.float16)
            fl = 2.0 * M * N * K
            base = lambda: L.call_tools("reidmi_gemm_f16_tiled", 0, L.ptr(A), K, L.ptr(W), K, M, N, K, L.ptr(b), None,
                                        None, L.ptr(o1), N, 2, 0, L.stream())
            w4 = lambda: L.call_tools("reidmi_gemm_f16_w4", L.ptr(A), K, L.ptr(W), K, M, N, K, L.ptr(b), L.ptr(o2), N,
                                      0, L.stream())
            w4n = lambda: L.call_tools("reidmi_gemm_f16_w4", L.ptr(A), K, L.ptr(W), K, M, N, K, L.ptr(b), L.ptr(o2), N,
                                       1, L.stream())
            t_b = timeit(base)
            t_w = timeit(w4)
            same = torch.equal(o1, o2)
            t_n = timeit(w4n)
            print(f"r{r} {name:5s} M={M} N={N} K={K}: persistent {fl / t_b / 1e9:7.1f}  w4 {fl / t_w / 1e9:7.1f}  "
                  f"w4-nostore {fl / t_n / 1e9:7.1f} TF/s  {'bit-identical' if same else 'DIFFERENT'}", flush=True)
            del A, W, b, o1, o2
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
