"""Our fp16 GEMM (auto tile, fp16-store epilogue) vs torch.matmul (hipBLASLt) on the
encoder's shapes, interleaved in one process.  Prints TFLOP/s medians."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import _lib as L  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 512 * 211
SHAPES = [("qkv", 2304, 768), ("out_proj", 768, 768), ("c_fc", 3072, 768), ("c_proj", 768, 3072)]


def timeit(fn, n=10):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    dev = torch.device("cuda")
    res = {}
    for _ in range(5):
        for name, N, K in SHAPES:
            A = (torch.rand(M, K, device=dev) * 2 - 1).half()
            W = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).half()
            b = torch.rand(N, device=dev)
            o = torch.empty(M, N, device=dev, dtype=torch.float16)
            args = (0, L.ptr(A), K, L.ptr(W), K, M, N, K, L.ptr(b), None, None, L.ptr(o), N, L.stream())
            fl = 2.0 * M * N * K
            ms = timeit(lambda: L.call("reidmi_gemm_f16", *args))
            res.setdefault((name, "ours"), []).append(fl / ms / 1e9)
            ms = timeit(lambda: torch.matmul(A, W.t(), out=o))
            res.setdefault((name, "hipblaslt"), []).append(fl / ms / 1e9)
            bb = b.half()
            ms = timeit(lambda: torch.addmm(bb, A, W.t(), out=o))
            res.setdefault((name, "hipblaslt+bias"), []).append(fl / ms / 1e9)
    for name, N, K in SHAPES:
        line = [f"{name:9s} M={M} N={N} K={K}"]
        for v in ("ours", "hipblaslt", "hipblaslt+bias"):
            xs = sorted(res[(name, v)])
            line.append(f"{v}: {xs[len(xs) // 2]:7.1f}")
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
