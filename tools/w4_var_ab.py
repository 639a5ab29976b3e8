"""Timing variants of the one-wave-per-SIMD GEMM prototype across library builds
(tools/build_variant.py NAME gemm.hip -DREIDMI_TOOLS -DW4_VAR_...): the mainloop (no stores) of
each build on the encoder's shapes, interleaved rounds.
    python tools/w4_var_ab.py LIB.so[,LIB2.so,...] [ROUNDS] [M]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import _lib as L  # noqa: E402
from lib_ab import open_lib  # noqa: E402

SHAPES = [("cfc", 3072, 768), ("projp", 768, 3072)]


def main():
    libs = []
    for p in sys.argv[1].split(","):
        lib = open_lib(p)
        lib.reidmi_gemm_f16_w4.argtypes = L.TOOLS_SIGNATURES["reidmi_gemm_f16_w4"]
        lib.reidmi_gemm_f16_w4.restype = ctypes.c_int32
        libs.append((os.path.basename(p), lib))
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    M = int(sys.argv[3]) if len(sys.argv) > 3 else 864256
    dev = torch.device("cuda")
    for r in range(rounds):
        for name, N, K in SHAPES:
            A = (torch.rand(M, K, device=dev) * 2 - 1).half()
            W = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).half()
            b = torch.rand(N, device=dev)
            o = torch.empty(M, N, device=dev, dtype=torch.float16)
            fl = 2.0 * M * N * K
            for lname, lib in libs:
                args = (L.ptr(A), K, L.ptr(W), K, M, N, K, L.ptr(b), L.ptr(o), N, 1, L.stream())
                assert lib.reidmi_gemm_f16_w4(*args) == 0, lib.reidmi_last_error()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    lib.reidmi_gemm_f16_w4(*args)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / 5
                print(f"r{r} {name:5s} M={M} N={N} K={K} {lname:28s}: {ms * 1e3:8.1f} us {fl / ms / 1e9:7.1f} TF/s",
                      flush=True)
            del A, W, b, o
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
