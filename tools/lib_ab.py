"""In-process A/B of whole library builds (tools/build_variant.py) on the encoder's GEMM
shapes: rounds x (shape, library), interleaved in one process (cdna_hip_programming.md rule
24); random operands, folded LayerNorm where the encoder folds it.

    python tools/lib_ab.py LIB.so[,LIB2.so,...] [ROUNDS] [--shapes cfc,qkv,out,proj] [--M 216064]"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import _lib as L  # noqa: E402

SHAPES = {"cfc": (3072, 768, 1, True), "qkv": (2304, 768, 0, True), "out": (768, 768, 6, False),
          "proj": (768, 3072, 6, False), "outp": (768, 768, 6, "pst"), "projp": (768, 3072, 6, "pst")}
# "outp" / "projp": the encoder's form of out_proj / c_proj (residual + LayerNorm partials,
# reidmi_gemm_f16_resid_partials)


def open_lib(path):
    lib = ctypes.CDLL(os.path.abspath(path))
    lib.reidmi_last_error.restype = ctypes.c_char_p
    for name, args in L.SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = ctypes.c_int64 if name.endswith("_bytes") or name in L.INT64_RESULT else ctypes.c_int32
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs")
    ap.add_argument("rounds", type=int, nargs="?", default=3)
    ap.add_argument("--shapes", default="cfc,qkv,out,proj")
    ap.add_argument("--M", type=int, default=216064)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    libs = [(os.path.basename(p), open_lib(p)) for p in a.libs.split(",")]
    dev = torch.device("cuda")
    M = a.M
    for r in range(a.rounds):
        for name in a.shapes.split(","):
            N, K, epi, fold = SHAPES[name]
            g = torch.Generator(device=dev).manual_seed(r)
            A = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).half()
            W = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) / K ** 0.5).half()
            b = torch.rand(N, device=dev, generator=g)
            out = (torch.rand(M, N, device=dev, generator=g) - 0.5).half()
            rs = cs = None
            pst = torch.empty((N // 64) * M * 2, device=dev) if fold == "pst" else None
            if fold is True:
                rs = torch.stack([torch.rand(M + 256, device=dev) + 0.5, torch.rand(M + 256, device=dev) - 0.5], 1)
                cs = torch.rand(N, device=dev)
            if pst is not None:
                fn_name = "reidmi_gemm_f16_resid_partials"
                args = (L.ptr(A), K, L.ptr(W), K, M, N, K, L.ptr(b), L.ptr(out), N, L.ptr(pst), L.stream())
            else:
                fn_name = "reidmi_gemm_f16"
                args = (epi, L.ptr(A), K, L.ptr(W), K, M, N, K, L.ptr(b), L.ptr(rs), L.ptr(cs), L.ptr(out), N,
                        L.stream())
            for lname, lib in libs:
                fn = getattr(lib, fn_name)
                for _ in range(3):
                    assert fn(*args) == 0, lib.reidmi_last_error()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    fn(*args)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / a.reps
                print(f"r{r} {name:5s} M={M} N={N} K={K} {lname:28s}: {ms * 1e3:8.1f} us "
                      f"{2.0 * M * N * K / ms / 1e9:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
