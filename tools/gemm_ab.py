"""In-process A/B of the GEMM tilings on the encoder's shapes (random operands, folded
LayerNorm where the encoder folds it): rounds x (shape, tile), interleaved
(cdna_hip_programming.md rule 24).

    python tools/gemm_ab.py [ROUNDS] [--tiles 1,2] [--shapes cfc,qkv,out,proj] [--M 216064]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import _lib as L  # noqa: E402

SHAPES = {"cfc": (3072, 768, 1, True), "qkv": (2304, 768, 0, True), "out": (768, 768, 6, False),
          "proj": (768, 3072, 6, False)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("rounds", type=int, nargs="?", default=3)
    ap.add_argument("--tiles", default="2,3")
    ap.add_argument("--shapes", default="cfc,qkv,out,proj")
    ap.add_argument("--M", type=int, default=216064)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda")
    M = a.M
    bufs = {}
    for name in a.shapes.split(","):
        N, K, epi, fold = SHAPES[name]
        A = (torch.rand(M, K, device=dev) * 2 - 1).half()
        W = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).half()
        b = torch.rand(N, device=dev)
        out = (torch.rand(M, N, device=dev) - 0.5).half()
        rs = cs = None
        if fold:
            rs = torch.stack([torch.rand(M + 256, device=dev) + 0.5, torch.rand(M + 256, device=dev) - 0.5], 1)
            cs = torch.rand(N, device=dev)
        bufs[name] = (epi, L.ptr(A), K, L.ptr(W), K, M, N, K, L.ptr(b), L.ptr(rs), L.ptr(cs), L.ptr(out), N,
                      L.stream(), (A, W, b, out, rs, cs))
    tiles = [int(t) for t in a.tiles.split(",")]
    for r in range(a.rounds):
        for name, args in bufs.items():
            N, K = args[6], args[7]
            for t in tiles:
                targs = args[:13] + (t, 0, args[13])
                for _ in range(3):
                    L.call_tools("reidmi_gemm_f16_tiled", *targs)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    L.call_tools("reidmi_gemm_f16_tiled", *targs)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / a.reps
                print(f"r{r} {name:5s} M={M} N={N} K={K} tile={t}: {ms * 1e3:8.1f} us "
                      f"{2.0 * M * N * K / ms / 1e9:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
