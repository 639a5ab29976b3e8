"""In-process A/B of the persistent GEMM's tile walk (XCD N-groups) at the bench's launch size:
ngroups 1 (one group, M-major), 2 (two XCD groups, N split evenly between them: c_fc's auto),
and -2 / -3 (one group, the tile sequence ordered by N-slices, so each XCD's contiguous range
covers mostly one slice's W panels whatever the slice count).  Outputs are checked
bit-identical across walks.

    python tools/walk_ab.py [ROUNDS] [--shapes qkv,cfc] [--walks 1,2,-2,-3] [--M 4068291]"""
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
    ap.add_argument("--walks", default="1,2,-2,-3")
    ap.add_argument("--shapes", default="qkv,cfc")
    ap.add_argument("--M", type=int, default=19281 * 211)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda")
    M = a.M
    walks = [int(w) for w in a.walks.split(",")]
    for r in range(a.rounds):
        for name in a.shapes.split(","):
            N, K, epi, fold = SHAPES[name]
            g = torch.Generator(device=dev).manual_seed(1)
            A = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).half()
            W = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) / K ** 0.5).half()
            b = torch.rand(N, device=dev, generator=g)
            rs = cs = None
            if fold:
                rs = torch.stack([torch.rand(M + 256, device=dev, generator=g) + 0.5,
                                  torch.rand(M + 256, device=dev, generator=g) - 0.5], 1)
                cs = torch.rand(N, device=dev, generator=g)
            ref = None
            for w in walks:
                out = torch.zeros(M, N, device=dev, dtype=torch.float16)
                args = (epi, L.ptr(A), K, L.ptr(W), K, M, N, K, L.ptr(b), L.ptr(rs), L.ptr(cs), L.ptr(out), N, 2, w,
                        L.stream())
                if epi == 6:  # residual epilogue: a fresh residual for the check, then timing
                    out.copy_(A[:, :N] if N <= K else out)
                L.call_tools("reidmi_gemm_f16_tiled", *args)
                torch.cuda.synchronize()
                same = ""
                if epi != 6:
                    if ref is None:
                        ref = out.clone()
                    else:
                        same = " bit-identical" if torch.equal(out.view(torch.int16), ref.view(torch.int16)) else " DIFFERENT"
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    L.call_tools("reidmi_gemm_f16_tiled", *args)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / a.reps
                print(f"r{r} {name:5s} M={M} N={N} K={K} walk={w:2d}: {ms * 1e3:9.1f} us "
                      f"{2.0 * M * N * K / ms / 1e9:7.1f} TF/s{same}", flush=True)
                del out
            del A, W, ref
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
