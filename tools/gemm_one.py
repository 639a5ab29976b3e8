"""Run one GEMM shape REPS times (for rocprofv3 --pmc / --kernel-trace passes and A/B of the
persistent tile walk).

    python tools/gemm_one.py M N K EPI [REPS] [fold] [--tile T] [--walk G,G,...]

EPI: 0 fp16, 1 QuickGELU fp16, 5 fp32, 6 fp16 residual.  Uniform random operands
(MI355X_MICROARCH.md: quote random-data numbers, not zero-filled).  "fold": the encoders'
folded-LayerNorm form (row statistics + colsum), EPI 0/1.  --walk times each N-group count."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import _lib as L  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("M", type=int)
    ap.add_argument("N", type=int)
    ap.add_argument("K", type=int)
    ap.add_argument("epi", type=int)
    ap.add_argument("reps", type=int, nargs="?", default=20)
    ap.add_argument("fold", nargs="?", default="")
    ap.add_argument("--tile", type=int, default=0)
    ap.add_argument("--walk", default="0")
    ap.add_argument("--warm", type=int, default=0)
    a = ap.parse_args()
    M, N, K, epi = a.M, a.N, a.K, a.epi
    dev = torch.device("cuda")
    A = (torch.rand(M, K, device=dev) * 2 - 1).half()
    W = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).half()
    b = torch.rand(N, device=dev)
    out = torch.zeros(M, N, device=dev) if epi == 5 else torch.zeros(M, N, device=dev, dtype=torch.float16)
    rs = cs = None
    if a.fold == "fold":
        rs = torch.stack([torch.rand(M + 256, device=dev) + 0.5, torch.rand(M + 256, device=dev) - 0.5], 1)
        cs = torch.rand(N, device=dev)
    base = (epi, L.ptr(A), K, L.ptr(W), K, M, N, K, L.ptr(b), L.ptr(rs), L.ptr(cs), L.ptr(out), N)
    for _ in range(a.warm):  # clocks up before the first timed walk
        L.call_tools("reidmi_gemm_f16_tiled", *base, a.tile, 0, L.stream())
    for walk in (int(w) for w in a.walk.split(",")):
        args = base + (a.tile, walk, L.stream())
        L.call_tools("reidmi_gemm_f16_tiled", *args)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            L.call_tools("reidmi_gemm_f16_tiled", *args)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        print(f"M={M} N={N} K={K} epi={epi} tile={a.tile} walk={walk}: {ms * 1e3:.1f} us  "
              f"{2.0 * M * N * K / ms / 1e9:.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
