"""Run one GEMM shape/variant REPS times (for rocprofv3 --pmc / --kernel-trace passes).

    python tools/gemm_one.py M N K EPI VARIANT [REPS] [fold]

EPI: 0 bf16, 1 QuickGELU bf16, 2 fp32 residual, 5 fp32.  Uniform random operands
(MI355X_MICROARCH.md: quote random-data numbers, not zero-filled).  "fold": the encoders'
fp16 GEMM with a folded LayerNorm (reidmi_gemm_f16 + row statistics + colsum), EPI 0/1."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import _lib as L  # noqa: E402


def main():
    M, N, K, epi, var = (int(v) for v in sys.argv[1:6])
    reps = int(sys.argv[6]) if len(sys.argv) > 6 else 20
    dev = torch.device("cuda")
    A = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
    W = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).bfloat16()
    b = torch.rand(N, device=dev)
    out = torch.zeros(M, N, device=dev) if epi in (2, 5) else torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    L.call("reidmi_gemm_set_variant", var)
    fold = len(sys.argv) > 7 and sys.argv[7] == "fold"
    if fold:
        A, W = A.half(), W.half()
        rs = torch.stack([torch.rand(M + 256, device=dev) + 0.5, torch.rand(M + 256, device=dev) - 0.5], 1)
        cs = torch.rand(N, device=dev)
        args = (epi, L.ptr(A), K, L.ptr(W), K, M, N, K, L.ptr(b), L.ptr(rs), L.ptr(cs), L.ptr(out), N, L.stream())
        name = "reidmi_gemm_f16"
    else:
        args = (epi, L.ptr(A), K, L.ptr(W), K, M, N, K, L.ptr(b), L.ptr(out), N, L.stream())
        name = "reidmi_gemm_bf16"
    L.call(name, *args)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        L.call(name, *args)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"M={M} N={N} K={K} epi={epi} v{var}: {ms * 1e3:.1f} us  {2.0 * M * N * K / ms / 1e9:.1f} TF/s")


if __name__ == "__main__":
    main()
