"""Vision attention (mhsa_pipe_kernel) time per (image, head) across sequence lengths, to tell
whether its time follows the busiest SIMD's work (ceil(waves / 4) waves x key blocks: 7 waves on
4 SIMDs leave one SIMD half idle) or the workgroup's total work (waves x key blocks).
Interleaved rounds, NSEQ images x 12 heads:  python tools/attn_scan.py [ROUNDS]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import _lib as L  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    nseq, H = int(os.environ.get("NSEQ", "1024")), 12
    lib = L.load()
    dev = torch.device("cuda")
    cases = {}
    for Lq in (96, 128, 160, 192, 211, 224, 256):
        lp = lib.reidmi_attn_lpad(Lq)
        q = (torch.randn(nseq * H, Lq, 64, device=dev) * 2).half()
        k = (torch.randn(nseq * H, Lq, 64, device=dev) * 2).half()
        vt = torch.randn(nseq * H, 64, lp, device=dev).half()
        o = torch.empty(nseq * Lq, H * 64, dtype=torch.float16, device=dev)
        cases[Lq] = (q, k, vt, o)
    for r in range(rounds):
        for Lq, (q, k, vt, o) in cases.items():
            args = (L.ptr(q), L.ptr(k), L.ptr(vt), L.ptr(o), nseq, Lq, H, 0, L.stream())
            for _ in range(3):
                L.call("reidmi_mhsa_f16", *args)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                L.call("reidmi_mhsa_f16", *args)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 10 * 1e3
            nkb = (Lq + 31) // 32
            simd = (nkb + 3) // 4 * nkb
            print(f"r{r} L={Lq} NKB={nkb}: {us:.1f} us  {us / (nseq * H) * 256 * 1e3:.0f} ns per head per CU"
                  f"  busiest-SIMD units {simd}  total units {nkb * nkb}", flush=True)


if __name__ == "__main__":
    main()
