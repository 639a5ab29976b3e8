"""Run the encoder's attention kernel on the bench shape (NSEQ (default 1024) images x 12 heads, L = 211)
REPS times, for rocprofv3 --pmc / --kernel-trace passes:  python tools/attn_one.py [REPS]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import _lib as L  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    nseq, H, Lq = int(os.environ.get("NSEQ", "1024")), 12, 211
    lib = L.load()
    lp = lib.reidmi_attn_lpad(Lq)
    dev = torch.device("cuda")
    q = (torch.randn(nseq * H, Lq, 64, device=dev) * 2).half()
    k = (torch.randn(nseq * H, Lq, 64, device=dev) * 2).half()
    vt = torch.randn(nseq * H, 64, lp, device=dev).half()
    o = torch.empty(nseq * Lq, H * 64, dtype=torch.float16, device=dev)
    args = (L.ptr(q), L.ptr(k), L.ptr(vt), L.ptr(o), nseq, Lq, H, 0, L.stream())
    L.call("reidmi_mhsa_f16", *args)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        L.call("reidmi_mhsa_f16", *args)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    fl = 4.0 * nseq * H * Lq * Lq * 64
    by = (3 * nseq * H * Lq * 64 + nseq * Lq * H * 64) * 2
    print(f"mhsa {nseq}x{H} L={Lq}: {ms * 1e3:.1f} us  {fl / ms / 1e9:.1f} TF/s  {by / ms / 1e6:.1f} GB/s (q,k,v,o once)")


if __name__ == "__main__":
    main()
