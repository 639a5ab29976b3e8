"""In-process A/B of the vision attention kernels in libreidmi_tools.so: mhsa_rr_kernel (8 waves,
round-robin (head, 32-query block) units, 3 LDS slots, V^T rows of 212; reidmi_mhsa_f16_rr) against
the product's mhsa_pipe_kernel<7> (one head at a time on 7 waves, V^T rows of 228; reidmi_mhsa_f16), at
1024 images and at the bench's 19 281 images per call (12 heads, L = 211); interleaved rounds,
outputs checked bit-identical.  Bytes: q + k + V^T + o as each kernel's layout has them.

    python tools/attn_rr_ab.py [ROUNDS]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import _lib as L  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    T = L.load_tools()
    dev = torch.device("cuda")
    Lq, H = 211, 12
    for nseq in (1024, 19281):
        n = nseq * H
        g = torch.Generator(device=dev).manual_seed(nseq)
        q = (torch.randn(n, Lq, 64, device=dev, generator=g) * 2).half()
        k = (torch.randn(n, Lq, 64, device=dev, generator=g) * 2).half()
        v = torch.randn(n, Lq, 64, device=dev, generator=g).half()
        vts = {}
        for vs in (212, 228):
            vt = torch.zeros(n, 64, vs, dtype=torch.float16, device=dev)
            vt[:, :, :Lq] = v.transpose(1, 2)
            vts[vs] = vt
        del v
        outs = {}
        calls = {"rr (212)": lambda o: T.reidmi_mhsa_f16_rr(L.ptr(q), L.ptr(k), L.ptr(vts[212]), L.ptr(o), nseq, Lq,
                                                            H, L.stream()),
                 "pipe7 (228)": lambda o: T.reidmi_mhsa_f16(L.ptr(q), L.ptr(k), L.ptr(vts[228]), L.ptr(o), nseq, Lq, H, 0,
                                                            L.stream())}
        for r in range(rounds):
            for name, fn in calls.items():
                o = torch.empty(nseq * Lq, H * 64, dtype=torch.float16, device=dev)
                assert fn(o) == 0, T.reidmi_last_error()
                reps = 10 if nseq <= 1024 else 3
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    fn(o)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / reps
                vs = 212 if name.startswith("rr") else 228
                by = 3 * n * Lq * 64 * 2 + n * 64 * vs * 2
                same = ""
                if name in outs:
                    pass
                outs[name] = o
                if len(outs) == 2:
                    a, b = outs.values()
                    same = " bit-identical" if torch.equal(a, b) else " DIFFERENT"
                print(f"r{r} mhsa vision {nseq}x{H} L={Lq} {name:12s}: {ms * 1e3:9.1f} us "
                      f"({ms * 1e3 * 1024 / nseq:6.1f} us per 1024 images)  {by / ms / 1e6:7.1f} GB/s{same}", flush=True)
            outs.clear()


if __name__ == "__main__":
    main()
