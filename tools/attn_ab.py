"""In-process A/B of the attention kernel across library builds (tools/build_variant.py):
vision (1024 images x 12 heads, L = 211) and text (42000 x 8 heads, L = 50 causal) shapes,
interleaved rounds, outputs checked bit-identical across the builds.

    python tools/attn_ab.py LIB.so[,LIB2.so,...] [ROUNDS]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import _lib as L  # noqa: E402
from lib_ab import open_lib  # noqa: E402


def main():
    libs = [(os.path.basename(p), open_lib(p)) for p in sys.argv[1].split(",")]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda")
    cases = []
    for name, nseq, H, Lq, causal in (("vision", 1024, 12, 211, 0), ("text", 42000, 8, 50, 1)):
        lp = libs[0][1].reidmi_attn_lpad(Lq)
        g = torch.Generator(device=dev).manual_seed(Lq)
        q = (torch.randn(nseq * H, Lq, 64, device=dev, generator=g) * 2).half()
        k = (torch.randn(nseq * H, Lq, 64, device=dev, generator=g) * 2).half()
        vt = torch.randn(nseq * H, 64, lp, device=dev, generator=g).half()
        cases.append((name, nseq, H, Lq, causal, q, k, vt))
    for r in range(rounds):
        for name, nseq, H, Lq, causal, q, k, vt in cases:
            ref = None
            for lname, lib in libs:
                o = torch.empty(nseq * Lq, H * 64, dtype=torch.float16, device=dev)
                args = (L.ptr(q), L.ptr(k), L.ptr(vt), L.ptr(o), nseq, Lq, H, causal, L.stream())
                assert lib.reidmi_mhsa_f16(*args) == 0, lib.reidmi_last_error()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    lib.reidmi_mhsa_f16(*args)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / 10
                same = "" if ref is None else (" bit-identical" if torch.equal(ref, o) else " DIFFERENT")
                ref = o if ref is None else ref
                fl = 4.0 * nseq * H * Lq * Lq * 64
                by = 4 * nseq * H * Lq * 64 * 2
                print(f"r{r} mhsa {name} {nseq}x{H} L={Lq} {lname:22s}: {ms * 1e3:8.1f} us {fl / ms / 1e9:6.1f} TF/s "
                      f"{by / ms / 1e6:7.1f} GB/s{same}", flush=True)


if __name__ == "__main__":
    main()
