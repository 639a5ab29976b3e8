"""In-process A/B of the exact-fp32 distance kernel across library builds
(tools/build_variant.py): Market, MSMT17 and a re-rank-chunk shape, interleaved rounds, outputs
checked bit-identical across builds.

    python tools/distmat_lib_ab.py LIB.so[,LIB2.so,...] [ROUNDS]"""
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
    shapes = [("market", 3368, 15913, 1280), ("msmt17", 11659, 82161, 1280), ("rr-chunk", 5592, 93820, 1280),
              ("1m-gallery", 4096, 1000000, 768)]
    data = []
    for name, Q, G, D in shapes:
        g = torch.Generator(device=dev).manual_seed(Q)
        data.append((name, Q, G, D, torch.randn(Q, D, device=dev, generator=g), torch.randn(G, D, device=dev, generator=g)))
    for r in range(rounds):
        for name, Q, G, D, q, g in data:
            ref = None
            for lname, lib in libs:
                out = torch.empty(Q, G, device=dev)
                ws = torch.empty(Q + G, device=dev)
                args = (L.ptr(q), Q, D, L.ptr(g), G, D, D, L.ptr(out), G, L.ptr(ws), L.stream())
                assert lib.reidmi_distmat_f32(*args) == 0, lib.reidmi_last_error()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    lib.reidmi_distmat_f32(*args)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / 5
                same = "" if ref is None else (" bit-identical" if torch.equal(ref.view(torch.int32), out.view(torch.int32))
                                               else " DIFFERENT")
                ref = out if ref is None else ref
                print(f"r{r} distmat {name:8s} {Q}x{G}x{D} {lname:22s}: {ms:8.3f} ms {2.0 * Q * G * D / ms / 1e9:6.1f} TF/s"
                      f"{same}", flush=True)
            del ref, out
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
