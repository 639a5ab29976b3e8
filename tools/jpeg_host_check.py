"""Host-side check of csrc/jpeg_core.h against Pillow (no GPU): plan with libreidmi's
reidmi_jpeg_plan, decode serially with tools/build/libjpeghost.so (the kernels' per-image
code compiled for the host), compare with Image.open(...).convert("RGB").

    python tools/jpeg_host_check.py"""
import ctypes
import io
import os
import sys

import numpy as np
from PIL import Image

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import synthetic as syn  # noqa: E402
from multimodal_reid_amd.data_prepare import JpegBatch  # noqa: E402

HOST = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "build", "libjpeghost.so"))


def cases():
    out = []
    for (h, w) in [(128, 64), (1, 1), (2, 2), (3, 5), (17, 33), (15, 2), (2, 15), (64, 128), (200, 97), (31, 1)]:
        for ss in (0, 1, 2):
            for q in (50, 95):
                out.append((f"{h}x{w} ss{ss} q{q}", syn.jpeg_files(1, h, w, seed=h * 1000 + w, quality=q,
                                                                   subsampling=ss, offset=ss)[0]))
    out.append(("rst", syn.jpeg_files(1, 128, 64, seed=3, restart_marker_blocks=3)[0]))
    out.append(("rst rows", syn.jpeg_files(1, 77, 45, seed=4, restart_marker_rows=1)[0]))
    out.append(("optimize", syn.jpeg_files(1, 128, 64, seed=5, optimize=True)[0]))
    out.append(("q100", syn.jpeg_files(1, 128, 64, seed=6, quality=100, subsampling=0)[0]))
    g = io.BytesIO()
    Image.fromarray(syn.crop_rgb(37, 29, 7)[:, :, 0]).save(g, "JPEG", quality=85)
    out.append(("gray", g.getvalue()))
    p = io.BytesIO()
    Image.fromarray(syn.crop_rgb(64, 32, 8)).save(p, "JPEG", progressive=True)
    out.append(("progressive", p.getvalue()))
    return out


def main():
    cs = cases()
    jb = JpegBatch([b for _, b in cs])
    out = np.zeros(max(jb.out_bytes, 1), np.uint8)
    err = np.zeros(jb.B, np.int32)
    HOST.jpeg_host_decode(jb.buf.ctypes.data_as(ctypes.c_void_p), jb.plan.ctypes.data_as(ctypes.c_void_p),
                          jb.info.ctypes.data_as(ctypes.c_void_p), out.ctypes.data_as(ctypes.c_void_p),
                          err.ctypes.data_as(ctypes.c_void_p))
    bad = 0
    for i, (name, b) in enumerate(cs):
        ref = np.asarray(Image.open(io.BytesIO(b)).convert("RGB"))
        if jb.status[i]:
            print(f"{name:24s} status {jb.status[i]}")
            continue
        off, h, w = jb.meta[i]
        got = out[off:off + h * w * 3].reshape(h, w, 3)
        d = np.abs(got.astype(int) - ref.astype(int))
        ok = d.max() == 0 and err[i] == 0
        bad += not ok
        print(f"{name:24s} err {err[i]} maxdiff {d.max():3d} ndiff {(d > 0).sum()}" + ("" if ok else "   <-- MISMATCH"))
    print("mismatches:", bad)


if __name__ == "__main__":
    main()
