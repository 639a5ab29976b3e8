"""Device JPEG decode on its own (for rocprofv3 --kernel-trace --stats): N Market-shaped
(128 x 64, 4:2:0, quality 90) Pillow-encoded files resident in HBM, decoded REPS times, then
decode + Resize/ToTensor/Normalize to fp16 [N, 3, 256, 128].

    python tools/jpeg_one.py [N (default 19281)] [REPS (default 5)]"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import _lib, data_prepare  # noqa: E402
from multimodal_reid_amd import synthetic as syn  # noqa: E402


def market_files(n, unique=2048, seed=0):
    u = syn.jpeg_files(min(n, unique), 128, 64, seed=seed, quality=90)
    return [u[i % len(u)] for i in range(n)]


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    n = int(args[0]) if args else 19281
    reps = int(args[1]) if len(args) > 1 else 5
    files = market_files(n)
    t = time.perf_counter()
    jb = data_prepare.JpegBatch(files)
    t_plan = time.perf_counter() - t
    dev = torch.device("cuda")
    dfiles = data_prepare._to_device(jb.buf, dev)
    dplan = data_prepare._to_device(jb.plan, dev)
    ws = torch.empty(jb.ws_bytes, dtype=torch.uint8, device=dev)
    pix = torch.empty(jb.out_bytes, dtype=torch.uint8, device=dev)
    err = torch.empty(n, dtype=torch.int32, device=dev)
    info = jb.info.copy()
    s = _lib.stream(dev)

    def decode():
        _lib.call("reidmi_jpeg_decode", _lib.ptr(dfiles), _lib.ptr(dplan), info.ctypes.data_as(ctypes.c_void_p), n,
                  _lib.ptr(ws), ws.numel(), _lib.ptr(pix), _lib.ptr(err), s)

    decode()
    torch.cuda.synchronize()
    assert not err.any().item()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        decode()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    fb, ob = int(jb.buf.size), int(jb.out_bytes)
    print(f"jpeg decode {n} files ({fb / n:.0f} B/file): {ms:.3f} ms  {n / ms * 1e3:.0f} img/s  "
          f"{(fb + ob) / ms / 1e6:.1f} GB/s (file + RGB bytes); host plan {t_plan * 1e3:.1f} ms "
          f"({n / t_plan:.0f} files/s)")
    out = torch.empty((n, 3, 256, 128), dtype=torch.float16, device=dev)
    data_prepare.preprocess_jpeg(files[:64], out=out[:64])
    torch.cuda.synchronize()
    meta = torch.from_numpy(jb.meta).to(dev)
    mean = (ctypes.c_float * 3)(0.5, 0.5, 0.5)
    e0.record()
    for _ in range(reps):
        decode()
        _lib.call("reidmi_preprocess_u8", _lib.ptr(pix), _lib.ptr(meta), n, jb.max_h, jb.max_w, 256, 128, mean, mean,
                  1, _lib.ptr(out), s)
    e1.record()
    torch.cuda.synchronize()
    ms2 = e0.elapsed_time(e1) / reps
    print(f"decode + preprocess to fp16 [N,3,256,128]: {ms2:.3f} ms  {n / ms2 * 1e3:.0f} img/s")
    import io
    from PIL import Image
    k = min(n, 1000)
    t = time.perf_counter()
    for f in files[:k]:
        np.asarray(Image.open(io.BytesIO(f)).convert("RGB"))
    dt = time.perf_counter() - t
    print(f"Pillow decode, 1 thread: {k / dt:.0f} img/s")


if __name__ == "__main__":
    main()
