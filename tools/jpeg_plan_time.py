"""Host side of the JPEG leg, by part (GPU box host): read_files (joining the file bytes),
reidmi_jpeg_plan (marker parse, threaded), on a Market split of synthetic files.
    python tools/jpeg_plan_time.py"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import _lib, data_prepare, synthetic as syn  # noqa: E402

u = syn.jpeg_files(2048, 128, 64, seed=0, quality=90)
for B in (2047, 19281):
    files = [u[i % len(u)] for i in range(B)]
    for r in range(3):
        t0 = time.perf_counter()
        buf, off = data_prepare.read_files(files)
        t1 = time.perf_counter()
        meta = np.zeros((B, 3), np.int64)
        st = np.zeros(B, np.int32)
        info = np.zeros(10, np.int64)
        plan = np.zeros(4096 + B * 256 + 64 * 1536, np.uint8)
        t2 = time.perf_counter()
        _lib.call("reidmi_jpeg_plan", buf.ctypes.data_as(ctypes.c_void_p), off.ctypes.data_as(ctypes.c_void_p), B,
                  plan.ctypes.data_as(ctypes.c_void_p), plan.size, meta.ctypes.data_as(ctypes.c_void_p),
                  st.ctypes.data_as(ctypes.c_void_p), info.ctypes.data_as(ctypes.c_void_p))
        t3 = time.perf_counter()
        print(f"B={B} rep {r}: read_files {1e3 * (t1 - t0):.2f} ms, plan {1e3 * (t3 - t2):.2f} ms, "
              f"cpus {os.cpu_count()}", flush=True)
