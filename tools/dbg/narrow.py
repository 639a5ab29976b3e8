import ctypes, io, os, sys
import numpy as np
from PIL import Image
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import reidmi_boot; reidmi_boot.load()
from multimodal_reid_amd import data_prepare
from test_jpeg import parity_cases, pil_rgb
cases = parity_cases()
jb = data_prepare.JpegBatch([b for _, b in cases])
vp = ctypes.c_void_p
print(open('/proc/cpuinfo').read().split('model name')[1].split('\n')[0], 'avx512f' in open('/proc/cpuinfo').read())
res = {}
for m in range(3):
    L = ctypes.CDLL(f"tools/dbg/libjpeghost{m}.so")
    out = np.zeros(jb.out_bytes, np.uint8); err = np.zeros(jb.B, np.int32)
    L.jpeg_host_decode(jb.buf.ctypes.data_as(vp), jb.plan.ctypes.data_as(vp), jb.info.ctypes.data_as(vp), out.ctypes.data_as(vp), err.ctypes.data_as(vp))
    res[m] = out
for i, (name, b) in enumerate(cases):
    off, h, w = jb.meta[i]; ref = pil_rgb(b)
    ok = [np.array_equal(res[m][off:off+h*w*3].reshape(h, w, 3), ref) for m in range(3)]
    if not all(ok): print(name, ok)
