"""Per-phase cycle stamps of the vision attention kernel (diagnostic build: -DATTN_STAMPS, see
tools/build_variant.py).  Runs mhsa at the bench shape (1024 images x 12 heads, L = 211), then
prints the median / p90 cycles of each phase (mhsa_pipe_kernel's stamps 0-5) of heads 8..15 of every workgroup, per wave.

    python tools/attn_stamps.py abvar/libreidmi_attn_stamps.so"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import _lib as L  # noqa: E402
from lib_ab import open_lib  # noqa: E402

PHASES = ["prefetch issue (waves 0-3)", "S = K Q^T + max", "softmax + P.V (+ next Q / V)",
          "O stores + vmcnt wait", "barrier"]


def main():
    lib = open_lib(sys.argv[1])
    fn = getattr(lib, "reidmi_attn_stamps")
    fn.argtypes = [ctypes.c_void_p]
    fn.restype = ctypes.c_int
    dev = torch.device("cuda")
    nseq, H, Lq = 1024, 12, 211
    lp = lib.reidmi_attn_lpad(Lq)
    g = torch.Generator(device=dev).manual_seed(Lq)
    q = (torch.randn(nseq * H, Lq, 64, device=dev, generator=g) * 2).half()
    k = (torch.randn(nseq * H, Lq, 64, device=dev, generator=g) * 2).half()
    vt = torch.randn(nseq * H, 64, lp, device=dev, generator=g).half()
    o = torch.empty(nseq * Lq, H * 64, dtype=torch.float16, device=dev)
    args = (L.ptr(q), L.ptr(k), L.ptr(vt), L.ptr(o), nseq, Lq, H, 0, L.stream())
    for _ in range(20):
        assert lib.reidmi_mhsa_f16(*args) == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    assert lib.reidmi_mhsa_f16(*args) == 0
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    st = np.zeros(256 * 8 * 8 * 8, dtype=np.uint64)
    assert fn(st.ctypes.data) == 0
    st = st.reshape(256, 8, 8, 8).astype(np.int64)  # [wg][wave][head][stamp]
    waves = (Lq + 31) // 32
    st = st[:, :waves]
    print(f"mhsa 1024x12 L=211 (stamped build): {ms * 1e3:.1f} us")
    nxt = np.roll(st[..., 0], -1, axis=2)  # next head's start (last head of the window dropped)
    d = np.diff(st[..., :6], axis=-1)
    loop = (nxt - st[..., 5])[:, :, :-1]
    tot = (nxt - st[..., 0])[:, :, :-1]
    print(f"{'phase':28s} " + " ".join(f"w{w:<7d}" for w in range(waves)) + "  (median cycles; p90 in [])")
    for i, name in enumerate(PHASES):
        x = d[..., i]
        print(f"{name:28s} " + " ".join(f"{int(np.median(x[:, w])):6d}  " for w in range(waves)) +
              f" [{int(np.percentile(x, 90))}]")
    print(f"{'loop overhead':28s} " + " ".join(f"{int(np.median(loop[:, w])):6d}  " for w in range(waves)))
    print(f"{'head total':28s} " + " ".join(f"{int(np.median(tot[:, w])):6d}  " for w in range(waves)) +
          f" [{int(np.percentile(tot, 90))}]")
    print(f"heads per CU {nseq * H / 256:.0f}; median head x heads = {np.median(tot) * nseq * H / 256:.0f} cycles")


if __name__ == "__main__":
    main()
