"""HBM rate of eval_rows' access pattern alone (one workgroup per distance row, float4 loads,
a per-row sum): tells whether the Market eval is bound by how its rows are read or by its own
work.  Builds tools/rowread_bw.hip into tools/ablibs/librowread.so (on the CPU side, before
the GPU call) and times each variant at the Market and MSMT17 shapes with HIP events.

    python tools/rowread_bw.py build      # here
    python tools/rowread_bw.py            # on the GPU box"""
import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "ablibs", "librowread.so")
VARIANTS = ("256 thr x 4 float4", "256 thr x 8 float4", "256 thr x 16 float4", "512 thr x 4 float4",
            "1024 thr x 4 float4")


def build():
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", LIB,
                    os.path.join(HERE, "rowread_bw.hip")], check=True)
    print("built", LIB)


def main():
    import torch
    lib = ctypes.CDLL(LIB)
    lib.rowread.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int,
                            ctypes.c_void_p]
    dev = torch.device("cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for name, Q, G in (("market1501", 3368, 15912), ("msmt17", 11659, 82160)):
        d = torch.rand(Q, G, device=dev)
        out = torch.zeros(Q, device=dev)
        for v, vname in enumerate(VARIANTS):
            assert lib.rowread(ctypes.c_void_p(d.data_ptr()), Q, G, ctypes.c_void_p(out.data_ptr()), v, st) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                lib.rowread(ctypes.c_void_p(d.data_ptr()), Q, G, ctypes.c_void_p(out.data_ptr()), v, st)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 20
            nb = 4.0 * Q * G
            print(f"{name} {Q}x{G} {vname:22s}: {ms * 1e3:7.1f} us  {nb / ms / 1e6:7.1f} GB/s "
                  f"({nb / ms / 1e6 / 8000:.3f} of 8 TB/s)", flush=True)


if __name__ == "__main__":
    build() if sys.argv[1:] == ["build"] else main()
