"""A/B of the fused QKV GEMM + attention kernel against the two-kernel path (QKV GEMM with the
head-split epilogue, then the attention kernel) at the bench's shape: one vision block at
batch B (M = B * 211 token rows, ViT-B/16 width 768).  Random operands, HIP events.
usage: python tools/qkv_attn_ab.py [B] [L] [W] [reps] [variant.so ...]
Each variant library (a build of the same sources with timing macros, e.g. QA_NO_ATTN) is
timed on the fused path too."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import _lib as lib  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 211
    W = int(sys.argv[3]) if len(sys.argv) > 3 else 768
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    H = W // 64
    dev = torch.device("cuda")
    M = B * L
    x = (torch.rand(M, W, device=dev) * 2 - 1).half()
    wq = ((torch.rand(3 * W, W, device=dev) * 2 - 1) / W ** 0.5).half()
    bias = torch.rand(3 * W, device=dev) * 0.1
    cs = torch.rand(3 * W, device=dev)
    rs = torch.stack([torch.rand(M + 256, device=dev) + 0.5, torch.rand(M + 256, device=dev) - 0.5], 1).contiguous()
    lp = lib.load().reidmi_attn_lpad(L)
    q = torch.empty(B * H * L * 64, dtype=torch.float16, device=dev)
    k = torch.empty_like(q)
    vt = torch.zeros(B * H * 64 * lp, dtype=torch.float16, device=dev)
    o = torch.empty(M, W, dtype=torch.float16, device=dev)
    flop = 2.0 * M * 3 * W * W + 4.0 * B * H * L * L * 64
    hbm_unfused = 2.0 * (M * W + 3 * M * W + 3 * M * W + M * W)  # x, q/k/v written + read, o
    variants = [(os.path.basename(p), ctypes.CDLL(os.path.abspath(p))) for p in sys.argv[5:]]
    for _, V in variants:
        V.reidmi_qkv_attention_f16.argtypes = lib.TOOLS_SIGNATURES["reidmi_qkv_attention_f16"]
    for rnd in range(3):
        for fused, name, V in [(0, "", None), (1, "", None)] + [(1, n, V) for n, V in variants]:
            def run():
                if V is not None:
                    assert V.reidmi_qkv_attention_f16(lib.ptr(x), W, lib.ptr(wq), W, lib.ptr(bias), lib.ptr(cs),
                                                      lib.ptr(rs), B, L, H, W, None, None, None, lib.ptr(o), 1,
                                                      lib.stream()) == 0
                    return
                lib.call_tools("reidmi_qkv_attention_f16", lib.ptr(x), W, lib.ptr(wq), W, lib.ptr(bias), lib.ptr(cs), lib.ptr(rs),
                         B, L, H, W, lib.ptr(q), lib.ptr(k), lib.ptr(vt), lib.ptr(o), fused, lib.stream())
            for _ in range(3):
                run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            print(f"r{rnd} B={B} L={L} W={W} fused={fused}{' ' + name if name else ''}: {ms * 1e3:8.1f} us  {flop / ms / 1e9:7.1f} TF/s"
                  + (f"  (two-kernel HBM bytes {hbm_unfused / 1e9:.2f} GB)" if not fused else ""), flush=True)


if __name__ == "__main__":
    main()
