import sys, os
sys.path.insert(0, os.getcwd())
import torch
import reidmi_boot
reidmi_boot.load()
from multimodal_reid_amd import _lib as L
M, N, K = 16, 128, 64
A = torch.zeros(M, K, dtype=torch.bfloat16, device="cuda")
W = torch.zeros(N, K, dtype=torch.bfloat16, device="cuda")
b = torch.arange(N, dtype=torch.float32, device="cuda")
for epi in (6, 2):
    out = (torch.zeros(M, N, device="cuda", dtype=torch.float16 if epi == 6 else torch.float32)
           + torch.arange(M, device="cuda")[:, None] * 1000)
    L.call("reidmi_gemm_bf16", epi, L.ptr(A), K, L.ptr(W), K, M, N, K, L.ptr(b), L.ptr(out), N, L.stream())
    torch.cuda.synchronize()
    print(epi, out[0, :40].float().tolist())
    print(epi, out[1, :40].float().tolist())
