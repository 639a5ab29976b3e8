import sys, os, torch, time
sys.path.insert(0, os.getcwd())
import reidmi_boot; reidmi_boot.load()
from multimodal_reid_amd import _lib as L, evaluate
dev = torch.device("cuda")
for (Q, G, D) in [(3368, 15913, 1280), (531, 1010000, 1792), (11659, 82161, 1280)]:
    q = torch.randn(Q, D, device=dev); g = torch.randn(G, D, device=dev)
    out = torch.empty(Q, G, device=dev)
    res = {}
    ws = torch.empty(Q + G, device=dev)
    for v in (1, 0, 1, 0):
        run = lambda: L.call_tools("reidmi_distmat_f32_variant", L.ptr(q), Q, D, L.ptr(g), G, D, D, L.ptr(out), G,
                             L.ptr(ws), v, L.stream())
        run(); torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(3): run()
        torch.cuda.synchronize(); ms = (time.perf_counter() - t) / 3 * 1e3
        res.setdefault(v, []).append(2.0 * Q * G * D / ms / 1e9)
    print(Q, G, D, {v: round(max(x), 1) for v, x in res.items()}, "TF/s", flush=True)
    del q, g, out; torch.cuda.empty_cache()
