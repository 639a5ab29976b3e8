"""First-use costs in a fresh process (profiles/r05/rr_first_call.txt): device allocations of the
re-rank scratch sizes, the first launch of a rerank.hip kernel, and the staged re-rank before and
after its kernels have run once (small, then MSMT17 size).  python tools/rr_first_call.py"""
import time, torch, sys, os
sys.path.insert(0, os.getcwd())
import reidmi_boot; reidmi_boot.load()
from multimodal_reid_amd import _lib
dev = torch.device("cuda"); torch.cuda.set_device(0)
x = torch.ones(10, device=dev); torch.cuda.synchronize()
def t(name, fn):
    torch.cuda.synchronize(); a = time.perf_counter(); r = fn(); torch.cuda.synchronize()
    print(f"{name}: {1e3*(time.perf_counter()-a):.2f} ms", flush=True); return r
for gib in (16, 3, 16):
    b = t(f"empty {gib} GiB", lambda: torch.empty(gib << 28, device=dev, dtype=torch.float32))
    t(f"  touch first+last", lambda: (b[:1].zero_(), b[-1:].zero_()))
    del b; torch.cuda.empty_cache()
f = torch.randn(93820, 1280, device=dev)
s = torch.empty(93820, device=dev)
t("first rerank.hip launch (row_sqnorm)", lambda: _lib.call("reidmi_row_sqnorm_f32", _lib.ptr(f), 93820, 1280, 1280, _lib.ptr(s), _lib.stream()))
t("second launch", lambda: _lib.call("reidmi_row_sqnorm_f32", _lib.ptr(f), 93820, 1280, 1280, _lib.ptr(s), _lib.stream()))
from multimodal_reid_amd import reranking, evaluate
q = evaluate.l2_normalize_device(torch.randn(500, 1280, device=dev))
g = evaluate.l2_normalize_device(torch.randn(3500, 1280, device=dev))
t("small staged re-rank #1 (first use of the R1-R7 kernels)", lambda: reranking.re_ranking_sharded(q, g, 50, 15, 0.3))
t("small staged re-rank #2", lambda: reranking.re_ranking_sharded(q, g, 50, 15, 0.3))
q = evaluate.l2_normalize_device(torch.randn(11659, 1280, device=dev))
g = evaluate.l2_normalize_device(torch.randn(82161, 1280, device=dev))
t("MSMT17-size re-rank #1", lambda: reranking.re_ranking_sharded(q, g, 50, 15, 0.3))
t("MSMT17-size re-rank #2", lambda: reranking.re_ranking_sharded(q, g, 50, 15, 0.3))
