"""In-process A/B of the R2 pre-filter (reidmi_rr_rank_rows_f16_ex) across library builds
(tools/build_variant.py): identity-clustered features as tools/scale_vitl_1m.py (N items,
dimension D), rows [0, R) ranked against all N, dense (stride 0) and sampled (stride 16)
forms, rounds interleaved; outputs must agree bit for bit across builds and forms.

    python tools/rr_rank_ab.py LIB.so[,LIB2.so,...] [--N 1010000] [--D 768] [--R 32768] [--rounds 2]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import _lib as L, synthetic as syn  # noqa: E402
from lib_ab import open_lib  # noqa: E402
from scale_vitl_1m import clustered_features  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs")
    ap.add_argument("--N", type=int, default=1010000)
    ap.add_argument("--D", type=int, default=768)
    ap.add_argument("--R", type=int, default=32768)
    ap.add_argument("--K", type=int, default=51)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--strides", default="0,16")
    a = ap.parse_args()
    dev = torch.device("cuda")
    N, D, R, K = a.N, a.D, a.R, a.K
    ids = max(N // 100, 10)
    qp, gp, _, _ = syn.labels(10000, N - 10000, ids, 8, seed=0, distractor_frac=0.1, junk_frac=0.0)
    f = clustered_features(np.concatenate([qp, gp]), ids, D, dev, seed=11).contiguous()
    Np, Dp = (N + 255) // 256 * 256, (D + 63) // 64 * 64
    sqn = torch.empty(N, device=dev)
    L.call("reidmi_row_sqnorm_f32", L.ptr(f), N, D, D, L.ptr(sqn), L.stream())
    nrm = torch.sqrt(sqn)
    x16 = torch.zeros((Np, Dp), dtype=torch.float16, device=dev)
    ok = torch.ones(1, dtype=torch.int32, device=dev)
    L.call("reidmi_rr_feat16", L.ptr(f), N, D, D, L.ptr(x16), Np, Dp, L.ptr(ok), L.stream())
    nmax2 = torch.empty(2, device=dev)
    L.call("reidmi_rr_norm_max", L.ptr(sqn), L.ptr(nrm), N, L.ptr(nmax2), L.stream())
    cc = 4096  # chunk rows of the dense form (reranking.HipStages at 16 GiB)
    chunk = torch.empty(cc * Np, device=dev)
    libs = [(os.path.basename(p), open_lib(p)) for p in a.libs.split(",")]
    strides = [int(x) for x in a.strides.split(",")]
    ref = None
    times = {}
    for rnd in range(a.rounds):
        for name, lib in libs:
            for S in strides:
                Rk = torch.full((R, K), -1, dtype=torch.int32, device=dev)
                rmax = torch.zeros(R, device=dev)
                need = torch.zeros(R, dtype=torch.int32, device=dev)
                pr = int(lib.reidmi_rr_rank_rows_f16_pass_rows(N, Np, cc, K, S))
                torch.cuda.synchronize()
                t = time.perf_counter()
                for lo in range(0, R, pr):
                    hi = min(R, lo + pr)
                    rc = lib.reidmi_rr_rank_rows_f16_ex(
                        L.ptr(f), N, D, D, L.ptr(sqn), L.ptr(nrm), L.ptr(nmax2), L.ptr(x16), Np, Dp, lo, hi, K,
                        L.ptr(Rk[lo:]), L.ptr(rmax[lo:]), L.ptr(need[lo:]), L.ptr(chunk), cc, S, L.stream())
                    assert rc == 0, lib.reidmi_last_error()
                torch.cuda.synchronize()
                dt = time.perf_counter() - t
                out = (Rk.cpu().numpy(), rmax.cpu().numpy().view(np.uint32), need.cpu().numpy())
                if ref is None:
                    ref = out
                good = out[2] == 0
                same = bool(np.array_equal(out[0][good & (ref[2] == 0)], ref[0][good & (ref[2] == 0)]))
                times.setdefault((name, S), []).append(dt)
                print(f"round {rnd} {name:40s} stride {S:2d}: {dt * 1e3:8.1f} ms for {R} rows "
                      f"({dt / R * N * 1e-3 * 1e3:6.0f} ms per {N} rows)  need {int(out[2].sum())}  same {same}",
                      flush=True)
    for (name, S), v in times.items():
        print(f"{name:40s} stride {S:2d}: best {min(v) * 1e3:8.1f} ms -> {min(v) / R * N:6.2f} s per N rows")


if __name__ == "__main__":
    main()
