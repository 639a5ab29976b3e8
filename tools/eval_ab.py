"""In-process A/B of reidmi_eval_rows across library builds (tools/build_variant.py) on Market-
and MSMT17-size random distance matrices with synthetic labels, and Market-size distances of
identity-clustered features; interleaved rounds, outputs
checked bit-identical across the builds.

    python tools/eval_ab.py LIB.so[,LIB2.so,...] [ROUNDS]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import _lib as L, synthetic as syn  # noqa: E402
from lib_ab import open_lib  # noqa: E402


def clustered_distances(qp, gp, dev, dim=256, noise=2.2):
    """Euclidean distances of L2-normalised identity-clustered features (positives near the
    top of each row, as in the bench's Market step) instead of uniform random ones."""
    from multimodal_reid_amd import evaluate
    qf, gf = syn.features(qp, gp, dim=dim, seed=0, noise=noise)
    qn = evaluate.l2_normalize_device(torch.from_numpy(qf).to(dev))
    gn = evaluate.l2_normalize_device(torch.from_numpy(gf).to(dev))
    return evaluate.euclidean_distance_device(qn, gn)


def main():
    libs = [(os.path.basename(p), open_lib(p)) for p in sys.argv[1].split(",")]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda")
    cases = []
    for name in ("market1501", "msmt17", "market1501-clustered"):
        sp = syn.DATASET_SPLITS[name.split("-")[0]]
        Q, G = sp["num_query"], sp["num_gallery"]
        qp, gp, qc, gc = syn.labels(Q, G, sp["num_ids"], sp["num_cams"], seed=0, junk_frac=0.02)
        d = torch.rand(Q, G, device=dev) if "-" not in name else clustered_distances(qp, gp, dev)
        lab = [torch.from_numpy(a).to(dev) for a in (qp, gp, qc, gc)]
        cases.append((name, Q, G, d, lab))
    for r in range(rounds):
        for name, Q, G, d, lab in cases:
            ref = None
            for lname, lib in libs:
                valid = torch.empty(Q, device=dev, dtype=torch.int32)
                first = torch.empty(Q, device=dev, dtype=torch.int64)
                ap = torch.empty(Q, device=dev, dtype=torch.float64)
                nk = torch.empty(Q, device=dev, dtype=torch.int64)
                ovf = torch.zeros(1, device=dev, dtype=torch.int32)
                ws = torch.empty(lib.reidmi_eval_rows_workspace_bytes(G), device=dev, dtype=torch.uint8)
                args = (L.ptr(d), Q, G, G, *(L.ptr(t) for t in lab), L.ptr(valid), L.ptr(first), L.ptr(ap), L.ptr(nk),
                        L.ptr(ovf), L.ptr(ws), ws.numel(), L.stream())
                assert lib.reidmi_eval_rows(*args) == 0, lib.reidmi_last_error()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    lib.reidmi_eval_rows(*args)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / 20
                out = [t.cpu().numpy() for t in (valid, first, ap, nk, ovf)]
                same = "" if ref is None else (" bit-identical" if all(np.array_equal(a.view(np.uint8), b.view(np.uint8))
                                                                         for a, b in zip(ref, out)) else " DIFFERENT")
                ref = ref if ref is not None else out
                nb = 4.0 * Q * G + 16.0 * G
                print(f"r{r} eval_rows {name} {Q}x{G} {lname:24s}: {ms * 1e3:7.1f} us  {nb / ms / 1e6:7.1f} GB/s "
                      f"({nb / ms / 1e6 / 8000:.3f} of 8 TB/s){same}", flush=True)


if __name__ == "__main__":
    main()
