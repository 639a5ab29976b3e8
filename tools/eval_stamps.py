"""Per-phase cycle stamps of eval_rows_wg_kernel (diagnostic build: tools/build_variant.py
stamps backend.hip -DEV_STAMPS=1), Market-size random distances (or, with a third argument
"clustered", distances of identity-clustered features).  Phases: P1 label pass,
P2 gather + sort + bucket table, P3 distance pass, P4 ranks + AP; start time spread."""
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

lib = open_lib(sys.argv[1])
name = sys.argv[2] if len(sys.argv) > 2 else "market1501"
dev = torch.device("cuda")
sp = syn.DATASET_SPLITS[name]
Q, G = sp["num_query"], sp["num_gallery"]
qp, gp, qc, gc = syn.labels(Q, G, sp["num_ids"], sp["num_cams"], seed=0, junk_frac=0.02)
if len(sys.argv) > 3 and sys.argv[3] == "clustered":
    from eval_ab import clustered_distances  # noqa: E402
    d = clustered_distances(qp, gp, dev)
else:
    d = torch.rand(Q, G, device=dev)
lab = [torch.from_numpy(a).to(dev) for a in (qp, gp, qc, gc)]
valid = torch.empty(Q, device=dev, dtype=torch.int32)
first = torch.empty(Q, device=dev, dtype=torch.int64)
ap = torch.empty(Q, device=dev, dtype=torch.float64)
nk = torch.empty(Q, device=dev, dtype=torch.int64)
ovf = torch.zeros(1, device=dev, dtype=torch.int32)
ws = torch.empty(lib.reidmi_eval_rows_workspace_bytes(G), device=dev, dtype=torch.uint8)
args = (L.ptr(d), Q, G, G, *(L.ptr(t) for t in lab), L.ptr(valid), L.ptr(first), L.ptr(ap), L.ptr(nk),
        L.ptr(ovf), L.ptr(ws), ws.numel(), L.stream())
for _ in range(5):
    lib.reidmi_eval_rows(*args)
torch.cuda.synchronize()
v = valid.cpu().numpy() == 1
f, k, a = first.cpu().numpy()[v].view(np.uint64), nk.cpu().numpy()[v].view(np.uint64), ap.cpu().numpy()[v]
ph = np.stack([f & 0xFFFFFFFF, f >> 32, k & 0xFFFFFFFF, k >> 32], 1).astype(np.float64)
print(f"{name}: {v.sum()} queries; cycles per phase (median / p90): ")
for i, n in enumerate(["P1 labels", "P2 sort+table", "P3 distances", "P4 ranks+AP"]):
    print(f"  {n:14s} {np.median(ph[:, i]):9.0f} {np.percentile(ph[:, i], 90):9.0f}")
tot = ph.sum(1)
print(f"  total          {np.median(tot):9.0f} {np.percentile(tot, 90):9.0f}  (~{np.median(tot) / 2.1e3:.1f} us at 2.1 GHz)")
st = (a - a.min()) / 100.0  # s_memrealtime: 100 MHz -> us
print(f"  start spread (us): p50 {np.median(st):.1f}  p90 {np.percentile(st, 90):.1f}  max {st.max():.1f}")
