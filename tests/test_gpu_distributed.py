"""The RCCL ("nccl" backend) code path on one GPU: a world-size-1 process group runs the
same all_gather_into_tensor / all_gather calls the multi-GPU eval makes (distributed.gather_rows
/ gather_var run their collective whenever a process group exists), through sharded_eval
with the libreidmi kernels as rows_fn and through the sharded k-reciprocal re-rank.  Results
must equal the single-process device path bit for bit.  (More ranks than GPUs is not an RCCL
configuration; N > 1 is covered by the gloo tests and the driver's multi-GPU bench.)"""
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402  (the spawned worker re-imports this module without conftest)

reidmi_boot.load()

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from multimodal_reid_amd import synthetic as syn

pytestmark = pytest.mark.gpu

Q, G = 300, 1700


def _data():
    qp, gp, qc, gc = syn.labels(Q, G, num_ids=120, num_cams=6, seed=31, junk_frac=0.03)
    qf, gf = syn.features(qp, gp, dim=256, seed=31)
    return qf, gf, qp, gp, qc, gc


def _rows_fn(q, g, qp, gp, qc, gc):
    from multimodal_reid_amd import evaluate
    d = evaluate.euclidean_distance_device(q, g)
    v, f, a, n, _ = evaluate.eval_rows_device(d, qp, gp, qc, gc)
    return v, f, a, n


def _single():
    from multimodal_reid_amd import evaluate, reranking
    qf, gf, qp, gp, qc, gc = _data()
    qn = evaluate.l2_normalize_device(torch.from_numpy(qf))
    gn = evaluate.l2_normalize_device(torch.from_numpy(gf))
    cmc, mAP = evaluate.eval_func_device(evaluate.euclidean_distance_device(qn, gn), qp, gp, qc, gc, 50)
    rr = reranking.re_ranking_device(qn, gn, 20, 6, 0.3)
    return cmc, mAP, rr.cpu().numpy()


def _worker(rank, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        from multimodal_reid_amd import distributed as rd, evaluate, reranking
        assert dist.get_backend() == "nccl"
        qf, gf, qp, gp, qc, gc = _data()
        qn = evaluate.l2_normalize_device(torch.from_numpy(qf))
        gn = evaluate.l2_normalize_device(torch.from_numpy(gf))
        cmc, mAP = rd.sharded_eval(qn, gn, qp, gp, qc, gc, Q, G, _rows_fn, 50)
        g_all = rd.gather_rows(gn, G)
        blob = torch.arange(1000, device=dev, dtype=torch.int16)
        rr = reranking.re_ranking_sharded(qn, gn, 20, 6, 0.3)
        torch.cuda.synchronize()
        out["res"] = (cmc, mAP, bool(torch.equal(g_all, gn)), bool(torch.equal(rd.gather_var(blob), blob)),
                      rr.cpu().numpy())
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_world1_matches_single_process(gpu):
    cmc_ref, map_ref, rr_ref = _single()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(_free_port(), out), nprocs=1, join=True)
    cmc, mAP, gathered_ok, var_ok, rr = out["res"]
    assert gathered_ok and var_ok
    assert np.array_equal(cmc, cmc_ref) and mAP == map_ref
    assert np.array_equal(rr.view(np.uint32), rr_ref.view(np.uint32))


def test_comm_capi_world1(gpu):
    """The C ABI's RCCL exchange (reidmi_comm_*, for callers that are not Python) at world 1:
    the padded in-place all-gather + in-order compaction returns the rows, and the all-reduce
    the input.  (Several ranks need several GPUs: RCCL refuses two ranks on one device.)"""
    import ctypes
    from multimodal_reid_amd import _lib
    L = _lib.load()
    uid = ctypes.create_string_buffer(128)
    _lib.call("reidmi_comm_unique_id", uid)
    comm = ctypes.c_void_p()
    _lib.call("reidmi_comm_init", ctypes.byref(comm), 1, 0, uid, 0)
    try:
        r, w = ctypes.c_int(), ctypes.c_int()
        _lib.call("reidmi_comm_rank", comm, ctypes.byref(r), ctypes.byref(w))
        assert (r.value, w.value) == (0, 1)
        rows = torch.randint(0, 255, (37, 12), dtype=torch.uint8, device=gpu)
        out = torch.zeros_like(rows)
        nb = L.reidmi_comm_allgather_rows_scratch_bytes(1, 37, 12)
        assert nb == 37 * 12
        scratch = torch.empty(nb, dtype=torch.uint8, device=gpu)
        _lib.call("reidmi_comm_allgather_rows", comm, _lib.ptr(rows), 37, 12, _lib.ptr(out), _lib.ptr(scratch), nb,
                  _lib.stream())
        x = torch.randn(1000, dtype=torch.float64, device=gpu)
        y = torch.empty_like(x)
        _lib.call("reidmi_comm_allreduce", comm, _lib.ptr(x), _lib.ptr(y), 1000, 1, _lib.stream())
        torch.cuda.synchronize()
        assert torch.equal(out, rows) and torch.equal(x, y)
    finally:
        _lib.call("reidmi_comm_destroy", comm)
