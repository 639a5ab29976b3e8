"""world_size-2 (and 3) gloo runs of the data-parallel eval on CPU: sharding, all-gather of
gallery feature blocks and the order-preserving reduction give CMC/mAP bit-identical to a
single process.  Per-rank compute here is the oracle (the GPU kernels are bit-exact with it,
tests/test_gpu_backend.py); the sharding, communication and reduction code is the product's
(multimodal_reid_amd.distributed + evaluate.aggregate_cmc_map)."""
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402  (spawned workers re-import this module without conftest)

reidmi_boot.load()

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from multimodal_reid_amd import distributed as rd
from multimodal_reid_amd import synthetic as syn

Q, G = 90, 410


def _data():
    qp, gp, qc, gc = syn.labels(Q, G, num_ids=50, num_cams=5, seed=21, junk_frac=0.03)
    qf, gf = syn.features(qp, gp, dim=128, seed=21)
    feats = oracle.l2norm(np.concatenate([qf, gf]))
    return feats[:Q], feats[Q:], qp, gp, qc, gc


def _rows_fn(q, g, qp, gp, qc, gc):
    d = oracle.distmat(q.numpy(), g.numpy())
    return oracle.eval_rows(d, qp, gp, qc, gc)


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    qf, gf, qp, gp, qc, gc = _data()
    qlo, qhi = rd.shard(Q, rank, world)
    glo, ghi = rd.shard(G, rank, world)
    cmc, mAP = rd.sharded_eval(torch.from_numpy(qf[qlo:qhi]), torch.from_numpy(gf[glo:ghi]), qp, gp, qc, gc, Q, G,
                               _rows_fn, 50)
    g_all = rd.gather_rows(torch.from_numpy(gf[glo:ghi]), G)
    # the variable-size all-to-all of the sharded R2 (rank r sends q + r + 1 values to rank q)
    send = torch.cat([torch.full((q + rank + 1,), 100 * rank + q, dtype=torch.int64) for q in range(world)])
    recv, splits = rd.all_to_all_var(send, [q + rank + 1 for q in range(world)])
    want = torch.cat([torch.full((rank + s + 1,), 100 * s + rank, dtype=torch.int64) for s in range(world)])
    a2a_ok = torch.equal(recv, want) and splits == [rank + s + 1 for s in range(world)]
    # the drop-in's default: no collective (distributed.local) even with a process group
    with rd.local():
        local_ok = rd.world() == (0, 1) and rd.gather_rows(torch.ones(3), 3).shape == (3,)
    out[rank] = (cmc, mAP, bool(torch.equal(g_all, torch.from_numpy(gf))), bool(a2a_ok), bool(local_ok),
                 rd.world() == (rank, world))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_eval_matches_single_process(world):
    qf, gf, qp, gp, qc, gc = _data()
    ref_cmc, ref_map = oracle.eval_func(oracle.distmat(qf, gf), qp, gp, qc, gc, 50)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        cmc, mAP, gathered_ok, a2a_ok, local_ok, world_ok = out[r]
        assert gathered_ok and a2a_ok and local_ok and world_ok
        assert np.array_equal(cmc, ref_cmc) and mAP == ref_map


def test_shard_partition():
    for n in (1, 7, 3368, 82161):
        for w in (1, 2, 3, 8):
            parts = [rd.shard(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in parts]
            assert max(sizes) - min(sizes) <= 1


def test_aggregate_refuses_overflowed_queries():
    """valid = -1 (a query beyond eval_rows' positive-list capacity) travels through the
    gathered per-query rows and makes the aggregation raise instead of reporting a wrong AP."""
    from multimodal_reid_amd import _lib
    from multimodal_reid_amd.distributed import pack_rows, unpack_rows
    from multimodal_reid_amd.evaluate import aggregate_cmc_map
    rows = pack_rows(np.array([1, -1, 1]), np.array([0, -1, 3]), np.array([1.0, 0.0, 0.25]), np.array([90, 90, 90]))
    with pytest.raises(_lib.ReidmiError):
        aggregate_cmc_map(*unpack_rows(rows), 100, 50)
    cmc, mAP = aggregate_cmc_map(*unpack_rows(rows[[0, 2]]), 100, 50)
    assert mAP == np.mean([1.0, 0.25]) and cmc[0] == 0.5 and cmc[3] == 1.0
