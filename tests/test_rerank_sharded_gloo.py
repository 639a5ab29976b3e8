"""Staged / sharded k-reciprocal re-ranking on CPU.

The product's orchestration (multimodal_reid_amd.reranking.staged_rerank: row-range stages,
all-gathers of initial_rank, od divisors and CSR rows of V / V_qe) is driven with the
oracle's stage restatement (oracle.RerankStages) as the per-rank compute, under gloo with
world sizes 1-3.  Every world size must reproduce the one-call oracle (itself pinned
bit-exact to the reference's re_ranking, tests/test_oracle.py) bit for bit."""
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
from multimodal_reid_amd import reranking
from multimodal_reid_amd import synthetic as syn

CASES = [(40, 260, 20, 6), (37, 211, 50, 15), (30, 170, 10, 1)]


def _feat(Q, G, seed):
    qp, gp, _, _ = syn.labels(Q, G, num_ids=30, num_cams=4, seed=seed)
    qf, gf = syn.features(qp, gp, dim=64, seed=seed)
    return oracle.l2norm(np.concatenate([qf, gf]))


def _reference(feat, Q, k1, k2):
    return oracle.rerank_from_dist(oracle.distmat(feat, feat), Q, k1, k2, 0.3)


@pytest.mark.parametrize("Q,G,k1,k2", CASES)
def test_staged_single_process_matches_one_call(Q, G, k1, k2):
    feat = _feat(Q, G, seed=Q + G)
    stages = oracle.RerankStages(feat, Q, k1, k2, 0.3)
    out = reranking.staged_rerank(stages, Q + G, Q).numpy()
    ref = _reference(feat, Q, k1, k2)
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))


def _worker(rank, world, port, case, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    Q, G, k1, k2 = case
    feat = _feat(Q, G, seed=Q + G)
    stages = oracle.RerankStages(feat, Q, k1, k2, 0.3)
    part = reranking.staged_rerank(stages, Q + G, Q)
    full = rd.gather_rows(part, Q)
    out[rank] = full.numpy()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("case", CASES[:2])
def test_sharded_rerank_matches_single_process(world, case):
    Q, G, k1, k2 = case
    ref = _reference(_feat(Q, G, seed=Q + G), Q, k1, k2)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), case, out), nprocs=world, join=True)
    for r in range(world):
        assert np.array_equal(out[r].view(np.uint32), ref.view(np.uint32))


def test_gather_var_single_process_identity():
    x = torch.arange(7, dtype=torch.int32)
    assert torch.equal(rd.gather_var(x), x)
