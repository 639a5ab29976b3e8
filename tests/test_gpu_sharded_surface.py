"""The sharded eval exactly as it runs in production, on one GPU:

* bench.py's own Market step (Workload.step: sharded embed, all-gather of the gallery blocks,
  distmat + eval of the rank's queries, all-gather of per-query results) and its MSMT17 leg
  (msmt17_leg: + the row-sharded k-reciprocal re-rank) at reduced split sizes, with 2 and 3
  gloo ranks sharing cuda:0 -> CMC/mAP identical to one process;
* the reference call surface under a process group: zero_shot_learning.get_cmc_map(...,
  reranking=False/True, sharded=True) given each rank's shards (R1_mAP_eval's sharded compute)
  -> identical to one process over the whole split;
* re_ranking_device(..., sharded=True) with the full features on every rank (row-sharded
  stages + all-gather of the final rows) -> the one-process matrix bit for bit;
* the default (unsharded) surface under a process group issues no collective: only the last
  rank calls get_cmc_map / re_ranking_device on the full split (as a DDP script evaluating on
  one rank does) and gets the one-process result; the other ranks never call it (no hang).
(gloo moves the collectives' bytes through the host; RCCL refuses several ranks on one GPU.)"""
import os
import socket
import sys

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import reidmi_boot  # noqa: E402

reidmi_boot.load()

from multimodal_reid_amd import synthetic as syn  # noqa: E402

pytestmark = pytest.mark.gpu

MARKET = dict(num_query=97, num_gallery=410, num_ids=40, num_cams=6)
MSMT = dict(num_query=83, num_gallery=377, num_ids=30, num_cams=15)
BATCH = 48


def _model(dev):
    from multimodal_reid_amd.model import VisionTransformer
    return VisionTransformer(syn.vit_state_dict("ViT-B/16", seed=0), device=dev)


def _surface(dev, rank, world):
    """get_cmc_map over this rank's shards of identity-clustered features (plain and re-ranked)
    and re_ranking_device with the full features on every rank."""
    from multimodal_reid_amd import distributed as rd, reranking, zero_shot_learning as zsl
    Q, G = 130, 620
    qp, gp, qc, gc = syn.labels(Q, G, num_ids=50, num_cams=6, seed=7, junk_frac=0.02)
    qf, gf = syn.features(qp, gp, dim=256, seed=7)
    qlo, qhi = rd.shard(Q, rank, world)
    glo, ghi = rd.shard(G, rank, world)
    q = torch.from_numpy(qf[qlo:qhi]).to(dev)
    g = torch.from_numpy(gf[glo:ghi]).to(dev)
    res = {}
    for rr in (False, True):
        cmc, mAP = zsl.get_cmc_map(g, q, torch.from_numpy(gp[glo:ghi]), torch.from_numpy(qp[qlo:qhi]),
                                   torch.from_numpy(gc[glo:ghi]), torch.from_numpy(qc[qlo:qhi]), reranking=rr,
                                   sharded=rd._initialized())
        res[rr] = (np.asarray(cmc), float(mAP))
    from multimodal_reid_amd import evaluate
    qn = evaluate.l2_normalize_device(torch.from_numpy(qf).to(dev))
    gn = evaluate.l2_normalize_device(torch.from_numpy(gf).to(dev))
    full = reranking.re_ranking_device(qn, gn, 20, 6, 0.3, sharded=rd._initialized()).cpu().numpy()
    if rank == world - 1:
        # the default surface on the full split, on one rank only: single-process semantics
        for rr in (False, True):
            cmc, mAP = zsl.get_cmc_map(torch.from_numpy(gf).to(dev), torch.from_numpy(qf).to(dev),
                                       torch.from_numpy(gp), torch.from_numpy(qp), torch.from_numpy(gc),
                                       torch.from_numpy(qc), reranking=rr)
            res[("full", rr)] = (np.asarray(cmc), float(mAP))
        res["full_rr"] = reranking.re_ranking_device(qn, gn, 20, 6, 0.3).cpu().numpy()
    return res, full


def _bench(dev, rank, world):
    import bench
    model = _model(dev)
    wl = bench.Workload(dev, rank, world, BATCH, dataset=MARKET, model=model)
    cmc, mAP, _, _, _ = wl.step()
    leg = bench.msmt17_leg(model, dev, rank, world, BATCH, dataset=MSMT)
    return np.asarray(cmc), float(mAP), leg["mAP"], (leg["rerank"]["mAP_rerank"], leg["rerank_embedded"]["mAP_rerank"])


def _worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        out[rank] = (_bench(dev, rank, world), _surface(dev, rank, world))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def single(gpu):
    return _bench(gpu, 0, 1), _surface(gpu, 0, 1)


@pytest.mark.parametrize("world", [2, 3])
def test_bench_step_and_surface_sharded_equal_single(single, world):
    import torch.multiprocessing as mp
    (cmc1, map1, ms1, msrr1), (surf1, full1) = single
    assert cmc1[0] > 0 and 0 < map1 <= 1  # a real ranking, not an empty one
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        (cmc, mAP, ms, msrr), (surf, full) = out[r]
        assert np.array_equal(cmc, cmc1) and mAP == map1, (r, mAP, map1)
        assert ms == ms1 and msrr == msrr1, (r, ms, ms1, msrr, msrr1)
        for rr in (False, True):
            assert np.array_equal(surf[rr][0], surf1[rr][0]) and surf[rr][1] == surf1[rr][1], (r, rr)
        assert np.array_equal(full.view(np.uint32), full1.view(np.uint32))
    last = out[world - 1][1][0]
    for rr in (False, True):
        assert np.array_equal(last[("full", rr)][0], surf1[rr][0]) and last[("full", rr)][1] == surf1[rr][1], rr
    assert np.array_equal(last["full_rr"].view(np.uint32), full1.view(np.uint32))
