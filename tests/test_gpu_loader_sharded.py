"""The files-to-mAP flow, sharded one process per rank: loader.get_loader(..., shard=(rank, world))
-> inference() (zero_shot_learning.py:61-134) -> get_cmc_map(..., sharded=True)
(zero_shot_learning.py:137-150 over R1_mAP_eval's sharded compute), with 2 gloo ranks sharing
cuda:0, gives the CMC/mAP of one process over the whole split (plain and re-ranked); each rank's
loaders walk its contiguous shard with the RandomCrop offsets those items have in one process.
(gloo moves the collectives' bytes through the host; RCCL refuses several ranks on one GPU.)"""
import os
import socket
import sys
import types

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import reidmi_boot  # noqa: E402

reidmi_boot.load()

from multimodal_reid_amd import synthetic as syn  # noqa: E402

pytestmark = pytest.mark.gpu

Q, G, BATCH = 61, 203, 40


def _dataset():
    qp, gp, qc, gc = syn.labels(Q, G, num_ids=25, num_cams=6, seed=4, junk_frac=0.03)
    files = syn.jpeg_files(Q + G, 128, 64, seed=9, quality=90)
    q = [(files[k], int(qp[k]), int(qc[k]), 0, k) for k in range(Q)]
    g = [(files[Q + k], int(gp[k]), int(gc[k]), 0, k) for k in range(G)]
    return types.SimpleNamespace(query=q, gallery=g)


def _run(dev, rank, world):
    from multimodal_reid_amd import loader, model, zero_shot_learning as zsl
    vit = model.VisionTransformer(syn.vit_state_dict("ViT-B/16", seed=2), device=dev)
    shard = (rank, world) if world > 1 else None
    lg, lq, lga, lqa = loader.get_loader(_dataset(), BATCH, 256, 128, "vit", device=dev, tta_seed=5, shard=shard)
    g_emb, g_pid, g_cam, _ = zsl.inference(vit, None, None, None, lg, lga, False, "vit")
    q_emb, q_pid, q_cam, _ = zsl.inference(vit, None, None, None, lq, lqa, False, "vit")
    res = {"n": (len(g_pid), len(q_pid))}
    for rr in (False, True):
        cmc, mAP = zsl.get_cmc_map(g_emb, q_emb, g_pid, q_pid, g_cam, q_cam, reranking=rr, sharded=world > 1)
        res[rr] = (np.asarray(cmc), float(mAP))
    return res


def _worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        out[rank] = _run(torch.device("cuda", 0), rank, world)
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sharded_loaders_to_map_equal_single(gpu):
    import torch.multiprocessing as mp
    one = _run(gpu, 0, 1)
    assert one["n"] == (G, Q)
    assert one[False][0][-1] > 0 and 0 < one[False][1] <= 1
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    assert out[0]["n"][0] + out[1]["n"][0] == G and out[0]["n"][1] + out[1]["n"][1] == Q
    for r in range(2):
        for rr in (False, True):
            cmc, mAP = out[r][rr]
            assert np.array_equal(cmc, one[rr][0]) and mAP == one[rr][1], (r, rr, mAP, one[rr][1])
