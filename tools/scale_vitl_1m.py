"""BASELINE.json configs[4]: ViT-L/14 synthetic 1M-image gallery of 256x128 crops (the
HBM-roofline stress), sharded over the GPUs of one node (torchrun, one process per GPU;
plain `python` = 1 GPU).  Prints one JSON line (rank 0).

Legs (each timed on its own, wall seconds max over ranks):
  embed   ViT-L/14 as the reference executes it (12 of 24 blocks, 211 tokens), 2 passes per
          image, on a sample of this rank's gallery shard -> images/s (whole job)
  eval    Q x G exact-fp32 distmat + CMC/mAP on identity-clustered synthetic features,
          D_feat = 1024 + 768 = 1792, each rank its query shard against the whole gallery
  rerank  k-reciprocal re-rank (k1=50, k2=15, lambda=0.3) over N = Q + G, row-sharded
          staged path (reranking.re_ranking_sharded) + CMC/mAP
  embed_full (--embed-full) every one of the Q + G images embedded (not a sample): crops
          generated on the device block by block (seeded per block, never all resident), both
          passes, features written into the gallery / query matrices; then L2-normalise, the
          exact distance and CMC/mAP on THOSE features (eval_embedded).  The random network's
          embeddings carry no identity signal (mAP at chance); the leg times the whole
          configs[4] job end to end instead of projecting the embed from a sample.

    python tools/scale_vitl_1m.py [--gallery 1000000] [--query 10000] [--embed-sample 4096]
                                  [--no-rerank] [--no-embed] [--embed-full] [--batch 256]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import distributed as rd, evaluate, reranking, synthetic as syn  # noqa: E402
from multimodal_reid_amd import zero_shot_learning as zsl  # noqa: E402
from multimodal_reid_amd.model import VisionTransformer  # noqa: E402

VITL_GFLOP_PER_PASS = 66.49


def sync(world):
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()


def tmax(t, dev, world):
    v = torch.tensor([t], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
    return float(v.item())


def clustered_features(pids, num_ids, dim, dev, seed):
    """Identity-clustered Gaussian features (centre N(0, I), noise sigma 4), L2-normalised."""
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    centres = torch.randn((num_ids + 1, dim), generator=g, device=dev)
    p = torch.from_numpy(pids).to(dev)
    x = centres[p.clamp(min=0)] + 4.0 * torch.randn((len(pids), dim), generator=g, device=dev)
    own = p <= 0
    k = int(own.sum())
    x[own] = torch.randn((k, dim), generator=g, device=dev) + 4.0 * torch.randn((k, dim), generator=g, device=dev)
    return evaluate.l2_normalize_device(x)


def cmc_map(d, qp, gp, qc, gc, Q, G):
    valid, first, ap, nkept, ovf = evaluate.eval_rows_device(d, qp, gp, qc, gc)
    rows = rd.gather_rows(torch.stack([valid.double(), first.double(), ap, nkept.double()], 1), Q)
    rows = rows.cpu().numpy()
    return evaluate.aggregate_cmc_map(rows[:, 0].astype(np.int64), rows[:, 1].astype(np.int64), rows[:, 2],
                                      rows[:, 3].astype(np.int64), G, 50)


def embed_leg(dev, rank, world, n, batch, G):
    sd = syn.vit_state_dict("ViT-L/14", seed=0, layers=12)
    m = VisionTransformer(sd, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(7 + rank)
    imgs = (torch.rand((n, 3, 256, 128), generator=gen, device=dev) * 2 - 1).half()
    tta = torch.from_numpy(syn.tta_offsets(n, seed=3, offset=rank * n)).to(dev)
    emb = torch.empty((n, m.width + m.out_dim), device=dev)

    def run():
        for s in range(0, n, batch):
            e = min(s + batch, n)
            zsl.embed_pair(m, imgs[s:e], tta=tta[s:e], out=emb[s:e])

    run()
    sync(world)
    t = time.perf_counter()
    run()
    sync(world)
    te = tmax(time.perf_counter() - t, dev, world)
    rate = world * n / te
    tf = rate * 2 * VITL_GFLOP_PER_PASS / 1e3
    return {"sample_imgs_per_rank": n, "imgs_per_s": round(rate, 1), "TFLOPs": round(tf, 1),
            "frac_of_fp16_peak": round(tf / (2500.0 * world), 4), "projected_gallery_embed_s": round(G / rate, 1)}


def embed_full_leg(dev, rank, world, Q, G, batch, block=8192):
    """Embed this rank's shard of the Q + G images (both passes) -> (record, fp32 features of
    the shard [n, 1792]).  Progress on stderr every block (a 1M job runs for minutes)."""
    sd = syn.vit_state_dict("ViT-L/14", seed=0, layers=12)
    m = VisionTransformer(sd, device=dev)
    lo, hi = rd.shard(Q + G, rank, world)
    n = hi - lo
    feat = torch.empty((n, m.width + m.out_dim), device=dev)
    gen = torch.Generator(device=dev)
    imgs = torch.empty((block, 3, 256, 128), device=dev, dtype=torch.float16)
    sync(world)
    t = time.perf_counter()
    # global blocks of `block` images, each generated whole from its own seed and cut to this
    # rank's range, so image k is the same for any world size
    for gb in range(lo // block, -(-hi // block)):
        g0, g1 = gb * block, min((gb + 1) * block, Q + G)
        gen.manual_seed(1_000_003 * gb + 17)
        x = imgs[:g1 - g0]
        x.copy_(torch.rand((g1 - g0, 3, 256, 128), generator=gen, device=dev) * 2 - 1)
        tta = torch.stack([torch.randint(0, 11, (g1 - g0,), generator=gen, device=dev),
                           torch.randint(0, 21, (g1 - g0,), generator=gen, device=dev)], 1).to(torch.int32)
        a, b = max(g0, lo), min(g1, hi)
        for s in range(a, b, batch):
            e = min(s + batch, b)
            zsl.embed_pair(m, x[s - g0:e - g0], tta=tta[s - g0:e - g0], out=feat[s - lo:e - lo])
        if rank == 0 and gb % 8 == 0:
            torch.cuda.synchronize()
            print(f"embed_full: {b - lo}/{n} images of rank 0's shard, {time.perf_counter() - t:.1f} s",
                  file=sys.stderr, flush=True)
    sync(world)
    te = tmax(time.perf_counter() - t, dev, world)
    rate = (Q + G) / te
    tf = rate * 2 * VITL_GFLOP_PER_PASS / 1e3
    rec = {"images": Q + G, "wall_s": round(te, 2), "imgs_per_s": round(rate, 1), "TFLOPs": round(tf, 1),
           "frac_of_fp16_peak": round(tf / (2500.0 * world), 4), "batch": batch,
           "finite": bool(torch.isfinite(feat).all().item())}
    del m, imgs
    return rec, feat


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gallery", type=int, default=1000000)
    ap.add_argument("--query", type=int, default=10000)
    ap.add_argument("--ids", type=int, default=10000)
    ap.add_argument("--embed-sample", type=int, default=4096)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--no-rerank", action="store_true")
    ap.add_argument("--no-embed", action="store_true")
    ap.add_argument("--embed-full", action="store_true")
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    Q, G, D = a.query, a.gallery, 1024 + 768
    out = {"config": f"ViT-L/14 synthetic gallery {G} x query {Q}, {world} GPU(s)", "n_gpus": world}
    if not a.no_embed:
        out["embed"] = embed_leg(dev, rank, world, a.embed_sample, a.batch, G)
        torch.cuda.empty_cache()

    qp, gp, qc, gc = syn.labels(Q, G, a.ids, 8, seed=0, distractor_frac=0.1, junk_frac=0.0)
    if a.embed_full:
        rec, f = embed_full_leg(dev, rank, world, Q, G, a.batch)
        torch.cuda.empty_cache()
        sync(world)
        t = time.perf_counter()
        f = rd.gather_rows(evaluate.l2_normalize_device(f), Q + G)  # images are [queries | gallery]
        qlo, qhi = rd.shard(Q, rank, world)
        d = evaluate.euclidean_distance_device(f[qlo:qhi], f[Q:])
        cmc, mAP = cmc_map(d, qp[qlo:qhi], gp, qc[qlo:qhi], gc, Q, G)
        sync(world)
        tv = tmax(time.perf_counter() - t, dev, world)
        out["embed_full"] = rec
        out["eval_embedded"] = {"wall_s": round(tv, 3), "mAP": round(float(mAP), 6), "rank1": round(float(cmc[0]), 6),
                                "end_to_end_s": round(rec["wall_s"] + tv, 2)}
        del d, f
        torch.cuda.empty_cache()
    feats = clustered_features(np.concatenate([qp, gp]), a.ids, D, dev, seed=11)
    qn, gn = feats[:Q], feats[Q:]
    qlo, qhi = rd.shard(Q, rank, world)
    sync(world)
    t = time.perf_counter()
    d = evaluate.euclidean_distance_device(qn[qlo:qhi], gn)
    cmc, mAP = cmc_map(d, qp[qlo:qhi], gp, qc[qlo:qhi], gc, Q, G)
    sync(world)
    tv = tmax(time.perf_counter() - t, dev, world)
    out["eval"] = {"wall_s": round(tv, 3), "mAP": round(float(mAP), 6), "rank1": round(float(cmc[0]), 6),
                   "distmat_TFLOP": round(2.0 * Q * G * D / 1e12, 2), "distmat_bytes": 4 * Q * G}
    del d
    torch.cuda.empty_cache()

    if not a.no_rerank:
        sync(world)
        t = time.perf_counter()
        final = reranking.re_ranking_sharded(qn, gn, 50, 15, 0.3)
        cmc_r, mAP_r = cmc_map(final, qp[qlo:qhi], gp, qc[qlo:qhi], gc, Q, G)
        sync(world)
        tr = tmax(time.perf_counter() - t, dev, world)
        N = Q + G
        out["rerank"] = {"N": N, "wall_s": round(tr, 3), "mAP": round(float(mAP_r), 6),
                         "rank1": round(float(cmc_r[0]), 6), "top_k_distance_TFLOP": round(2.0 * N * N * D / 1e12, 1),
                         "finite": bool(torch.isfinite(final).all().item())}
        del final
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
