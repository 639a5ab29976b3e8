"""bench.py — BASELINE.json configs[1]: ViT-B/16 Market-1501 full eval on MI355X.

One step = the whole hot path over the Market-1501 test split (3368 query + 15913 gallery
synthetic 256x128 crops resident in HBM): every image through the ViT-B/16 stride-12
encoder twice (plain + flip/pad/crop TTA view, zero_shot_learning.py:80-128), fused feature
epilogue, L2-normalise, exact-fp32 query x gallery distance matrix, CMC/mAP
(evaluate.py:29-135).  value = images (query+gallery) per second over the whole step.

Multi-GPU (torchrun, one process per GPU, RCCL): rank r embeds its contiguous shard of
the query and of the gallery images; gallery features are all-gathered (the path's one
exchange step); each rank scores its query shard against the full gallery; per-query
results are all-gathered and rank 0 reduces them in query order (bit-identical to N=1).
Total work is fixed as N grows ("strong").

Extra legs in the same JSON line (not part of `value`): "msmt17" = configs[3] / the north
star's target, MSMT17 end to end on all ranks (sharded embed, all-gather, distmat + CMC/mAP,
sharded k-reciprocal re-rank + CMC/mAP, wall seconds max over ranks); "rerank" = configs[2]'s
Duke-size re-rank on rank 0 with the C port timed on the full config; "text" = the --mm
zero-shot classifier's text side at Market size (750 x 56 token rows, TF/s); "backend" /
"preprocess" = retrieval-kernel and transform rooflines; "jpeg" = the loaders' JPEG decode of
a Market split of files on the device (and + transform), Pillow timed beside it; "files_to_map" =
the same Market eval from 19 281 host JPEG buffers through get_loader -> inference ->
get_cmc_map (N = 1); "cpu_baseline".

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B (default 20480)] [--backend nccl|gloo]
                    [--no-cpu-baseline] [--no-rerank] [--no-msmt17] [--no-text] [--no-jpeg] [--no-files]

`--gpus N` under torchrun (WORLD_SIZE set) must equal the world size; without torchrun,
bench.py starts the N rank processes itself (launch_ranks) and relays rank 0's line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import _lib, evaluate, synthetic as syn  # noqa: E402
from multimodal_reid_amd.distributed import gather_rows, shard  # noqa: E402
from multimodal_reid_amd import zero_shot_learning as zsl  # noqa: E402
from multimodal_reid_amd.model import VisionTransformer  # noqa: E402

PEAK_F16_TFLOPS = 2500.0  # MI355X dense fp16/bf16 MFMA (MI355X_MICROARCH.md)
PEAK_F32_MATRIX_TFLOPS = 157.3  # MI355X fp32 matrix (v_mfma_f32_32x32x2_f32)
PEAK_HBM_GBPS = 8000.0
EPI_GELU = 1  # the c_fc GEMM (+QuickGELU epilogue): the largest single kernel per block
# HBM-side bytes per full-batch c_fc launch (ln_2-folded fp16 GEMM, M = batch * 211, N = 3072,
# K = 768, auto tile walk = 2 N-groups), from rocprofv3 PMC passes of that launch
# (tools/prof_round.sh): FETCH_SIZE doubled (gfx950 reports half of 16-B/lane streaming reads,
# MI355X_MICROARCH.md "HBM") + WRITE_SIZE, KiB, mean of 6 launches.  FETCH_SIZE also counts
# Infinity-Cache hits: A panels are re-read by the 2 XCD groups and W panels by the rounds of
# an XCD (4 MB L2).  Other batches: not measured (null).
#   batch 1024 (profiles/r02/pmc_c_fc_fp16_walk2_*): 736 400 / 1 296 384 KiB; algorithmic
#     A 332 MB + W 4.7 MB + out 1 327 MB = 1.66 GB
#   batch 4096 (profiles/r04/final/pmc_c_fc_b4096_*, mean of 6 launches; r03: 3 142 462 /
#     5 185 615): 2 998 177 / 5 185 700 KiB; algorithmic A 1 327 MB + W 4.7 MB + out 5 310 MB = 6.64 GB
#   batch 19281, the one call per pass at Market size (profiles/r05/prof/pmc_c_fc_b19281_*, median
#     of 6 launches): 13 840 234 / 24 410 478 KiB; algorithmic A 6 249 MB + W 4.7 MB + out 24 996 MB
#     = 31.25 GB
C_FC_TRAFFIC_BYTES = {1024: (2 * 736400 + 1296384) * 1024, 4096: (2 * 2998177 + 5185700) * 1024,
                      19281: (2 * 13840234 + 24410478) * 1024}


def _max_over_ranks(values, dev):
    """Max over ranks of host floats (RCCL moves device tensors, gloo host tensors)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [float(v) for v in values]
    t = torch.tensor(values, dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.cpu()]


def _all_ranks(values, dev):
    """Every rank's list of host floats, in rank order (one all-gather)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [[float(v) for v in values]]
    t = torch.tensor(values, dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [[float(v) for v in o.cpu()] for o in out]


def _crops(lo, hi, seed, dev, block=128):
    """fp16 U(-1,1) crops [hi-lo, 3, 256, 128] of global image indices lo..hi: block b of
    `block` images comes from a generator seeded (seed, b), so a shard's images do not depend
    on how the split is sharded."""
    out = torch.empty((hi - lo, 3, 256, 128), dtype=torch.float16, device=dev)
    gen = torch.Generator(device=dev)
    for b in range(lo // block, -(-hi // block)):
        a, z = max(lo, b * block), min(hi, (b + 1) * block)
        gen.manual_seed(seed * 1000003 + b)
        x = torch.rand((block, 3, 256, 128), generator=gen, device=dev)
        out[a - lo:z - lo] = (x[a - b * block:z - b * block] * 2 - 1).half()
    return out


class IdentityCrops:
    """Identity-structured synthetic crops on the device (the same construction as
    synthetic.identity_crops, generated with torch on the GPU so a 93 820-image split takes
    seconds): a base image per pid (a 16x8 U(-1,1) grid upsampled bilinearly + a fixed
    high-frequency texture; distractors pid <= 0 take one of 1024 bases of their own by image
    index), a colour cast and a horizontal shift per camera, Gaussian noise per image, clipped
    to [-1, 1], fp16.  Image k depends only on (seed, pids, cams, k): independent of sharding."""

    def __init__(self, num_ids, num_cams, seed, dev, height=256, width=128, noise=0.6, detail=0.3, cast=0.02,
                 n_distractor_bases=1024):
        self.dev, self.noise, self.seed = dev, noise, seed
        self.num_ids, self.nd = num_ids, n_distractor_bases
        gen = torch.Generator(device=dev)
        nb = num_ids + n_distractor_bases
        self.bases = torch.empty((nb, 3, height, width), dtype=torch.float16, device=dev)
        for a in range(0, nb, 256):
            z = min(nb, a + 256)
            gen.manual_seed(seed * 7919 + a)
            coarse = torch.rand((z - a, 3, 16, 8), generator=gen, device=dev) * 2 - 1
            up = torch.nn.functional.interpolate(coarse, size=(height, width), mode="bilinear", align_corners=True)
            up += detail * (torch.rand((z - a, 3, height, width), generator=gen, device=dev) * 2 - 1)
            self.bases[a:z] = up.half()
        gen.manual_seed(seed * 7919 + 104729)
        self.cast = cast * torch.randn((num_cams, 3, 1, 1), generator=gen, device=dev)
        self.shift = torch.randint(-1, 2, (num_cams,), generator=gen, device=dev)
        col = torch.arange(width, device=dev)
        self.cols = (col[None, :] - self.shift[:, None]) % width  # np.roll by shift along width

    def __call__(self, pids, cams, lo, hi, block=128):
        """fp16 [hi-lo, 3, H, W] crops of global image indices lo..hi (pids / cams: the split's
        full label arrays)."""
        H, W = self.bases.shape[2:]
        out = torch.empty((hi - lo, 3, H, W), dtype=torch.float16, device=self.dev)
        gen = torch.Generator(device=self.dev)
        p_all = torch.from_numpy(np.asarray(pids)).to(self.dev)
        c_all = torch.from_numpy(np.asarray(cams)).to(self.dev)
        for b in range(lo // block, -(-hi // block)):
            a, z = max(lo, b * block), min(hi, (b + 1) * block)
            gen.manual_seed(self.seed * 1000003 + b)
            nz = self.noise * torch.randn((block, 3, H, W), generator=gen, device=self.dev)[a - b * block:z - b * block]
            idx = torch.arange(a, z, device=self.dev)
            p, c = p_all[a:z], c_all[a:z]
            bi = torch.where(p > 0, p - 1, self.num_ids + idx % self.nd)
            base = self.bases[bi].float()
            cols = self.cols[c]  # [n, W]
            base = torch.gather(base, 3, cols[:, None, None, :].expand(-1, 3, H, -1))
            out[a - lo:z - lo] = (base + self.cast[c] + nz).clamp_(-1.0, 1.0).half()
        return out


class Workload:
    def __init__(self, dev, rank, world, batch, dataset="market1501", model=None, crops="uniform", streams=1,
                 resid_gain=1.0):
        # dataset: a name of synthetic.DATASET_SPLITS, or such a dict (tests run reduced splits)
        sp = syn.DATASET_SPLITS[dataset] if isinstance(dataset, str) else dataset
        self.Q, self.G = sp["num_query"], sp["num_gallery"]
        self.q_pids, self.g_pids, self.q_cams, self.g_cams = syn.labels(
            self.Q, self.G, sp["num_ids"], sp["num_cams"], seed=0, distractor_frac=0.1, junk_frac=0.02)
        self.rank, self.world, self.batch, self.dev = rank, world, batch, dev
        self.sd = syn.vit_state_dict("ViT-B/16", seed=0, resid_gain=resid_gain) if model is None else None
        self.model = VisionTransformer(self.sd, device=dev) if model is None else model
        # synthetic crops of this rank's shards, resident in HBM as fp16 (U(-1,1)); image k of a
        # split is the same for every world size (generated in seeded blocks of global indices)
        self.qlo, self.qhi = shard(self.Q, rank, world)
        self.glo, self.ghi = shard(self.G, rank, world)
        if crops == "identity":  # identity-structured (the MSMT17 leg: real-like k-reciprocal neighbourhoods)
            ic = IdentityCrops(sp["num_ids"], sp["num_cams"], 5, dev, noise=0.3)
            self.q_img = ic(self.q_pids, self.q_cams, self.qlo, self.qhi)
            ic.seed = 6
            self.g_img = ic(self.g_pids, self.g_cams, self.glo, self.ghi)
            del ic
        else:
            self.q_img = _crops(self.qlo, self.qhi, 1000, dev)
            self.g_img = _crops(self.glo, self.ghi, 2000, dev)
        # one image stream per rank: its query shard then its gallery shard (views of one tensor),
        # embedded in balanced encoder calls of at most `batch` images (one call per pass at
        # Market size: fewer, larger persistent GEMM launches; profiles/r05/bench_batch*.json)
        nq = self.qhi - self.qlo
        self.img = torch.cat([self.q_img, self.g_img])
        self.q_img, self.g_img = self.img[:nq], self.img[nq:]
        self.tta = torch.cat([torch.from_numpy(syn.tta_offsets(nq, seed=1, offset=self.qlo)),
                              torch.from_numpy(syn.tta_offsets(self.ghi - self.glo, seed=2, offset=self.glo))]).to(dev)
        self.q_tta, self.g_tta = self.tta[:nq], self.tta[nq:]
        D = self.model.width + self.model.out_dim
        self.emb = torch.empty(self.img.shape[0], D, device=dev)
        self.q_emb, self.g_emb = self.emb[:nq], self.emb[nq:]
        n = self.img.shape[0]
        nb = max(1, -(-n // batch))
        self.bounds = [n * i // nb for i in range(nb + 1)]
        self.max_call = max((b - a for a, b in zip(self.bounds, self.bounds[1:])), default=0)
        self.dist = torch.empty(self.qhi - self.qlo, self.G, device=dev)
        # encoder batches alternate over `streams` HIP streams: one batch's kernels fill the CUs a
        # neighbour's leave idle (the last partial round of tiles of each persistent GEMM launch,
        # the short LayerNorm / attention launches, launch gaps); each stream has its workspace
        self.streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(streams - 1)]

    def embed(self):
        """Both TTA passes of every image of this rank (queries then gallery)."""
        main = torch.cuda.current_stream(self.dev)
        for st in self.streams[1:]:
            st.wait_stream(main)
        for i, (s, e) in enumerate(zip(self.bounds, self.bounds[1:])):
            with torch.cuda.stream(self.streams[i % len(self.streams)]):
                zsl.embed_pair(self.model, self.img[s:e], tta=self.tta[s:e], out=self.emb[s:e])
        for st in self.streams[1:]:
            main.wait_stream(st)

    def step(self):
        """One Market eval; returns (cmc, mAP, embed s, all-gather s, eval s) of this rank.  The
        all-gather of the normalised gallery blocks (RCCL under nccl) is timed on its own: it
        includes waiting for the slowest rank, so its minimum over ranks is the collective."""
        t0 = time.perf_counter()
        self.embed()
        qn = evaluate.l2_normalize_device(self.q_emb)
        gl = evaluate.l2_normalize_device(self.g_emb)
        torch.cuda.synchronize()
        ta = time.perf_counter()
        gn = gather_rows(gl, self.G)
        self.gather_bytes = gn.numel() * gn.element_size() if self.world > 1 else 0
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        evaluate.euclidean_distance_device(qn, gn, out=self.dist)
        valid, first, ap, nkept, ovf = evaluate.eval_rows_device(
            self.dist, self.q_pids[self.qlo:self.qhi], self.g_pids, self.q_cams[self.qlo:self.qhi], self.g_cams)
        rows = torch.stack([valid.double(), first.double(), ap, nkept.double()], 1)
        rows = gather_rows(rows, self.Q)
        torch.cuda.synchronize()
        rows = rows.cpu().numpy()
        cmc, mAP = evaluate.aggregate_cmc_map(rows[:, 0].astype(np.int64), rows[:, 1].astype(np.int64), rows[:, 2],
                                              rows[:, 3].astype(np.int64), self.G, 50)
        t2 = time.perf_counter()
        return cmc, mAP, ta - t0, t1 - ta, t2 - t1


MSMT17_RESID_GAIN = 4.0  # synthetic.vit_state_dict resid_gain of the MSMT17 leg's network


def msmt17_leg(model, dev, rank, world, batch, dataset="msmt17"):
    """configs[3] + the north star's target: MSMT17 (11659q x 82161g) end to end — sharded
    embed of every image (2 TTA passes), RCCL all-gather of the normalised feature blocks,
    exact distmat + CMC/mAP, then the sharded k-reciprocal re-rank (k1=50, k2=15, lambda=0.3;
    row-range stages with all-gathers of initial_rank / V / V_qe) + CMC/mAP.  Identity-
    structured crops (IdentityCrops: 3060 ids, 15 cameras), so the embeddings have real
    k-reciprocal neighbourhoods and R2 takes the fp16 pre-filter path the way real features do
    (the U(-1,1) crops put every gallery item inside the bound and send each R2 row to the
    exact fallback).  ``model`` None: ViT-B/16 with CLIP's init except residual-branch output
    projections MSMT17_RESID_GAIN x larger (synthetic.vit_state_dict resid_gain): at CLIP's init
    the blocks barely move the CLS row, every image embeds to nearly the same vector (cosine to
    the mean 0.997) and R2 sends every row to the exact fallback; at gain 4 (0.97-0.98) the
    embedded crops take the fp16 pre-filter path like trained features
    (profiles/r04/feature_spread.txt).  Timed once, after the Market steps (kernels warm); wall
    seconds are max over ranks."""
    from multimodal_reid_amd import reranking
    model_own = model is None
    if model_own:
        model = VisionTransformer(syn.vit_state_dict("ViT-B/16", seed=0, resid_gain=MSMT17_RESID_GAIN), device=dev)
    wl = Workload(dev, rank, world, batch, dataset=dataset, model=model, crops="identity")
    Q, G = wl.Q, wl.G

    def sync():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    def rows_to_map(d):
        valid, first, ap, nkept, ovf = evaluate.eval_rows_device(
            d, wl.q_pids[wl.qlo:wl.qhi], wl.g_pids, wl.q_cams[wl.qlo:wl.qhi], wl.g_cams)
        rows = gather_rows(torch.stack([valid.double(), first.double(), ap, nkept.double()], 1), Q)
        rows = rows.cpu().numpy()
        return evaluate.aggregate_cmc_map(rows[:, 0].astype(np.int64), rows[:, 1].astype(np.int64), rows[:, 2],
                                          rows[:, 3].astype(np.int64), G, 50)

    sync()
    t0 = time.perf_counter()
    wl.embed()
    qn = gather_rows(evaluate.l2_normalize_device(wl.q_emb), Q)
    gn = gather_rows(evaluate.l2_normalize_device(wl.g_emb), G)
    sync()
    t1 = time.perf_counter()
    evaluate.euclidean_distance_device(qn[wl.qlo:wl.qhi], gn, out=wl.dist)
    cmc, mAP = rows_to_map(wl.dist)
    # The re-rank kernels' first launches in a process load their code (~0.1 s, once, whatever
    # the size: profiles/r05/rr_first_call.txt); a small re-rank takes that before the timed
    # call, as the Market steps' warm-up does for the encoder, and its time is reported
    sync()
    tw = time.perf_counter()
    reranking.re_ranking_sharded(qn[:256], gn[:2048], 50, 15, 0.3)
    sync()
    t2 = time.perf_counter()
    stats = {}
    final = reranking.re_ranking_sharded(qn, gn, 50, 15, 0.3, stats=stats)
    cmc_rr, mAP_rr = rows_to_map(final)
    sync()
    t3 = time.perf_counter()
    del final, qn, gn
    # The re-rank + eval timed again on the §8d back-end features (identity-clustered Gaussians,
    # D = 1280) of the same split, the reference point of earlier rounds.
    qf_np, gf_np = syn.features(wl.q_pids, wl.g_pids, dim=1280, seed=0)
    qs = evaluate.l2_normalize_device(torch.from_numpy(qf_np).to(dev))
    gs = evaluate.l2_normalize_device(torch.from_numpy(gf_np).to(dev))
    del qf_np, gf_np
    sync()
    t4 = time.perf_counter()
    stats8 = {}
    final = reranking.re_ranking_sharded(qs, gs, 50, 15, 0.3, stats=stats8)
    cmc8, mAP8 = rows_to_map(final)
    sync()
    t5 = time.perf_counter()
    te, tv, tr, t8, twu = _max_over_ranks([t1 - t0, tw - t1, t3 - t2, t5 - t4, t2 - tw], dev)
    N, D = Q + G, qs.shape[1]
    wl_D = wl.model.width + wl.model.out_dim
    tri_e = N * N * wl_D
    # floors: the R2 pre-filter's product at the fp16 peak, plus the blend's exact fp32 Q x G
    # distances (original_dist, reranking.py:97-99) at the fp32 matrix peak
    fl_e = 2.0 * tri_e / (PEAK_F16_TFLOPS * 1e12) + 2.0 * Q * G * wl_D / (PEAK_F32_MATRIX_TFLOPS * 1e12)
    del wl, final, qs, gs
    torch.cuda.empty_cache()
    tri = N * N * D  # the R2 pre-filter's fp16 product over the upper triangle (2 N^2 D / 2)
    embed_flop = 2 * N * 37.90e9
    fl = 2.0 * tri / (PEAK_F16_TFLOPS * 1e12) + 2.0 * Q * G * D / (PEAK_F32_MATRIX_TFLOPS * 1e12)
    hb = 8.0 * Q * G / (PEAK_HBM_GBPS * 1e9)
    return {"config": f"MSMT17 {Q}q x {G}g, identity-structured crops (3060 ids, 15 cams, noise 0.3), ViT-B/16 "
                      f"(synthetic, residual gain {MSMT17_RESID_GAIN if model_own else 'caller'}) 2 passes/img, "
                      f"{world} GPU(s): sharded embed + all-gather, exact distmat + CMC/mAP, sharded k-reciprocal "
                      "re-rank (k1=50 k2=15 lambda=0.3) + CMC/mAP",
            "imgs_per_s": round((Q + G) / te, 1), "embed_wall_s": round(te, 4), "eval_wall_s": round(tv, 4),
            # end to end = this run's own embedded features through embed, eval and re-rank + eval
            # (ADVICE r4); the Gaussian-feature re-rank below is a separate reference number
            "rerank_eval_wall_s": round(tr, 4), "end_to_end_wall_s": round(te + tv + tr, 4),
            "rerank_kernel_load_warmup_s": round(twu, 4),
            "mAP": float(mAP), "rank1": float(cmc[0]),
            "rerank": {"features": "SURVEY.md §8d identity-clustered Gaussians (D=1280, sigma 4) of this split: the "
                                   "fp16 pre-filter path", "wall_s": round(t8, 4), "mAP_rerank": float(mAP8),
                       "rank1_rerank": float(cmc8[0]), "r2_rows": stats8.get("rows"), "r2_exact_fallback_rows": stats8.get("exact_rows"),
                       "r2_form": stats8.get("form"),
                       "roofline": {"bound": "mfma (R2 fp16 pre-filter 2 N^2 D at the fp16 peak + the blend's exact "
                                             "fp32 Q x G distances 2 Q G D at the fp32 matrix peak)",
                                    "algorithmic_flop": 2.0 * tri, "blend_distance_flop": 2.0 * Q * G * D,
                                    "flop_floor_s": round(fl, 5),
                                    "hbm_floor_s": round(hb, 5), "frac": round(max(fl, hb) / t8, 4)}},
            "rerank_embedded": {"features": f"the embedded crops (D={wl_D}; synthetic network, residual gain "
                                            f"{MSMT17_RESID_GAIN if model_own else 'caller'})", "wall_s": round(tr, 4),
                                "mAP_rerank": float(mAP_rr), "rank1_rerank": float(cmc_rr[0]),
                                "r2_rows": stats.get("rows"), "r2_exact_fallback_rows": stats.get("exact_rows"),
                                "r2_form": stats.get("form"),
                                "roofline": {"bound": "mfma (R2 fp16 pre-filter 2 N^2 D at the fp16 peak + the "
                                                      "blend's exact fp32 Q x G distances 2 Q G D at the fp32 "
                                                      "matrix peak)",
                                             "algorithmic_flop": 2.0 * tri_e, "blend_distance_flop": 2.0 * Q * G * wl_D,
                                             "flop_floor_s": round(fl_e, 5),
                                             "frac": round(max(fl_e, hb) / tr, 4)}},
            "roofline": {"embed": {"bound": "mfma", "achieved": round(embed_flop / te / 1e12, 1),
                                   "peak": PEAK_F16_TFLOPS, "unit": "TFLOP/s",
                                   "frac": round(embed_flop / te / 1e12 / PEAK_F16_TFLOPS, 4),
                                   # the reference's work per pass (SURVEY.md §8d, 37.90 GFLOP); this
                                   # encoder executes 34.6: the last block runs for the CLS row only and
                                   # forms no K / V
                                   "flop_basis": "reference-equivalent 37.90 GFLOP/pass (executed 34.6)",
                                   "executed_TFLOPs": round(embed_flop * 34.6 / 37.90 / te / 1e12, 1)}}}


def rerank_leg(dev, cpu=True, threads=1):
    """configs[2]'s back end: DukeMTMC-size k-reciprocal re-rank (k1=50, k2=15, lambda=0.3;
    reranking.py:29-100, evaluate.py:124-132) + CMC/mAP on identity-clustered synthetic
    features, timed on its own after the Market steps (not part of `value`).
    Roofline: the reference's formulation is bound by the exact-fp32 N x N distance GEMM
    (2 N^2 D FLOP on the 157 TF/s fp32 matrix peak) — far above its HBM floor (4 N^2 distance
    bytes + 4 Q G final bytes at 8 TB/s); frac = max(floors) / wall.  (N >= STAGED_MIN_N runs
    the staged path, whose R2 goes through the fp16 pre-filter: fewer fp32 FLOPs than that
    floor, the same bits.)  cpu_port: the C restatement on the
    full configuration, `threads` host threads."""
    from multimodal_reid_amd import reranking
    sp = syn.DATASET_SPLITS["dukemtmc"]
    Q, G = sp["num_query"], sp["num_gallery"]
    qp, gp, qc, gc = syn.labels(Q, G, sp["num_ids"], sp["num_cams"], seed=0, distractor_frac=0.1, junk_frac=0.02)
    qf_np, gf_np = syn.features(qp, gp)
    qf = evaluate.l2_normalize_device(torch.from_numpy(qf_np).to(dev))
    gf = evaluate.l2_normalize_device(torch.from_numpy(gf_np).to(dev))
    D = qf.shape[1]

    def run():
        d = reranking.re_ranking_device(qf, gf, 50, 15, 0.3)
        valid, first, ap, nkept, ovf = evaluate.eval_rows_device(d, qp, gp, qc, gc)
        torch.cuda.synchronize()
        return evaluate.aggregate_cmc_map(valid.cpu().numpy(), first.cpu().numpy(), ap.cpu().numpy(),
                                          nkept.cpu().numpy(), G, 50, ovf.cpu().numpy())

    run()
    torch.cuda.synchronize()
    t = time.perf_counter()
    cmc, mAP = run()
    wall = time.perf_counter() - t
    N = Q + G
    flop_floor = 2.0 * N * N * D / (PEAK_F32_MATRIX_TFLOPS * 1e12)
    nbytes = 4 * N * N + 4 * Q * G
    byte_floor = nbytes / (PEAK_HBM_GBPS * 1e9)
    out = {"config": f"DukeMTMC {Q}q x {G}g (N={N}) synthetic features D={D}, k1=50 k2=15 lambda=0.3, "
                     "distance + re-rank + CMC/mAP on 1 GPU",
           "wall_s": round(wall, 4), "mAP": round(float(mAP), 6),
           "roofline": {"bound": "mfma-fp32 (exact N x N distance)", "flop_floor_s": round(flop_floor, 5),
                        "hbm_floor_s": round(byte_floor, 5), "algorithmic_flop": 2.0 * N * N * D,
                        "algorithmic_bytes": nbytes, "frac": round(max(flop_floor, byte_floor) / wall, 4)},
           "reference_cpu_s_survey": 122.0}
    if cpu:
        import oracle
        oracle.set_threads(threads)
        t = time.perf_counter()
        oracle.re_ranking(oracle.l2norm(qf_np), oracle.l2norm(gf_np), 50, 15, 0.3)
        tc = time.perf_counter() - t
        out["cpu_port"] = {"sample": f"oracle C re-rank (distance + R2-R7), full {Q}q x {G}g", "wall_s": round(tc, 2),
                           "cores": threads, "kind": "port",
                           "note": "not extrapolated; the reference's numpy took 122 s for this config on 8 cores "
                                   "(SURVEY.md §6)"}
    return out


def backend_rooflines(wl, reps=10):
    """The retrieval kernels of the Market step on their own (HIP events on the launch
    stream, the step's own buffers): exact-fp32 distance (MFMA fp32 bound: 2 Q G D FLOP)
    and eval_rows (HBM bound: one read of the Q x G distances + the gallery labels once,
    4 Q G + 16 G bytes); this rank's query and gallery shards (the whole split at N = 1)."""
    qn = evaluate.l2_normalize_device(wl.q_emb)
    gn = evaluate.l2_normalize_device(wl.g_emb)
    Q, G, D = qn.shape[0], gn.shape[0], qn.shape[1]
    qp, qc = wl.q_pids[wl.qlo:wl.qhi], wl.q_cams[wl.qlo:wl.qhi]

    def timed(fn):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e-3

    dist_buf = torch.empty(Q, G, device=wl.dev)
    gp, gc = wl.g_pids[wl.glo:wl.ghi], wl.g_cams[wl.glo:wl.ghi]
    td16 = timed(lambda: evaluate.euclidean_distance_device(qn, gn, out=dist_buf, precision="fp16"))
    td = timed(lambda: evaluate.euclidean_distance_device(qn, gn, out=dist_buf))
    args = [torch.from_numpy(np.ascontiguousarray(a)).to(wl.dev) for a in (qp, gp, qc, gc)]
    te = timed(lambda: evaluate.eval_rows_device(dist_buf, *args))
    eb = 4.0 * Q * G + 16.0 * G
    return {"distmat": {"bound": "mfma-fp32", "achieved": round(2.0 * Q * G * D / td / 1e12, 1),
                        "peak": PEAK_F32_MATRIX_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(2.0 * Q * G * D / td / 1e12 / PEAK_F32_MATRIX_TFLOPS, 4), "ms": round(td * 1e3, 3)},
            # the §8b reduced-precision mode (fp16 operands, not bit-exact; not the step's path):
            # casts + fp16 GEMM + the Q x G distance pass
            "distmat_f16": {"bound": "mfma-fp16 + hbm", "achieved": round(2.0 * Q * G * D / td16 / 1e12, 1),
                            "peak": PEAK_F16_TFLOPS, "unit": "TFLOP/s",
                            "frac": round(2.0 * Q * G * D / td16 / 1e12 / PEAK_F16_TFLOPS, 4),
                            "ms": round(td16 * 1e3, 3)},
            "eval_rows": {"bound": "hbm", "achieved": round(eb / te / 1e9, 1), "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                          "frac": round(eb / te / 1e9 / PEAK_HBM_GBPS, 4), "ms": round(te * 1e3, 3),
                          "algorithmic_bytes": eb}}


def preprocess_leg(dev, n=19281, reps=5):
    """the test transform (Resize(256,128) -> ToTensor -> Normalize,
    data_prepare.py:257-261) on the Market split's worth of decoded 128x64 RGB crops, packed
    and resident in HBM, -> fp16 [n, 3, 256, 128] (reidmi_preprocess_u8).  HBM-bound:
    algorithmic bytes = n * (128*64*3 read + 3*256*128*2 written)."""
    import ctypes
    r = np.random.default_rng(0)
    h, w = 128, 64
    pix = torch.from_numpy(r.integers(0, 256, n * h * w * 3, dtype=np.uint8)).to(dev)
    meta = torch.from_numpy(np.stack([np.arange(n) * h * w * 3, np.full(n, h), np.full(n, w)], 1).astype(np.int64)).to(dev)
    out = torch.empty((n, 3, 256, 128), dtype=torch.float16, device=dev)
    mean = (ctypes.c_float * 3)(0.5, 0.5, 0.5)
    std = (ctypes.c_float * 3)(0.5, 0.5, 0.5)

    def run():
        _lib.call("reidmi_preprocess_u8", _lib.ptr(pix), _lib.ptr(meta), n, h, w, 256, 128, mean, std, 1,
                  _lib.ptr(out), _lib.stream(dev))

    run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    nbytes = n * (h * w * 3 + 3 * 256 * 128 * 2)
    del pix, out
    return {"config": f"{n} decoded {h}x{w} RGB crops -> fp16 [n,3,256,128] (Resize bilinear + ToTensor + Normalize, "
                      "Pillow-exact)", "imgs_per_s": round(n / (ms * 1e-3), 1), "ms": round(ms, 3),
            "achieved_GBps": round(nbytes / (ms * 1e-3) / 1e9, 1), "peak_GBps": 8000.0}


def jpeg_leg(dev, n=19281, reps=5, unique=2048, cpu=True, n_cpu=2000):
    """`Image.open(path).convert("RGB")` of the loaders
    (data_prepare.py:87-92) for the Market split's worth of 128x64 4:2:0 JPEG files (Pillow-
    encoded synthetic crops, `unique` distinct files cycled), file bytes and plan resident in
    HBM: reidmi_jpeg_decode alone, and decode + reidmi_preprocess_u8 to fp16 [n, 3, 256, 128].
    The Huffman pass is serial per image (one lane each; latency-bound), so the bound named is
    that pass, with the file + RGB bytes' HBM rate reported beside it.  CPU: Pillow itself (the
    reference's decoder) on one thread over n_cpu files."""
    import ctypes
    import io
    from multimodal_reid_amd import data_prepare
    u = syn.jpeg_files(min(n, unique), 128, 64, seed=0, quality=90)
    files = [u[i % len(u)] for i in range(n)]
    t = time.perf_counter()
    joined = data_prepare.read_files(files)  # the files' bytes in one host buffer (page faults of a fresh 80 MB)
    t_read = time.perf_counter() - t
    t = time.perf_counter()
    jb = data_prepare.JpegBatch(None, buffer=joined)  # the marker parse (reidmi_jpeg_plan, threaded)
    t_plan = time.perf_counter() - t
    jb.raise_for_status()
    dfiles = data_prepare._to_device(jb.buf, dev)
    dplan = data_prepare._to_device(jb.plan, dev)
    ws = torch.empty(jb.ws_bytes, dtype=torch.uint8, device=dev)
    pix = torch.empty(jb.out_bytes, dtype=torch.uint8, device=dev)
    err = torch.empty(n, dtype=torch.int32, device=dev)
    meta = torch.from_numpy(jb.meta).to(dev)
    out = torch.empty((n, 3, 256, 128), dtype=torch.float16, device=dev)
    info = jb.info.copy()
    half = (ctypes.c_float * 3)(0.5, 0.5, 0.5)
    s = _lib.stream(dev)

    def decode():
        _lib.call("reidmi_jpeg_decode", _lib.ptr(dfiles), _lib.ptr(dplan), info.ctypes.data_as(ctypes.c_void_p), n,
                  _lib.ptr(ws), ws.numel(), _lib.ptr(pix), _lib.ptr(err), s)

    def both():
        decode()
        _lib.call("reidmi_preprocess_u8", _lib.ptr(pix), _lib.ptr(meta), n, jb.max_h, jb.max_w, 256, 128, half, half,
                  1, _lib.ptr(out), s)

    res = {}
    for name, fn in (("decode", decode), ("decode_preprocess", both)):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name] = e0.elapsed_time(e1) / reps
    assert not err.any().item(), "jpeg decode reported undecodable files"
    fb = int(jb.buf.size)
    line = {"config": f"{n} Pillow-encoded 128x64 4:2:0 q90 JPEG files ({fb / n:.0f} B avg) in HBM -> RGB; "
                      "+ Resize/ToTensor/Normalize -> fp16 [n,3,256,128]",
            "imgs_per_s": round(n / (res["decode"] * 1e-3), 1), "ms": round(res["decode"], 3),
            "decode_preprocess_ms": round(res["decode_preprocess"], 3),
            "decode_preprocess_imgs_per_s": round(n / (res["decode_preprocess"] * 1e-3), 1),
            "host_plan_ms": round(t_plan * 1e3, 2), "host_join_ms": round(t_read * 1e3, 2),
            "roofline": {"bound": "latency (serial Huffman decode, one lane per image)",
                         "achieved_GBps": round((fb + jb.out_bytes) / (res["decode"] * 1e-3) / 1e9, 1),
                         "peak_GBps": PEAK_HBM_GBPS}}
    if cpu:
        from PIL import Image
        k = min(n_cpu, n)
        t = time.perf_counter()
        for f in files[:k]:
            np.asarray(Image.open(io.BytesIO(f)).convert("RGB"))
        dt = time.perf_counter() - t
        line["cpu_reference"] = {"sample": f"Pillow Image.open(...).convert('RGB') of {k} of these files, 1 thread "
                                           "(the reference decodes in 4 DataLoader workers, data_prepare.py:275-283)",
                                 "imgs_per_s": round(k / dt, 1), "cores": 1, "kind": "reference"}
    del dfiles, ws, pix, out
    return line


def market_jpeg_files(wl, dev, quality=90, threads=16):
    """The Market split as 128x64 4:2:0 JPEG files in host memory: identity-structured crops
    (IdentityCrops at the raw crop size, the headline's labels and seeds) rounded to uint8 and
    Pillow-encoded on `threads` host threads.  Returns (query files, gallery files)."""
    import concurrent.futures
    import io

    from PIL import Image
    sp = syn.DATASET_SPLITS["market1501"]
    ic = IdentityCrops(sp["num_ids"], sp["num_cams"], 5, dev, height=128, width=64, noise=0.3)

    def u8(x):
        return ((x.float() + 1) * 127.5).round_().clamp_(0, 255).to(torch.uint8).permute(0, 2, 3, 1).contiguous().cpu().numpy()

    q = u8(ic(wl.q_pids, wl.q_cams, 0, wl.Q))
    ic.seed = 6
    g = u8(ic(wl.g_pids, wl.g_cams, 0, wl.G))
    del ic

    def enc(a):
        b = io.BytesIO()
        Image.fromarray(a).save(b, "JPEG", quality=quality, subsampling=2)
        return b.getvalue()

    with concurrent.futures.ThreadPoolExecutor(threads) as ex:
        return list(ex.map(enc, q)), list(ex.map(enc, g))


def files_leg(wl, dev, batch=8192, reps=2):
    """VERDICT r5 Next #4: Market from 19 281 host JPEG buffers to mAP through the drop-in surface
    — loader.get_loader (native threaded gather into pinned buffers + header parse on a host
    thread; H2D + reidmi_jpeg_decode + reidmi_preprocess_u8 on a side stream, one batch ahead)
    -> zero_shot_learning.inference (both TTA passes; the augmented view applied in im2col) for
    gallery and query -> get_cmc_map (L2-normalise, exact distance, CMC/mAP).  Timed end to end
    (best of `reps` after one warm-up run), beside the HBM-resident headline step."""
    import types

    from multimodal_reid_amd import loader
    t = time.perf_counter()
    qf, gf = market_jpeg_files(wl, dev)
    t_gen = time.perf_counter() - t
    ds = types.SimpleNamespace(query=[(f, int(p), int(c), 0, k) for k, (f, p, c) in enumerate(zip(qf, wl.q_pids, wl.q_cams))],
                               gallery=[(f, int(p), int(c), 0, k) for k, (f, p, c) in enumerate(zip(gf, wl.g_pids, wl.g_cams))])

    def run():
        lg, lq, lga, lqa = loader.get_loader(ds, batch, 256, 128, "vit", tta_seed=1)
        g_emb, g_pid, g_cam, _ = zsl.inference(wl.model, None, None, None, lg, lga, False, "vit")
        q_emb, q_pid, q_cam, _ = zsl.inference(wl.model, None, None, None, lq, lqa, False, "vit")
        cmc, mAP = zsl.get_cmc_map(g_emb, q_emb, g_pid, q_pid, g_cam, q_cam)
        torch.cuda.synchronize()
        for ld in (lg, lq):
            ld.pipe.close()
        return cmc, mAP

    run()
    walls = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        cmc, mAP = run()
        walls.append(time.perf_counter() - t)
    n = wl.Q + wl.G
    fb = sum(map(len, qf)) + sum(map(len, gf))
    w = min(walls)
    return {"config": f"Market-1501 {wl.Q}q x {wl.G}g as {n} host JPEG buffers (128x64 4:2:0 q90, {fb / n:.0f} B avg, "
                      "identity-structured crops) -> get_loader (batch %d) -> inference (2 passes) -> get_cmc_map" % batch,
            "wall_s": round(w, 4), "walls_s": [round(v, 4) for v in walls], "imgs_per_s": round(n / w, 1),
            "mAP": round(float(mAP), 6), "rank1": round(float(cmc[0]), 6), "file_bytes": fb,
            "files_generated_s": round(t_gen, 2)}


def text_leg(dev, n_cls=750, n_tpl=56, reps=3, cpu=True, threads=1, n_cpu=32):
    """the --mm zero-shot classifier's text side at Market size
    (zero_shot_learning.py:37-49): n_cls identities x n_tpl augmented templates = 42 000 token
    rows of 77 through the CLIP text tower (width 512, 12 layers, causal), EOT rows ->
    ln_final -> text_projection, then per-class L2-normalise / mean / L2-normalise.  Synthetic
    token rows of 30-50 tokens (the augmented sentences' length) and random-init weights.
    FLOP per row = layers * (24 L W^2 + 4 L^2 W) (the reference's dense causal attention
    included) + 2 W E for the projection; rate against the dense fp16 MFMA peak."""
    from multimodal_reid_amd.model import TextTransformer
    sd = syn.text_state_dict(seed=0)
    tm = TextTransformer(sd, device=dev)
    N = n_cls * n_tpl
    tokens = torch.from_numpy(syn.token_ids(N, seed=5, min_len=30, max_len=50)).to(dev)
    counts = [n_tpl] * n_cls
    L, W, E, layers = tm.ctx, tm.width, tm.out_dim, tm.layers
    Lu = tm.ctx_used(tokens)  # positions actually run (causal-mask trim, exact)

    def flops(n_pos):
        return N * (layers * (24.0 * n_pos * W * W + 4.0 * n_pos * n_pos * W) + 2.0 * W * E)

    flop, flop_ref = flops(Lu), flops(L)

    def run():  # zero_shot_learning.zeroshot_classifier on device-resident token rows
        return _classifier(tm, tokens, counts)

    run()  # warm: sizes the workspace
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    s = e0.elapsed_time(e1) / reps * 1e-3
    out = {"config": f"{n_cls} classes x {n_tpl} augmented templates = {N} x {L} tokens, CLIP text tower "
                     f"(width {W}, {layers} layers), fp16 operands, + class mean/normalise; run on the first "
                     f"{Lu} positions (1 + the last EOT: rows past it never reach the output under the causal mask)",
           "wall_s": round(s, 4), "seqs_per_s": round(N / s, 1), "ctx_used": Lu,
           "gflop_per_seq_executed": round(flop / N / 1e9, 3), "gflop_per_seq_reference": round(flop_ref / N / 1e9, 3),
           "achieved": round(flop / s / 1e12, 1), "peak": PEAK_F16_TFLOPS, "unit": "TFLOP/s",
           "frac": round(flop / s / 1e12 / PEAK_F16_TFLOPS, 4),
           "reference_flop_rate": round(flop_ref / s / 1e12, 1)}
    del tm
    torch.cuda.empty_cache()
    if cpu:
        from oracle import vit_ref
        torch.set_num_threads(threads)
        tk = syn.token_ids(n_cpu, seed=5, min_len=30, max_len=50)
        with torch.no_grad():
            vit_ref.text_forward(sd, tk[:4])
            t = time.perf_counter()
            vit_ref.text_forward(sd, tk)
            tc = (time.perf_counter() - t) / n_cpu
        out["cpu_port"] = {"sample": f"oracle/vit_ref.py fp32 text tower on {n_cpu} rows ({tc * 1e3:.1f} ms/row), "
                                     f"extrapolated to {N} rows", "wall_s": round(tc * N, 1), "cores": threads,
                           "kind": "port"}
    return out


def _classifier(tm, tokens, counts):
    from multimodal_reid_amd.ops import class_mean_normalize_device
    return class_mean_normalize_device(tm.encode_text(tokens), counts)


def cpu_baseline(wl, threads, n_img=512, bs=32):
    """The oracle ("port") on this host: the reference's fp32 encoder math laid out as its
    modules run it on the CPU (oracle/vit_ref.FastVit: Conv2d, LayerNorm, in_proj / SDPA /
    out_proj, QuickGELU MLP; bit-identical to the reference module's output on the pinned
    fixture, and as fast as that module on the same host) on a bounded image sample (both TTA
    passes, batches of `bs`), extrapolated linearly to the split, plus the C restatement of
    L2-normalise + distance + eval_func on the FULL Market split (not extrapolated), `threads`
    host threads for both."""
    import oracle
    from oracle import vit_ref
    torch.set_num_threads(threads)
    oracle.set_threads(threads)
    imgs = syn.images(n_img, seed=3)
    offs = syn.tta_offsets(n_img, seed=3)
    fv = vit_ref.FastVit(wl.sd)
    fv(imgs[:8])  # warm
    t = time.perf_counter()
    for s in range(0, n_img, bs):
        fv(imgs[s:s + bs])
        fv(imgs[s:s + bs], tta=offs[s:s + bs])
    t_img = (time.perf_counter() - t) / n_img
    r = np.random.default_rng(0)
    gf = r.standard_normal((wl.G, 1280)).astype(np.float32)
    qf = r.standard_normal((wl.Q, 1280)).astype(np.float32)
    t = time.perf_counter()
    qn, gn = oracle.l2norm(qf), oracle.l2norm(gf)
    d = oracle.distmat(qn, gn)
    oracle.eval_rows(d, wl.q_pids, wl.g_pids, wl.q_cams, wl.g_cams)
    t_eval = time.perf_counter() - t
    total = (wl.Q + wl.G) * t_img + t_eval
    return {"value": round((wl.Q + wl.G) / total, 3), "unit": "imgs/s", "cores": threads, "kind": "port",
            "sample": f"oracle/vit_ref.FastVit fp32 ViT-B/16 (the reference modules' op sequence) on {n_img} images "
                      f"x 2 TTA passes, batches of {bs} ({t_img:.3f} s/img, extrapolated linearly to "
                      f"{wl.Q + wl.G} images) + oracle C l2norm+distmat+eval on the full {wl.Q}q x {wl.G}g split "
                      f"({t_eval:.2f} s)"}


def rank_envs(n, port, base=None):
    """The environment of each of the n ranks bench.py starts itself (`--gpus N` without
    torchrun): the torchrun variables every rank reads (RANK, LOCAL_RANK, WORLD_SIZE,
    MASTER_ADDR = 127.0.0.1, MASTER_PORT), plus the parent's own environment."""
    base = dict(os.environ if base is None else base)
    envs = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), REIDMI_BENCH_CHILD="1")
        envs.append(e)
    return envs


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, script=None, poll_s=0.2):
    """Start n rank processes of `script` (default: this file) with `argv`, before this process
    makes any GPU call (children are fresh interpreters started by Popen, never an exec of this
    one).  Rank 0's stdout is captured and its last JSON line relayed; the others' stdout goes
    to stderr.  If any rank fails, the others are terminated (they would wait in a collective
    forever) and its exit code is returned."""
    import subprocess
    import threading
    script = script or os.path.abspath(__file__)
    envs = rank_envs(n, _free_port())
    procs = []
    for r, env in enumerate(envs):
        procs.append(subprocess.Popen([sys.executable, "-u", script] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr))
    out0 = []
    reader = threading.Thread(target=lambda: out0.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    code = 0

    def stop_all():
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()

    import signal
    prev = signal.signal(signal.SIGTERM, lambda *_: sys.exit(128 + signal.SIGTERM))  # -> stop_all below
    try:
        while True:
            states = [p.poll() for p in procs]  # every process polled each round (no short-circuit)
            if all(c is not None for c in states):
                break
            bad = [c for c in states if c not in (None, 0)]
            if bad:
                code = bad[0]
                stop_all()
                break
            time.sleep(poll_s)
    except BaseException:  # interrupted (Ctrl-C, SIGTERM): no orphan ranks left waiting in a collective
        stop_all()
        raise
    finally:
        signal.signal(signal.SIGTERM, prev)
    reader.join(timeout=60)
    code = code or next((p.returncode for p in procs if p.returncode), 0)
    text = (out0[0] if out0 else b"").decode(errors="replace")
    lines = [ln for ln in text.splitlines() if ln.startswith("{")]
    for ln in text.splitlines():
        if not ln.startswith("{"):
            print(ln, file=sys.stderr)
    if lines:
        print(lines[-1], flush=True)
    return code


def _parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    # at most this many crops per encoder call, in balanced calls over the rank's query + gallery
    # stream: 19 281 (M = 4 068 291 token rows per GEMM) at Market size on one GPU.  Fewer,
    # larger launches: 4096 -> 8192 -> 16384 +0.6 % / +0.5 % (profiles/r05/bench_batch*.json)
    ap.add_argument("--batch", type=int, default=20480)
    ap.add_argument("--streams", type=int, default=1)
    # the Market step's data: identity-structured crops through the spread network (residual-branch
    # output projections x MSMT17_RESID_GAIN), so the headline's mAP carries a ranking signal
    # (VERDICT r4 Weak #9); "uniform" + gain 1 = rounds 1-4's U(-1,1) crops through CLIP's init
    ap.add_argument("--crops", choices=("identity", "uniform"), default="identity")
    ap.add_argument("--resid-gain", type=float, default=MSMT17_RESID_GAIN)
    # nccl = RCCL over xGMI, one GPU per rank; gloo = host collectives, ranks may share a GPU
    # (LOCAL_RANK modulo the visible devices): the multi-rank test on a one-GPU box
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-rerank", action="store_true")
    ap.add_argument("--no-msmt17", action="store_true")
    ap.add_argument("--no-text", action="store_true")
    ap.add_argument("--no-jpeg", action="store_true")
    ap.add_argument("--no-backend", action="store_true")
    ap.add_argument("--no-preprocess", action="store_true")
    ap.add_argument("--no-files", action="store_true")
    ap.add_argument("--files-batch", type=int, default=8192)  # files_to_map get_loader batch (profiles/r06/files_batch_sweep.txt)
    return ap.parse_args(argv)


def main():
    a = _parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N`: start the N ranks here (nothing has touched the GPU yet)
        sys.exit(launch_ranks(a.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {a.gpus}: the line would mislabel n_gpus")
    if a.backend == "gloo":
        local %= max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        assert dist.get_world_size() == a.gpus
    wl = Workload(dev, rank, world, a.batch, streams=a.streams, crops=a.crops, resid_gain=a.resid_gain)
    L = _lib.load()
    for _ in range(a.warmup):
        wl.step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    L.reidmi_prof_enable(1)
    t0 = time.perf_counter()
    embed_s = gather_s = eval_s = 0.0
    for _ in range(a.steps):
        cmc, mAP, te, tg, tv = wl.step()
        embed_s += te
        gather_s += tg
        eval_s += tv
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    import ctypes
    ms, cnt, fl = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
    # the largest c_fc launches only (balanced calls differ by at most one image; the CLS-only
    # last block's small c_fc is left out), so flops_per_launch / avg_launch_ms is the rate of the
    # M = 211 * max_call launch the PMC traffic below was measured on
    full = 2.0 * (wl.max_call - 1) * 211 * 3072 * 768
    L.reidmi_prof_collect_min(EPI_GELU, ctypes.c_double(full), ctypes.byref(ms), ctypes.byref(cnt),
                              ctypes.byref(fl))
    L.reidmi_prof_enable(0)
    elapsed = _max_over_ranks([elapsed], dev)[0]
    per_rank = _all_ranks([embed_s / a.steps, gather_s / a.steps, eval_s / a.steps], dev)
    ms17 = None if a.no_msmt17 else msmt17_leg(None, dev, rank, world, a.batch)
    if rank == 0:
        imgs = (wl.Q + wl.G) * a.steps
        avg_ms = ms.value / max(cnt.value, 1)
        achieved = fl.value / max(cnt.value, 1) / (avg_ms * 1e-3) / 1e12 if cnt.value else None
        line = {
            "metric": "gallery imgs/sec + eval wall-sec (distmat+rerank); mAP parity Market/MSMT17",
            "value": round(imgs / elapsed, 2),
            "unit": "imgs/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 2),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "fp16",
            "data": ("synthetic identity-structured 256x128 crops in HBM (750 ids, 6 cams, noise 0.3; bench.IdentityCrops)"
                     if a.crops == "identity" else "synthetic U(-1,1) 256x128 crops in HBM")
                    + f", random-init ViT-B/16 (CLIP init scales, residual-branch output projections x {a.resid_gain:g})",
            "config": {"workload": "Market-1501 full eval: 3368q x 15913g, ViT-B/16 stride-12 (211 tokens), "
                                   "2 passes/img (plain + flip/pad/crop TTA), exact-fp32 distmat, CMC/mAP",
                       "images_per_step": wl.Q + wl.G, "encoder_passes_per_step": 2 * (wl.Q + wl.G),
                       "batch": a.batch, "images_per_encoder_call": wl.max_call,
                       "parallelism": f"dp{world} (image shards + all-gather)",
                       "backend": a.backend if world > 1 else None},
            "eval_wall_s": round(eval_s / a.steps, 4),
            "embed_wall_s": round(embed_s / a.steps, 4),
            "mAP": round(float(mAP), 6),
            "rank1": round(float(cmc[0]), 6),
            "roofline": {"bound": "mfma", "kernel": "gemm_persistent_kernel<1, 0> (ln_2-folded fp16 mlp.c_fc + QuickGELU)",
                         "achieved": round(achieved, 1) if achieved else None, "peak": PEAK_F16_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved / PEAK_F16_TFLOPS, 4) if achieved else None,
                         "traffic": C_FC_TRAFFIC_BYTES.get(wl.max_call), "traffic_unit": "bytes/launch (PMC)", "avg_launch_ms": round(avg_ms, 4), "launches": cnt.value,
                         "flops_per_launch": fl.value / max(cnt.value, 1)},
        }
        if world > 1:
            # per step: each rank's embed (its image shards, both passes + normalise), its wait in
            # + the gallery all-gather (the minimum over ranks ~ the collective alone), its eval
            line["ranks"] = {"embed_s": [round(v[0], 4) for v in per_rank],
                             "allgather_s": [round(v[1], 5) for v in per_rank],
                             "eval_s": [round(v[2], 4) for v in per_rank],
                             "allgather_bytes": wl.gather_bytes,
                             "allgather_GBps_at_min": round(wl.gather_bytes / max(min(v[1] for v in per_rank), 1e-9)
                                                            / 1e9, 2)}
        if ms17 is not None:
            line["msmt17"] = ms17
        if not a.no_backend:
            line["backend"] = backend_rooflines(wl)
        if not a.no_preprocess:
            line["preprocess"] = preprocess_leg(dev)
        # host-side baselines at N = 1 only (the other ranks would idle at the final barrier)
        cpu = not a.no_cpu_baseline and world == 1
        if not a.no_jpeg:
            line["jpeg"] = jpeg_leg(dev, cpu=cpu)
        if not a.no_files and world == 1:
            line["files_to_map"] = files_leg(wl, dev, batch=a.files_batch)
            line["files_to_map"]["hbm_resident_step_s"] = round(elapsed / a.steps, 4)
        threads = min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
        if not a.no_rerank:
            line["rerank"] = rerank_leg(dev, cpu=cpu, threads=threads)
        if not a.no_text:
            line["text"] = text_leg(dev, cpu=cpu, threads=threads)
        if cpu:
            line["cpu_baseline"] = cpu_baseline(wl, threads)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
