"""Data-parallel evaluation over one node: one process per GPU, torch.distributed with the
"nccl" backend (= RCCL over xGMI on MI355X); "gloo" for CPU tests.

The reference is single-GPU (no collective call sites).  The one exchange
step this path needs:
  1. rank r embeds its contiguous shard of query and gallery images (no communication);
  2. all-gather of the (L2-normalised) gallery feature blocks — every rank needs the
     whole gallery to rank its queries;
  3. each rank scores its query shard (distmat + eval rows) locally;
  4. all-gather of the per-query results (valid, first-match rank, AP, n_kept: 32 B/query),
     then every rank reduces them in global query order with numpy's own arithmetic, so the
     CMC/mAP are bit-identical for any world size.
Re-ranking (reranking.re_ranking_sharded) shards its rows too: rank r owns rows
shard(N, r, W) of the N = Q + G items for R1-R4 and queries shard(Q, r, W) for R6-R7, with
all-gathers of initial_rank[:, :K], the od divisors, and the CSR rows of V and V_qe between
the stages.

Contract of the drop-in surface under a process group (one place): nothing in
evaluate.py / reranking.py / zero_shot_learning.py issues a collective unless the caller asks
for it with ``sharded=True``.  By default every call has the reference's single-process
semantics on whatever this process passed (a DDP script that evaluates on rank 0 only, or
passes the full split on every rank, gets the single-process result and no hang):
  * R1_mAP_eval(..., sharded=True) / get_cmc_map(..., sharded=True): each rank passes ITS
    shard (its query rows, its gallery rows); every rank returns the CMC/mAP of the whole split.
  * re_ranking_device(..., sharded=True): every rank passes the FULL features; the stages are
    row-sharded over the ranks and every rank returns the whole (Q, G) matrix.
Inside a default (unsharded) call, ``local()`` hides the process group from these helpers.
"""
import contextlib
import threading

import numpy as np
import torch
import torch.distributed as dist

_tls = threading.local()


@contextlib.contextmanager
def local():
    """Run the enclosed calls as one process: world() = (0, 1), no collectives."""
    prev = getattr(_tls, "local", False)
    _tls.local = True
    try:
        yield
    finally:
        _tls.local = prev


def world():
    if _initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def _initialized():
    return not getattr(_tls, "local", False) and dist.is_available() and dist.is_initialized()


def shard(n, rank, world_size):
    """Contiguous [lo, hi) slice of n items for `rank` (sizes differ by at most one)."""
    return n * rank // world_size, n * (rank + 1) // world_size


def gather_rows(x, n_total):
    """All-gather row shards produced by `shard(n_total, r, W)` into one [n_total, ...] tensor
    (same device as x).  RCCL path: one padded all_gather_into_tensor (also run at world
    size 1 when a process group exists, so a 1-GPU box exercises the RCCL path)."""
    rank, W = world()
    if not _initialized():
        return x
    sizes = [shard(n_total, r, W)[1] - shard(n_total, r, W)[0] for r in range(W)]
    mx = max(sizes)
    dev = _collective_device(x)
    pad = torch.zeros((mx,) + tuple(x.shape[1:]), device=dev, dtype=x.dtype)
    pad[:x.shape[0]] = x.to(dev)
    if dist.get_backend() == "nccl":
        out = torch.empty((W * mx,) + tuple(x.shape[1:]), device=dev, dtype=x.dtype)
        dist.all_gather_into_tensor(out, pad)
        parts = [out[r * mx:r * mx + sizes[r]] for r in range(W)]
    else:
        bufs = [torch.empty_like(pad) for _ in range(W)]
        dist.all_gather(bufs, pad)
        parts = [bufs[r][:sizes[r]] for r in range(W)]
    return torch.cat(parts).to(x.device)


def _collective_device(x):
    """gloo moves host tensors: device tensors are staged through the host for it."""
    return x.device if dist.get_backend() == "nccl" else torch.device("cpu")


def gather_var(x):
    """All-gather 1-D pieces of different lengths; returns their concatenation in rank order
    (same device as x).  Used for the CSR payloads of the sharded re-ranking."""
    rank, W = world()
    if not _initialized():
        return x
    dev = _collective_device(x)
    dtype = x.dtype
    x = x.contiguous().view(torch.uint8)  # moved as bytes (gloo has no int16)
    n = torch.tensor([x.numel()], dtype=torch.int64, device=dev)
    ns = [torch.empty_like(n) for _ in range(W)]
    dist.all_gather(ns, n)
    ns = [int(v.item()) for v in ns]
    mx = max(max(ns), 1)
    pad = torch.zeros(mx, dtype=x.dtype, device=dev)
    pad[:x.numel()] = x.to(dev)
    bufs = [torch.empty_like(pad) for _ in range(W)]
    dist.all_gather(bufs, pad)
    return torch.cat([bufs[r][:ns[r]] for r in range(W)]).to(x.device).view(dtype)


def gather_rows_var(x):
    """All-gather row blocks of different lengths ([n_r, ...] on rank r); returns (their
    concatenation in rank order on x's device, [n_0, ..., n_{W-1}]).  The drop-in surface
    (evaluate.R1_mAP_eval, zero_shot_learning.get_cmc_map) uses it for whatever shards the
    caller's loaders produced."""
    rank, W = world()
    if not _initialized():
        return x, [x.shape[0]]
    dev = _collective_device(x)
    n = torch.tensor([x.shape[0]], dtype=torch.int64, device=dev)
    ns = [torch.empty_like(n) for _ in range(W)]
    dist.all_gather(ns, n)
    ns = [int(v.item()) for v in ns]
    mx = max(max(ns), 1)
    pad = torch.zeros((mx,) + tuple(x.shape[1:]), dtype=x.dtype, device=dev)
    pad[:x.shape[0]] = x.to(dev)
    if dist.get_backend() == "nccl":
        out = torch.empty((W * mx,) + tuple(x.shape[1:]), device=dev, dtype=x.dtype)
        dist.all_gather_into_tensor(out, pad)
        parts = [out[r * mx:r * mx + ns[r]] for r in range(W)]
    else:
        bufs = [torch.empty_like(pad) for _ in range(W)]
        dist.all_gather(bufs, pad)
        parts = [bufs[r][:ns[r]] for r in range(W)]
    return torch.cat(parts).to(x.device), ns


def all_to_all_var(send, in_splits):
    """Variable-size all-to-all of a 1-D tensor: rank r sends send[off_q : off_q + in_splits[q]]
    to rank q; returns (the received pieces concatenated in source-rank order, their sizes), on
    send's device.  RCCL moves device tensors (all_to_all_single), gloo host tensors."""
    rank, W = world()
    if not _initialized():
        return send, list(in_splits)
    dev = _collective_device(send)
    sizes = torch.tensor([int(v) for v in in_splits], dtype=torch.int64, device=dev)
    got = torch.empty_like(sizes)
    dist.all_to_all_single(got, sizes)
    out_splits = [int(v) for v in got.cpu()]
    recv = torch.empty(sum(out_splits), dtype=send.dtype, device=dev)
    dist.all_to_all_single(recv, send.contiguous().to(dev), out_splits, [int(v) for v in in_splits])
    return recv.to(send.device), out_splits


def pack_rows(valid, first, ap, nkept):
    """Per-query results as one float64 [Q_local, 4] block (indices < 2^53 are exact)."""
    return torch.stack([torch.as_tensor(valid).double(), torch.as_tensor(first).double(),
                        torch.as_tensor(ap).double(), torch.as_tensor(nkept).double()], 1)


def unpack_rows(rows):
    rows = rows.cpu().numpy() if isinstance(rows, torch.Tensor) else rows
    # valid keeps its sign: -1 = a query beyond eval_rows' capacity (aggregate_cmc_map raises)
    return rows[:, 0].astype(np.int64), rows[:, 1].astype(np.int64), rows[:, 2], rows[:, 3].astype(np.int64)


def sharded_eval(q_feat, g_feat, q_pids, g_pids, q_camids, g_camids, num_query, num_gallery, rows_fn, max_rank=50,
                 aggregate=None):
    """Steps 2-4 above.  q_feat / g_feat: this rank's normalised shards; pids/cams: full
    arrays; rows_fn(q, g, qp, gp, qc, gc) -> (valid, first, ap, nkept) computes this rank's
    query rows (libreidmi kernels in the product).  Returns (cmc, mAP) on every rank."""
    from .evaluate import aggregate_cmc_map
    rank, W = world()
    g_all = gather_rows(g_feat, num_gallery)
    qlo, qhi = shard(num_query, rank, W)
    v, f, a, n = rows_fn(q_feat, g_all, q_pids[qlo:qhi], g_pids, q_camids[qlo:qhi], g_camids)
    rows = pack_rows(v, f, a, n).to(g_feat.device)
    rows = gather_rows(rows, num_query)
    agg = aggregate or aggregate_cmc_map
    return agg(*unpack_rows(rows), num_gallery, max_rank)
