"""Drop-in for the reference's evaluate.py: same names, arguments, return types
and error behaviour, computed by libreidmi HIP kernels on the GPU.

    euclidean_distance(qf, gf) -> np.ndarray          evaluate.py:7-13
    cosine_similarity(qf, gf) -> np.ndarray           evaluate.py:16-26
    eval_func(distmat, q_pids, g_pids, q_camids, g_camids, max_rank=50)
                                   -> (cmc np.float32[max_rank], mAP np.float64)   evaluate.py:29-88
    R1_mAP_eval(num_query, max_rank=50, feat_norm=True, reranking=False)           evaluate.py:91-135

The *_device variants keep everything on the GPU (torch tensors in, torch tensors out)
and are what the fused pipeline (zero_shot_learning.py) uses.

Tie semantics: ranks inside groups of exactly equal distances are ordered by gallery
index (np.argsort(kind="stable")); the reference's unstable argsort orders such groups
in a host-dependent way.
"""
import numpy as np
import torch

from . import _lib


def _dev():
    if not torch.cuda.is_available():
        raise _lib.ReidmiError("no GPU visible: the libreidmi path runs on MI355X only")
    return torch.device("cuda", torch.cuda.current_device())


def _as_dev_f32(x):
    if isinstance(x, np.ndarray):
        x = torch.from_numpy(x)
    return x.to(device=_dev(), dtype=torch.float32).contiguous()


def _as_dev_i64(x):
    if isinstance(x, torch.Tensor):
        return x.to(device=_dev(), dtype=torch.int64).contiguous()
    return torch.from_numpy(np.ascontiguousarray(np.asarray(x), dtype=np.int64)).to(_dev())


# --------------------------------------------------------------------- kernels
def l2_normalize_device(x):
    """torch.nn.functional.normalize(x, dim=1, p=2) (evaluate.py:114) on the GPU."""
    x = _as_dev_f32(x)
    n, d = x.shape
    y = torch.empty_like(x)
    ws = torch.empty(max(n, 1), device=x.device, dtype=torch.float32)
    _lib.call("reidmi_l2norm_f32", _lib.ptr(x), n, d, d, _lib.ptr(y), d, _lib.ptr(ws), _lib.stream())
    return y


def euclidean_distance_device(qf, gf, out=None, precision="fp32"):
    """(Q,G) fp32 tensor: ||q||^2 + ||g||^2 - 2 q.g.  precision "fp32" (default): exact fp32
    (fmaf chain over k), the reference's distances up to BLAS order; "fp16": the q.g products on
    the fp16 MFMA GEMM (reidmi_distmat_f16, the §8b reduced-precision mode; not bit-exact)."""
    if precision not in ("fp32", "fp16"):
        raise ValueError(f"euclidean_distance_device: precision must be 'fp32' or 'fp16', not {precision!r}")
    qf, gf = _as_dev_f32(qf), _as_dev_f32(gf)
    Q, D = qf.shape
    G = gf.shape[0]
    if out is None:
        out = torch.empty((Q, G), device=qf.device, dtype=torch.float32)
    if precision == "fp16":
        nb = _lib.load().reidmi_distmat_f16_workspace_bytes(Q, G, D)
        ws = torch.empty(max(nb, 1), device=qf.device, dtype=torch.uint8)
        _lib.call("reidmi_distmat_f16", _lib.ptr(qf), Q, qf.stride(0), _lib.ptr(gf), G, gf.stride(0), D,
                  _lib.ptr(out), out.stride(0), _lib.ptr(ws), nb, _lib.stream())
        return out
    ws = torch.empty(Q + G, device=qf.device, dtype=torch.float32)
    _lib.call("reidmi_distmat_f32", _lib.ptr(qf), Q, qf.stride(0), _lib.ptr(gf), G, gf.stride(0), D,
              _lib.ptr(out), out.stride(0), _lib.ptr(ws), _lib.stream())
    return out


def topk_rows_device(x, k, row_div=None, with_values=False):
    """np.argsort(x, axis=1, kind='stable')[:, :k] on the GPU (any k <= columns)."""
    x = _as_dev_f32(x)
    rows, cols = x.shape
    idx = torch.empty((rows, k), device=x.device, dtype=torch.int32)
    val = torch.empty((rows, k), device=x.device, dtype=torch.float32) if with_values else None
    _lib.call("reidmi_topk_rows_f32", _lib.ptr(x), rows, cols, x.stride(0), _lib.ptr(row_div), k, _lib.ptr(idx),
              _lib.ptr(val), k, _lib.stream())
    return (idx, val) if with_values else idx


def eval_rows_device(dist, q_pids, g_pids, q_camids, g_camids):
    """Per-query (valid, first_match_rank, AP, n_kept) for eval_func (evaluate.py:40-80), any
    number of positives per query.  (valid = -1 / overflow = 1 were a capacity signal of older
    builds; aggregate_cmc_map still refuses them.)"""
    dist = _as_dev_f32(dist)
    Q, G = dist.shape
    qp, gp, qc, gc = (_as_dev_i64(a) for a in (q_pids, g_pids, q_camids, g_camids))
    dev = dist.device
    valid = torch.empty(Q, device=dev, dtype=torch.int32)
    first = torch.empty(Q, device=dev, dtype=torch.int64)
    ap = torch.empty(Q, device=dev, dtype=torch.float64)
    nkept = torch.empty(Q, device=dev, dtype=torch.int64)
    overflow = torch.empty(1, device=dev, dtype=torch.int32)  # written by the call
    ws = torch.empty(_lib.load().reidmi_eval_rows_workspace_bytes(G), device=dev, dtype=torch.uint8)
    _lib.call("reidmi_eval_rows", _lib.ptr(dist), Q, G, dist.stride(0), _lib.ptr(qp), _lib.ptr(gp), _lib.ptr(qc),
              _lib.ptr(gc), _lib.ptr(valid), _lib.ptr(first), _lib.ptr(ap), _lib.ptr(nkept), _lib.ptr(overflow),
              _lib.ptr(ws), ws.numel(), _lib.stream())
    return valid, first, ap, nkept, overflow


def aggregate_cmc_map(valid, first, ap, nkept, num_g, max_rank=50, overflow=None):
    """evaluate.py:37-39,82-88 on the per-query results, with numpy's exact arithmetic:
    CMC = float32 count / float32 num_valid, mAP = np.mean of the float64 APs in query order."""
    valid = np.asarray(valid)
    if (overflow is not None and int(np.asarray(overflow).reshape(-1)[0])) or \
            (valid.dtype != bool and (valid < 0).any()):
        raise _lib.ReidmiError("eval_rows: a query was not evaluated (overflow flag or valid < 0)")
    valid = valid > 0
    first, ap, nkept = np.asarray(first), np.asarray(ap), np.asarray(nkept)
    if num_g < max_rank:
        max_rank = num_g
        print("Note: number of gallery samples is quite small, got {}".format(num_g))
    num_valid = int(valid.sum())
    assert num_valid > 0, "Error: all query identities do not appear in gallery"
    lens = np.minimum(nkept[valid], max_rank)
    if (lens != lens[0]).any():
        # the reference's np.asarray(all_cmc) on ragged rows (evaluate.py:84)
        raise ValueError("setting an array element with a sequence. The requested array has an "
                         "inhomogeneous shape after 1 dimensions.")
    L = int(lens[0])
    f = first[valid]
    counts = (f[:, None] <= np.arange(L)[None, :]).sum(0)
    cmc = counts.astype(np.float32) / float(num_valid)
    mAP = np.mean(ap[valid])
    return cmc, mAP


# ------------------------------------------------------------ reference surface
def euclidean_distance(qf, gf):
    """evaluate.py:7-13 — returns a numpy float32 (Q,G) matrix."""
    return euclidean_distance_device(qf, gf).cpu().numpy()


def cosine_similarity(qf, gf):
    """evaluate.py:16-26 — arccos of the clipped cosine, numpy float32 (Q,G)."""
    from .ops import cosine_distance_device
    return cosine_distance_device(_as_dev_f32(qf), _as_dev_f32(gf)).cpu().numpy()


def eval_func_device(dist, q_pids, g_pids, q_camids, g_camids, max_rank=50):
    valid, first, ap, nkept, overflow = eval_rows_device(dist, q_pids, g_pids, q_camids, g_camids)
    torch.cuda.current_stream().synchronize()
    return aggregate_cmc_map(valid.cpu().numpy(), first.cpu().numpy(), ap.cpu().numpy(), nkept.cpu().numpy(),
                             dist.shape[1], max_rank, overflow.cpu().numpy())


def eval_func(distmat, q_pids, g_pids, q_camids, g_camids, max_rank=50):
    """evaluate.py:29-88 — Market-1501 CMC/mAP with same-pid-same-camera removal."""
    return eval_func_device(_as_dev_f32(distmat), q_pids, g_pids, q_camids, g_camids, max_rank)


class R1_mAP_eval():
    """evaluate.py:91-135.  Features stay on the GPU (the reference copies them to the CPU).
    As in the reference, ``max_rank`` is stored but compute() scores with eval_func's
    default 50 (evaluate.py:132): the CMC is 50 long whatever max_rank was given.

    ``sharded=True`` (torch.distributed process group, one process per GPU, SURVEY.md §8e;
    the contract: distributed.py): every rank holds ITS shard: its updates are its query rows
    followed by its gallery rows, and ``num_query`` is its own query count.  compute() then
    all-gathers the feature blocks and
    labels (gallery-sharded embed + RCCL all-gather, the north star's exchange step), scores
    the query rows shard(Q, rank, W) against the whole gallery (exact distance, or the
    row-sharded k-reciprocal re-rank), all-gathers the per-query results and reduces them in
    global query order: every rank returns the CMC/mAP of the single-process run over the
    rank-ordered concatenation of the shards, bit for bit (contiguous shards in rank order =
    the single-process order).  Default (``sharded=False``): the reference's single-process
    semantics on this process's data, no collective even under a process group."""

    def __init__(self, num_query, max_rank=50, feat_norm=True, reranking=False, sharded=False):
        super(R1_mAP_eval, self).__init__()
        self.num_query = num_query
        self.max_rank = max_rank
        self.feat_norm = feat_norm
        self.reranking = reranking
        self.sharded = sharded

    def reset(self):
        self.feats = []
        self.pids = []
        self.camids = []

    def update(self, output):  # called once for each batch
        feat, pid, camid = output
        self.feats.append(_as_dev_f32(feat))
        self.pids.extend(np.asarray(pid.cpu() if isinstance(pid, torch.Tensor) else pid))
        self.camids.extend(np.asarray(camid.cpu() if isinstance(camid, torch.Tensor) else camid))

    def compute(self):  # called after each epoch
        from . import distributed as rd
        feats = torch.cat(self.feats, dim=0)
        if self.feat_norm:
            print("The test feature is normalized")
            feats = l2_normalize_device(feats)
        if self.sharded:
            if not rd._initialized():
                raise _lib.ReidmiError("R1_mAP_eval(sharded=True) needs an initialised torch.distributed process group")
            return self._compute_sharded(feats)
        with rd.local():
            return self._compute_local(feats)

    def _compute_local(self, feats):
        qf = feats[:self.num_query]
        q_pids = np.asarray(self.pids[:self.num_query])
        q_camids = np.asarray(self.camids[:self.num_query])
        gf = feats[self.num_query:]
        g_pids = np.asarray(self.pids[self.num_query:])
        g_camids = np.asarray(self.camids[self.num_query:])
        if self.reranking:
            print('=> Enter reranking')
            from .reranking import re_ranking_device
            distmat = re_ranking_device(qf, gf, k1=50, k2=15, lambda_value=0.3)
        else:
            print('=> Computing DistMat with euclidean_distance')
            distmat = euclidean_distance_device(qf, gf)
        cmc, mAP = eval_func_device(distmat, q_pids, g_pids, q_camids, g_camids)
        self._print(cmc, mAP)
        return cmc, mAP

    @staticmethod
    def _print(cmc, mAP):
        print("Rank@{:d}:{:.1%}, Rank@{:d}:{:.1%}, Rank@{:d}:{:.1%}, mAP:{:.1%}".format(
            1, cmc[0], 5, cmc[4], 10, cmc[9], mAP))

    def _compute_sharded(self, feats):
        from . import distributed as rd
        rank, W = rd.world()
        nq = self.num_query
        lab = torch.from_numpy(np.stack([np.asarray(self.pids, np.int64), np.asarray(self.camids, np.int64)], 1))
        qf, _ = rd.gather_rows_var(feats[:nq].contiguous())
        gf, _ = rd.gather_rows_var(feats[nq:].contiguous())
        ql, _ = rd.gather_rows_var(lab[:nq].contiguous())
        gl, _ = rd.gather_rows_var(lab[nq:].contiguous())
        Q, G = qf.shape[0], gf.shape[0]
        qlo, qhi = rd.shard(Q, rank, W)
        if self.reranking:
            print('=> Enter reranking')
            from .reranking import re_ranking_sharded
            d = re_ranking_sharded(qf, gf, 50, 15, 0.3)  # this rank's rows shard(Q, rank, W)
        else:
            print('=> Computing DistMat with euclidean_distance')
            d = euclidean_distance_device(qf[qlo:qhi], gf)
        ql, gl = ql.numpy(), gl.numpy()
        valid, first, ap, nkept, ovf = eval_rows_device(d, ql[qlo:qhi, 0], gl[:, 0], ql[qlo:qhi, 1], gl[:, 1])
        if int(ovf.item()):
            raise _lib.ReidmiError("eval_rows: a query was not evaluated (overflow flag)")
        rows = rd.gather_rows(rd.pack_rows(valid, first, ap, nkept), Q)
        cmc, mAP = aggregate_cmc_map(*rd.unpack_rows(rows), G, 50)
        self._print(cmc, mAP)
        return cmc, mAP
