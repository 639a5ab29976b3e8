"""Drop-in for the reference's reranking.py:

    re_ranking(probFea, galFea, k1, k2, lambda_value, local_distmat=None, only_local=False)
        -> np.ndarray float32 (num_query, num_gallery)                  reranking.py:29-100

k-reciprocal encoding + Jaccard re-ranking (Zhong et al., CVPR'17) on the GPU through
libreidmi (rerank.hip).  Given the same original distances it reproduces the reference's
numpy arithmetic bit for bit (float32 exp/pairwise sums, float16 V / Jaccard), with ties in
the initial ranking ordered by index (np.argsort(kind="stable")).  The reference's dense
N x N float16 V / V_qe become sparse row lists, so MSMT17-size galleries fit.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from .evaluate import _as_dev_f32, euclidean_distance_device

STAGED_MIN_N = 32768  # from features, N >= this: staged path (no N x N fp32 buffer)
_CAP_MSG = {1: "V row capacity", 2: "V_qe row capacity (4096)", 4: "query-expansion staging capacity (6144)"}


def _lam(lambda_value):
    return int(np.float16(1 - lambda_value).view(np.uint16)), float(np.float32(lambda_value))


def _check(flags):
    f = int(flags.item())
    if f:
        raise _lib.ReidmiError("re_ranking: " + ", ".join(m for b, m in _CAP_MSG.items() if f & b) + " exceeded")


def re_ranking_device(probFea, galFea, k1, k2, lambda_value, local_distmat=None, only_local=False):
    """Device version: returns the (Q, G) fp32 torch tensor on the GPU."""
    Q = probFea.size(0) if isinstance(probFea, torch.Tensor) else len(probFea)
    G = galFea.size(0) if isinstance(galFea, torch.Tensor) else len(galFea)
    if not (only_local or local_distmat is not None) and Q + G >= STAGED_MIN_N:
        # N x N buffers would dominate: row-chunked stages, same bits
        from . import distributed as rd
        if rd.world()[1] > 1:
            raise _lib.ReidmiError("re_ranking_device is single-process; use re_ranking_sharded under torch.distributed")
        return re_ranking_sharded(probFea, galFea, k1, k2, lambda_value)
    dev = torch.device("cuda", torch.cuda.current_device())
    lam_h, lam_f = _lam(lambda_value)
    out = torch.empty((Q, G), device=dev, dtype=torch.float32)
    flags = torch.zeros(1, device=dev, dtype=torch.int32)
    L = _lib.load()
    st = _lib.stream()
    if only_local or local_distmat is not None:
        if only_local:
            D = _as_dev_f32(local_distmat)
            add = None
        else:
            feat = torch.cat([_as_dev_f32(probFea), _as_dev_f32(galFea)])
            D = euclidean_distance_device(feat, feat)
            add = _as_dev_f32(local_distmat)
        nbytes = L.reidmi_rerank_workspace_bytes(Q, G, k1, k2, 1, 1)
        ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)
        _lib.call("reidmi_rerank_from_dist", _lib.ptr(D), _lib.ptr(add), Q, G, 0, k1, k2, lam_h, lam_f,
                  _lib.ptr(out), G, _lib.ptr(ws), nbytes, _lib.ptr(flags), st)
    else:
        feat = torch.cat([_as_dev_f32(probFea), _as_dev_f32(galFea)]).contiguous()
        nbytes = L.reidmi_rerank_workspace_bytes(Q, G, k1, k2, 0, 0)
        ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)
        _lib.call("reidmi_rerank", _lib.ptr(feat), Q, G, feat.shape[1], feat.stride(0), k1, k2, lam_h, lam_f,
                  _lib.ptr(out), G, _lib.ptr(ws), nbytes, _lib.ptr(flags), st)
    _check(flags)
    return out


def re_ranking(probFea, galFea, k1, k2, lambda_value, local_distmat=None, only_local=False):
    """reranking.py:29-100 — returns the re-ranked (Q, G) distance as np.float32."""
    return re_ranking_device(probFea, galFea, k1, k2, lambda_value, local_distmat, only_local).cpu().numpy()


# ------------------------------------------------------------------ staged / sharded
# R1-R7 as row-range stages (reidmi_rr_*): the N x N distance is never materialised (row
# chunks of it are), intermediate rows are exactly sized CSR, and every stage takes a row
# range so the work shards over ranks.  Bit-identical to re_ranking_device.

# R2 (initial_rank) of the staged path through the fp16 pre-filter (reidmi_rr_rank_rows_f16):
# the same bits as the exact rows, ~5x fewer distance FLOPs in fp32.  False = exact rows only.
RANK_PREFILTER = True


class HipStages:
    """The product's stage kernels (libreidmi)."""

    def __init__(self, feat, num_query, k1, k2, lambda_value, chunk_bytes=16 << 30):
        _lib.require_cuda(feat)
        self.feat = _as_dev_f32(feat).contiguous()
        self.N, self.D = self.feat.shape
        self.Q = num_query
        self.k1, self.k2 = k1, k2
        self.K = min(max(k1 + 1, k2), self.N)
        self.lam_h, self.lam_f = _lam(lambda_value)
        self.dev = self.feat.device
        self.st = _lib.stream()
        self.sqn = torch.empty(self.N, device=self.dev, dtype=torch.float32)
        _lib.call("reidmi_row_sqnorm_f32", _lib.ptr(self.feat), self.N, self.D, self.D, _lib.ptr(self.sqn), self.st)
        # distance rows per pass: whole 128-row tiles of the distance kernel when possible (a
        # ragged last tile of every pass costs up to a tile's FLOPs per pass at 1M items)
        rows = int(max(1, min(65535, chunk_bytes // (4 * self.N))))
        self.chunk_rows = rows // 128 * 128 if rows >= 128 else rows
        self._chunk = None
        self._f16 = None
        self.flags = torch.zeros(1, device=self.dev, dtype=torch.int32)
        vc, qc = ctypes.c_int(), ctypes.c_int()
        _lib.call("reidmi_rr_caps", ctypes.byref(vc), ctypes.byref(qc))
        self.vcap, self.qcap = vc.value, qc.value

    def _chunk_buf(self, rows, cols):
        n = rows * cols
        if self._chunk is None or self._chunk.numel() < n:
            self._chunk = torch.empty(n, device=self.dev, dtype=torch.float32)
        return self._chunk

    def _feat16(self):
        """fp16 copy of the features for the rank_rows pre-filter ([Np][Dp] zero-padded), sqrt
        of the squared norms, and whether the features fit fp16 (one host sync per call)."""
        if self._f16 is None:
            Np, Dp = -(-self.N // 256) * 256, -(-self.D // 64) * 64
            x16 = torch.empty(Np * Dp, device=self.dev, dtype=torch.float16)
            ok = torch.ones(1, device=self.dev, dtype=torch.int32)
            _lib.call("reidmi_rr_feat16", _lib.ptr(self.feat), self.N, self.D, self.D, _lib.ptr(x16), Np, Dp,
                      _lib.ptr(ok), self.st)
            self._f16 = (x16, Np, Dp, torch.sqrt(self.sqn), bool(ok.item()))
        return self._f16

    def _exact_rows(self, lo, idx, R, rmax):
        """R2 of rows lo + idx with the exact distance kernel: the same distance bits as
        reidmi_rr_rank_rows (per-pair fp32 chain, same squared norms), row max, stable top-K of
        D / rowmax (reidmi_topk_rows_f32, as rr_rank_rows)."""
        n = int(idx.numel())
        if n == 0:
            return
        step = max(1, self.chunk_rows)
        for s in range(0, n, step):
            sub = idx[s:s + step]
            rows = self.feat[lo + sub].contiguous()
            # the row-pass scratch (stream-ordered after the pass that marked these rows)
            d = self._chunk_buf(rows.shape[0], self.N)[:rows.shape[0] * self.N].view(rows.shape[0], self.N)
            ws = torch.empty(rows.shape[0] + self.N, device=self.dev, dtype=torch.float32)
            _lib.call("reidmi_distmat_f32", _lib.ptr(rows), rows.shape[0], self.D, _lib.ptr(self.feat), self.N,
                      self.D, self.D, _lib.ptr(d), self.N, _lib.ptr(ws), self.st)
            # rowmax_kernel's fmaxf reduction: NaN entries are skipped
            m = torch.where(torch.isnan(d), float("-inf"), d).max(dim=1).values.contiguous()
            k = torch.empty((rows.shape[0], self.K), device=self.dev, dtype=torch.int32)
            _lib.call("reidmi_topk_rows_f32", _lib.ptr(d), rows.shape[0], self.N, self.N, _lib.ptr(m), self.K,
                      _lib.ptr(k), None, self.K, self.st)
            R[sub] = k
            rmax[sub] = m

    def rank_rows(self, lo, hi):
        R = torch.empty((hi - lo, self.K), device=self.dev, dtype=torch.int32)
        rmax = torch.empty(hi - lo, device=self.dev, dtype=torch.float32)
        if hi > lo:
            x16, Np, Dp, nrm, fits = self._feat16() if RANK_PREFILTER else (None, 0, 0, None, False)
            a = lo
            if fits:
                # the fp16 pre-filter (bit-identical to the exact rows; reidmi_rr_rank_rows_f16),
                # one row pass at a time: rows it cannot decide (distances too concentrated
                # for its bound) go through the exact rows, and once a pass has more of those
                # than not (a random network's embeddings) the rest skips the filter
                cr = min(max(256, self.chunk_rows * self.N // Np // 256 * 256), hi - lo)
                need = torch.empty(cr, device=self.dev, dtype=torch.int32)
                first = True
                while a < hi:
                    b = min(a + (min(cr, 512) if first else cr), hi)  # a small probe pass first
                    first = False
                    _lib.call("reidmi_rr_rank_rows_f16", _lib.ptr(self.feat), self.N, self.D, self.D,
                              _lib.ptr(self.sqn), _lib.ptr(nrm), _lib.ptr(x16), Np, Dp, a, b, self.K,
                              _lib.ptr(R[a - lo:]), _lib.ptr(rmax[a - lo:]), _lib.ptr(need),
                              _lib.ptr(self._chunk_buf(cr, Np)), cr, self.st)
                    idx = torch.nonzero(need[:b - a]).flatten()
                    self._exact_rows(a, idx, R[a - lo:b - lo], rmax[a - lo:b - lo])
                    undecided, rows = int(idx.numel()), b - a
                    a = b
                    if 2 * undecided > rows:
                        break
            if a < hi:
                cr = min(self.chunk_rows, hi - a)
                _lib.call("reidmi_rr_rank_rows", _lib.ptr(self.feat), self.N, self.D, self.D, _lib.ptr(self.sqn), a,
                          hi, self.K, _lib.ptr(R[a - lo:]), _lib.ptr(rmax[a - lo:]),
                          _lib.ptr(self._chunk_buf(cr, self.N)), cr, self.st)
        return R, rmax

    def offsets(self, nnz):
        off = torch.empty(nnz.numel() + 1, device=self.dev, dtype=torch.int64)
        _lib.call("reidmi_rr_row_offsets", _lib.ptr(nnz), nnz.numel(), _lib.ptr(off), self.st)
        return off

    def _pack(self, ecol, eval_, nnz, cap):
        off = self.offsets(nnz)
        total = int(off[-1].item())
        col = torch.empty(max(total, 1), device=self.dev, dtype=torch.int32)
        val = torch.empty(max(total, 1), device=self.dev, dtype=torch.int16)
        _lib.call("reidmi_rr_pack", _lib.ptr(ecol), _lib.ptr(eval_), _lib.ptr(nnz), nnz.numel(), cap, _lib.ptr(off),
                  _lib.ptr(col), _lib.ptr(val), self.st)
        return nnz, col[:total], val[:total]

    def v_rows(self, R, rmax, lo, hi):
        n = hi - lo
        ecol = torch.empty((max(n, 1), self.vcap), device=self.dev, dtype=torch.int32)
        evl = torch.empty((max(n, 1), self.vcap), device=self.dev, dtype=torch.int16)
        nnz = torch.zeros(n, device=self.dev, dtype=torch.int32)
        _lib.call("reidmi_rr_v_rows", _lib.ptr(self.feat), self.N, self.D, self.D, _lib.ptr(self.sqn), _lib.ptr(rmax),
                  _lib.ptr(R), self.K, lo, hi, self.k1, _lib.ptr(ecol), _lib.ptr(evl), _lib.ptr(nnz),
                  _lib.ptr(self.flags), self.st)
        return self._pack(ecol, evl, nnz, self.vcap)

    def qe_rows(self, R, V, lo, hi):
        off, col, val = V
        n = hi - lo
        ecol = torch.empty((max(n, 1), self.qcap), device=self.dev, dtype=torch.int32)
        evl = torch.empty((max(n, 1), self.qcap), device=self.dev, dtype=torch.int16)
        nnz = torch.zeros(n, device=self.dev, dtype=torch.int32)
        _lib.call("reidmi_rr_qe_rows", _lib.ptr(R), self.K, self.k2, lo, hi, _lib.ptr(off), _lib.ptr(col),
                  _lib.ptr(val), _lib.ptr(ecol), _lib.ptr(evl), _lib.ptr(nnz), _lib.ptr(self.flags), self.st)
        return self._pack(ecol, evl, nnz, self.qcap)

    def jaccard_rows(self, rmax, Vq, qlo, qhi):
        off, col, val = Vq
        N, Q = self.N, self.Q
        G = N - Q
        nnz = int(off[-1].item())
        L = _lib.load()
        wsb = L.reidmi_rr_csc_workspace_bytes(N, nnz)
        ws = torch.empty(max(wsb, 1), device=self.dev, dtype=torch.uint8)
        coff = torch.empty(N + 1, device=self.dev, dtype=torch.int64)
        irow = torch.empty(max(nnz, 1), device=self.dev, dtype=torch.int32)
        ival = torch.empty(max(nnz, 1), device=self.dev, dtype=torch.int16)
        _lib.call("reidmi_rr_csc", N, _lib.ptr(off), _lib.ptr(col), _lib.ptr(val), nnz, _lib.ptr(coff), _lib.ptr(irow),
                  _lib.ptr(ival), _lib.ptr(ws), wsb, self.st)
        del ws
        out = torch.empty((qhi - qlo, G), device=self.dev, dtype=torch.float32)
        if qhi > qlo and G > 0:
            # distance rows per pass + the rows the call keeps for its column chunk bounds
            extra = int(_lib.load().reidmi_rr_jaccard_reserved_rows(N, G))
            cr = int(max(1, min(65535 - extra, qhi - qlo, self.chunk_rows * N // max(G, 1)))) + extra
            _lib.call("reidmi_rr_jaccard_rows", _lib.ptr(self.feat), N, self.D, self.D, _lib.ptr(self.sqn),
                      _lib.ptr(rmax), Q, qlo, qhi, _lib.ptr(off), _lib.ptr(col), _lib.ptr(val), _lib.ptr(coff),
                      _lib.ptr(irow), _lib.ptr(ival), self.lam_h, self.lam_f, _lib.ptr(out), G,
                      _lib.ptr(self._chunk_buf(cr, G)), cr, self.st)
        return out

    def check(self):
        _check(self.flags)


def _gather_csr(stages, nnz_loc, col_loc, val_loc, N):
    from . import distributed as rd
    nnz = rd.gather_rows(nnz_loc, N)
    col = rd.gather_var(col_loc)
    val = rd.gather_var(val_loc)
    return stages.offsets(nnz), col, val


def staged_rerank(stages, N, Q):
    """R1-R7 over this rank's rows (torch.distributed world; world 1 = the whole job).
    Returns this rank's rows shard(Q, rank, W) of the final (Q, G) distance."""
    from . import distributed as rd
    rank, W = rd.world()
    lo, hi = rd.shard(N, rank, W)
    R_loc, rmax_loc = stages.rank_rows(lo, hi)                    # R1 + R2 (reranking.py:36-48)
    R = rd.gather_rows(R_loc, N)
    rmax = rd.gather_rows(rmax_loc, N)
    V = _gather_csr(stages, *stages.v_rows(R, rmax, lo, hi), N)  # R3 (reranking.py:51-71)
    if stages.k2 != 1:
        Vq = _gather_csr(stages, *stages.qe_rows(R, V, lo, hi), N)  # R4 (reranking.py:73-78)
    else:
        Vq = V
    qlo, qhi = rd.shard(Q, rank, W)
    out = stages.jaccard_rows(rmax, Vq, qlo, qhi)                 # R5-R7 (reranking.py:80-100)
    stages.check()
    return out


def re_ranking_sharded(probFea, galFea, k1, k2, lambda_value, chunk_bytes=16 << 30):
    """Sharded re_ranking: probFea / galFea are the FULL query and gallery features on this
    rank's GPU (all-gathered after a sharded embed).  Returns this rank's query rows
    shard(Q, rank, W) of the re-ranked (Q, G) distance as a device tensor; with one process
    it equals re_ranking_device bit for bit, without the N x N buffers."""
    Q = probFea.size(0)
    feat = torch.cat([_as_dev_f32(probFea), _as_dev_f32(galFea)]).contiguous()
    stages = HipStages(feat, Q, k1, k2, lambda_value, chunk_bytes)
    return staged_rerank(stages, feat.shape[0], Q)
