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

STAGED_MIN_N = 16384  # from features, N >= this: staged path (no N x N fp32 buffer; faster from ~16k: Duke 16 vs 19 ms)
# There is no capacity limit (any k1, k2, neighbourhood density): the flag can only report a
# row beyond a scratch bound computed from the same caps (a bug), never a data-dependent overflow.
_CAP_MSG = {8: "a row beyond its sized scratch (internal error)"}


def _lam(lambda_value):
    return int(np.float16(1 - lambda_value).view(np.uint16)), float(np.float32(lambda_value))


def _check(flags):
    f = int(flags.item())
    if f:
        raise _lib.ReidmiError("re_ranking: " + ", ".join(m for b, m in _CAP_MSG.items() if f & b) + " exceeded")


def re_ranking_device(probFea, galFea, k1, k2, lambda_value, local_distmat=None, only_local=False, sharded=False):
    """Device version: returns the (Q, G) fp32 torch tensor on the GPU.  ``sharded=True``
    (torch.distributed process group, every rank holding the FULL features): the stages are
    row-sharded over the ranks and the final rows all-gathered, so every rank returns the whole
    matrix.  Default: this process alone, no collective (distributed.py states the contract)."""
    from . import distributed as rd
    if sharded:
        if not rd._initialized():
            raise _lib.ReidmiError("re_ranking_device(sharded=True) needs an initialised torch.distributed process group")
        if only_local or local_distmat is not None:
            raise _lib.ReidmiError("re_ranking_device(sharded=True) re-ranks from features only")
        Q = probFea.size(0) if isinstance(probFea, torch.Tensor) else len(probFea)
        return rd.gather_rows(re_ranking_sharded(probFea, galFea, k1, k2, lambda_value), Q)
    with rd.local():
        return _re_ranking_local(probFea, galFea, k1, k2, lambda_value, local_distmat, only_local)


def _re_ranking_local(probFea, galFea, k1, k2, lambda_value, local_distmat, only_local):
    Q = probFea.size(0) if isinstance(probFea, torch.Tensor) else len(probFea)
    G = galFea.size(0) if isinstance(galFea, torch.Tensor) else len(galFea)
    if not (only_local or local_distmat is not None) and Q + G >= STAGED_MIN_N:
        # N x N buffers would dominate: row-chunked stages, same bits
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


def default_chunk_bytes(dev):
    """Distance scratch per row pass: 16 GiB (whole 128-row tiles at 1M items, and enough rows
    for the selection kernels to fill the GPU), but at most a quarter of the free device memory."""
    free, _ = torch.cuda.mem_get_info(dev)
    return int(max(64 << 20, min(16 << 30, free // 4)))


class HipStages:
    """The product's stage kernels (libreidmi)."""

    def __init__(self, feat, num_query, k1, k2, lambda_value, chunk_bytes=None):
        _lib.require_cuda(feat)
        self.feat = _as_dev_f32(feat).contiguous()
        self.N, self.D = self.feat.shape
        self.Q = num_query
        self.k1, self.k2 = k1, k2
        self.K = min(max(k1 + 1, k2), self.N)
        self.lam_h, self.lam_f = _lam(lambda_value)
        self.dev = self.feat.device
        self.st = _lib.stream()
        if chunk_bytes is None:
            chunk_bytes = default_chunk_bytes(self.dev)
        self.sqn = torch.empty(self.N, device=self.dev, dtype=torch.float32)
        _lib.call("reidmi_row_sqnorm_f32", _lib.ptr(self.feat), self.N, self.D, self.D, _lib.ptr(self.sqn), self.st)
        # distance rows per pass: whole 128-row tiles of the distance kernel when possible (a
        # ragged last tile of every pass costs up to a tile's FLOPs per pass at 1M items)
        rows = int(max(1, min(65535, chunk_bytes // (4 * self.N))))
        self.chunk_rows = rows // 128 * 128 if rows >= 128 else rows
        self._chunk = None
        self._f16 = None
        self.flags = torch.zeros(1, device=self.dev, dtype=torch.int32)
        vc, qc, vw, qw = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        _lib.call("reidmi_rr_caps", self.N, k1, k2, ctypes.byref(vc), ctypes.byref(qc), ctypes.byref(vw),
                  ctypes.byref(qw))
        self.vcap, self.qcap = vc.value, qc.value          # ELL widths of V and of on-chip V_qe rows
        self.v_ws_bytes, self.qe_ws_bytes = vw.value, qw.value  # scratch of the generic R3 / R4 kernels
        self.k2e = min(k2, self.K)  # initial_rank[i, :k2] has min(k2, N) entries
        # ELL batches of R3 / R4 rows: at most this many bytes of ELL at once (the CSR parts of
        # the batches are concatenated)
        self.ell_bytes = max(256 << 20, chunk_bytes // 2)
        self._ws = {}
        self.stats = {"rows": 0, "exact_rows": 0, "form": None, "exact_idx": []}

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
            nrm = torch.sqrt(self.sqn)
            nmax2 = torch.empty(2, device=self.dev, dtype=torch.float32)
            _lib.call("reidmi_rr_norm_max", _lib.ptr(self.sqn), _lib.ptr(nrm), self.N, _lib.ptr(nmax2), self.st)
            self._f16 = (x16, Np, Dp, nrm, bool(ok.item()), nmax2)
        return self._f16

    def _exact_rows(self, lo, idx, n, R, rmax):
        """R2 of rows lo + idx[:n] (idx: device int32, from reidmi_nonzero_i32) with the exact
        distance kernel: the same distance bits as reidmi_rr_rank_rows (per-pair fp32 chain,
        same squared norms), row max (reidmi_rowmax_f32: fmaxf, NaN skipped, as rowmax_kernel),
        stable top-K of D / rowmax (reidmi_topk_rows_f32, as rr_rank_rows)."""
        if n == 0:
            return
        step = max(1, self.chunk_rows)
        for s in range(0, n, step):
            m = min(step, n - s)
            sub = idx[s:s + m]
            rows = torch.empty((m, self.D), device=self.dev, dtype=torch.float32)
            _lib.call("reidmi_gather_rows_f32", _lib.ptr(self.feat), self.D, self.D, lo, _lib.ptr(sub), m,
                      _lib.ptr(rows), self.D, self.st)
            # the row-pass scratch (stream-ordered after the pass that marked these rows)
            d = self._chunk_buf(m, self.N)[:m * self.N].view(m, self.N)
            ws = torch.empty(m + self.N, device=self.dev, dtype=torch.float32)
            _lib.call("reidmi_distmat_f32", _lib.ptr(rows), m, self.D, _lib.ptr(self.feat), self.N,
                      self.D, self.D, _lib.ptr(d), self.N, _lib.ptr(ws), self.st)
            mx = torch.empty(m, device=self.dev, dtype=torch.float32)
            _lib.call("reidmi_rowmax_f32", _lib.ptr(d), m, self.N, self.N, _lib.ptr(mx), self.st)
            k = torch.empty((m, self.K), device=self.dev, dtype=torch.int32)
            _lib.call("reidmi_topk_rows_f32", _lib.ptr(d), m, self.N, self.N, _lib.ptr(mx), self.K,
                      _lib.ptr(k), None, self.K, self.st)
            pos = sub.long()
            R.index_copy_(0, pos, k)
            rmax.index_copy_(0, pos, mx)

    def rank_rows(self, lo, hi):
        R = torch.empty((hi - lo, self.K), device=self.dev, dtype=torch.int32)
        rmax = torch.empty(hi - lo, device=self.dev, dtype=torch.float32)
        if hi > lo:
            # the pre-filter's selection keeps K <= 64 on chip; larger K take the exact rows
            use = RANK_PREFILTER and self.K <= 64
            x16, Np, Dp, nrm, fits, nmax2 = self._feat16() if use else (None, 0, 0, None, False, None)
            a = lo
            if fits:
                # the fp16 pre-filter (bit-identical to the exact rows; reidmi_rr_rank_rows_f16),
                # one row pass at a time: rows it cannot decide (distances too concentrated
                # for its bound) go through the exact rows, and once a pass has more of those
                # than not (a random network's embeddings) the rest skips the filter
                cc = min(max(256, self.chunk_rows * self.N // Np // 256 * 256),  # chunk rows of Np floats
                         (hi - lo + 255) // 256 * 256)
                # rows per call: one internal pass (the in-epilogue selection holds ~0.3 MB per
                # row at N = 1M instead of 4 Np bytes, so a pass takes many more rows); N: the
                # whole problem in one call (the symmetric product's upper triangle, each pair
                # tested for both its rows), after the probe pass
                cr = int(_lib.load().reidmi_rr_rank_rows_f16_pass_rows(self.N, Np, cc, self.K, -1))
                tri = cr >= self.N and lo == 0 and hi == self.N
                cr = min(cr, hi - lo)
                need = torch.empty(cr, device=self.dev, dtype=torch.int32)
                idx = torch.empty(cr, device=self.dev, dtype=torch.int32)
                cnt = torch.empty(1, device=self.dev, dtype=torch.int32)
                first = True
                while a < hi:
                    b = min(a + (min(cr, 512) if first else cr), hi)  # a small probe pass first
                    if tri and not first:
                        a, b = 0, hi  # the triangle form takes all rows (the probe's again)
                    first = False
                    _lib.call("reidmi_rr_rank_rows_f16", _lib.ptr(self.feat), self.N, self.D, self.D,
                              _lib.ptr(self.sqn), _lib.ptr(nrm), _lib.ptr(nmax2), _lib.ptr(x16), Np, Dp, a, b,
                              self.K,
                              _lib.ptr(R[a - lo:]), _lib.ptr(rmax[a - lo:]), _lib.ptr(need),
                              _lib.ptr(self._chunk_buf(cc, Np)), cc, self.st)
                    _lib.call("reidmi_nonzero_i32", _lib.ptr(need), b - a, _lib.ptr(idx), _lib.ptr(cnt), self.st)
                    undecided, rows = int(cnt.item()), b - a
                    self.stats["form"] = "triangle" if tri else "row passes"
                    if not (tri and b - a < hi - lo):  # (the triangle form redoes the probe's rows)
                        self.stats["rows"] += rows
                        self.stats["exact_rows"] += undecided
                        if 0 < undecided <= 65536:  # which rows took the exact fallback (tests)
                            self.stats["exact_idx"].append(idx[:undecided].cpu().numpy().astype(np.int64) + a)
                    self._exact_rows(a, idx, undecided, R[a - lo:b - lo], rmax[a - lo:b - lo])
                    a = b
                    if 2 * undecided > rows:
                        break
            if a < hi:
                self.stats["rows"] += hi - a
                self.stats["exact_rows"] += hi - a
                cr = min(self.chunk_rows, hi - a)
                _lib.call("reidmi_rr_rank_rows", _lib.ptr(self.feat), self.N, self.D, self.D, _lib.ptr(self.sqn), a,
                          hi, self.K, _lib.ptr(R[a - lo:]), _lib.ptr(rmax[a - lo:]),
                          _lib.ptr(self._chunk_buf(cr, self.N)), cr, self.st)
        return R, rmax

    def rank_rows_tri_sharded(self, lo, hi):
        """R2 of this rank's rows lo..hi = shard(N) through the triangle form split over the
        ranks (reidmi_rr_tri_*, include/reidmi.h): records of every row all-gathered, this rank's
        contiguous share of the upper-triangle tile list run over all rows, the partial survivor
        lists exchanged all-to-all with their rows' owners, own rows selected, rows the selection
        marks through the exact rows.  The same bits as the one-GPU triangle (and as the exact
        rows) at 1/W of its MFMA work per rank.  None when the triangle form does not apply (no
        fp16 pre-filter, K > 64, a chunk too small, or concentrated features — every rank then
        agrees, through one all-reduce, to take rank_rows' row passes)."""
        from . import distributed as rd
        rank, W = rd.world()
        # every early return below decides on rank-uniform inputs (the same features, k1, k2 on
        # every rank); a rank-local reason (an empty shard, N < W) joins the all-reduced flag
        # instead, so no rank skips a collective the others enter
        if not (RANK_PREFILTER and self.K <= 64):
            return None
        x16, Np, Dp, nrm, fits, nmax2 = self._feat16()  # the same decision on every rank (same features)
        if not fits or Dp < 128:
            return None
        L = _lib.load()
        cc = max(256, self.chunk_rows * self.N // Np // 256 * 256)
        nt, cap, ns, sp = (ctypes.c_int64() for _ in range(4))
        _lib.call("reidmi_rr_tri_plan", self.N, Np, cc, self.K, ctypes.byref(nt), ctypes.byref(cap), ctypes.byref(ns),
                  ctypes.byref(sp))
        ntiles, cap, ns, sp = nt.value, cap.value, ns.value, sp.value
        # probe (as the one-call path): concentrated features (a random network's embeddings)
        # put every row beyond the bound; then all ranks take the exact row passes
        pr = min(512, hi - lo)
        bad_local = hi <= lo or cap == 0 or ntiles == 0
        if not bad_local:
            Rp = torch.empty((pr, self.K), device=self.dev, dtype=torch.int32)
            mp_ = torch.empty(pr, device=self.dev, dtype=torch.float32)
            need = torch.empty(pr, device=self.dev, dtype=torch.int32)
            _lib.call("reidmi_rr_rank_rows_f16", _lib.ptr(self.feat), self.N, self.D, self.D, _lib.ptr(self.sqn),
                      _lib.ptr(nrm), _lib.ptr(nmax2), _lib.ptr(x16), Np, Dp, lo, lo + pr, self.K, _lib.ptr(Rp),
                      _lib.ptr(mp_), _lib.ptr(need), _lib.ptr(self._chunk_buf(cc, Np)), cc, self.st)
            bad_local = 2 * int(need.sum().item()) > pr
            del Rp, mp_, need
        bad = torch.tensor([float(bad_local)], dtype=torch.float64)
        if rd._initialized():
            b = bad.to(rd._collective_device(self.feat))
            rd.dist.all_reduce(b, op=rd.dist.ReduceOp.MAX)
            bad = b.cpu()
        if bad.item() > 0:
            return None
        self._chunk = None  # the lists take the chunk's place
        N, K = self.N, self.K
        meta = torch.zeros(Np * 4, device=self.dev, dtype=torch.float32)
        wrow = torch.empty(N, device=self.dev, dtype=torch.float32)
        cnt = torch.zeros(N, device=self.dev, dtype=torch.int32)
        lst = torch.empty(N * cap * 2, device=self.dev, dtype=torch.int32)
        sqn_s = torch.empty(ns, device=self.dev, dtype=torch.float32)
        nrm_s = torch.empty(ns, device=self.dev, dtype=torch.float32)
        tiles = torch.empty(max(ntiles, 1), device=self.dev, dtype=torch.int32)
        _lib.call("reidmi_rr_tri_init", _lib.ptr(self.sqn), _lib.ptr(nrm), N, Np, ns, _lib.ptr(meta), _lib.ptr(sqn_s),
                  _lib.ptr(nrm_s), _lib.ptr(tiles), self.st)
        _lib.call("reidmi_rr_tri_sample", _lib.ptr(x16), Np, Dp, _lib.ptr(self.sqn), _lib.ptr(nrm), _lib.ptr(nmax2), N,
                  self.D, K, _lib.ptr(sqn_s), _lib.ptr(nrm_s), ns, lo, hi, _lib.ptr(lst), sp, _lib.ptr(meta),
                  _lib.ptr(wrow), _lib.ptr(cnt), cap, self.st)
        m4 = meta.view(Np, 4)
        m4[:N] = rd.gather_rows(m4[lo:hi].contiguous(), N)  # every row's record (the column records too)
        t0, t1 = rd.shard(ntiles, rank, W)
        _lib.call("reidmi_rr_tri_survivors", _lib.ptr(x16), Np, Dp, _lib.ptr(self.sqn), _lib.ptr(nrm), N, self.D,
                  _lib.ptr(meta), _lib.ptr(tiles), t0, t1, _lib.ptr(cnt), _lib.ptr(lst), cap, self.st)
        del tiles
        # partial lists of each owner's rows -> the owner
        bounds = [rd.shard(N, q, W) for q in range(W)]
        lens = cnt.clamp(max=cap).to(torch.int64)
        send_cnt, send_ent, ent_splits = [], [], []
        for q, (a, b) in enumerate(bounds):
            send_cnt.append(cnt[a:b])
            if q == rank or b == a:
                ent_splits.append(0)
                continue
            off = torch.zeros(b - a, device=self.dev, dtype=torch.int64)
            off[1:] = torch.cumsum(lens[a:b], 0)[:-1]
            total = int(lens[a:b].sum().item())
            out = torch.empty(max(total, 1) * 2, device=self.dev, dtype=torch.int32)
            _lib.call("reidmi_rr_sv_pack", _lib.ptr(cnt[a:]), _lib.ptr(lst[a * cap * 2:]), cap, b - a, _lib.ptr(off),
                      _lib.ptr(out), self.st)
            send_ent.append(out[:total * 2].view(torch.int64))
            ent_splits.append(total)
        rc, cnt_splits = rd.all_to_all_var(torch.cat(send_cnt), [b - a for a, b in bounds])
        re_, ent_got = rd.all_to_all_var(torch.cat(send_ent) if send_ent else torch.zeros(0, device=self.dev,
                                                                                           dtype=torch.int64),
                                         ent_splits)
        rows = hi - lo
        ro, eo = 0, 0
        for q in range(W):
            add_cnt = rc[ro:ro + cnt_splits[q]]
            ro += cnt_splits[q]
            if q != rank:
                alen = add_cnt.clamp(max=cap).to(torch.int64)
                off = torch.zeros(rows, device=self.dev, dtype=torch.int64)
                off[1:] = torch.cumsum(alen, 0)[:-1]
                _lib.call("reidmi_rr_sv_merge", _lib.ptr(cnt[lo:]), _lib.ptr(lst[lo * cap * 2:]), cap, rows,
                          _lib.ptr(add_cnt), _lib.ptr(off), _lib.ptr(re_[eo:]) if ent_got[q] else None, self.st)
            eo += ent_got[q]
        R = torch.empty((rows, K), device=self.dev, dtype=torch.int32)
        rmax = torch.empty(rows, device=self.dev, dtype=torch.float32)
        need = torch.empty(rows, device=self.dev, dtype=torch.int32)
        _lib.call("reidmi_rr_sv_select", _lib.ptr(cnt[lo:]), _lib.ptr(lst[lo * cap * 2:]), cap, _lib.ptr(wrow[lo:]),
                  _lib.ptr(self.feat), self.D, self.D, _lib.ptr(self.sqn), lo, rows, K, _lib.ptr(R), _lib.ptr(rmax),
                  _lib.ptr(need), self.st)
        del lst, re_
        idx = torch.empty(rows, device=self.dev, dtype=torch.int32)
        c = torch.empty(1, device=self.dev, dtype=torch.int32)
        _lib.call("reidmi_nonzero_i32", _lib.ptr(need), rows, _lib.ptr(idx), _lib.ptr(c), self.st)
        undecided = int(c.item())
        self.stats.update(form="triangle (sharded)", rows=self.stats["rows"] + rows,
                          exact_rows=self.stats["exact_rows"] + undecided)
        if 0 < undecided <= 65536:
            self.stats["exact_idx"].append(idx[:undecided].cpu().numpy().astype(np.int64) + lo)
        self._exact_rows(lo, idx, undecided, R, rmax)
        return R, rmax

    def offsets(self, nnz):
        off = torch.empty(nnz.numel() + 1, device=self.dev, dtype=torch.int64)
        _lib.call("reidmi_rr_row_offsets", _lib.ptr(nnz), nnz.numel(), _lib.ptr(off), self.st)
        return off

    def _pack(self, ecol, eval_, nnz, cap, full=None):
        """ELL rows -> CSR (nnz, col, val); `full` = the rows' true entry counts when some rows
        (the deferred V_qe rows, ELL length 0) are written into the CSR afterwards."""
        full = nnz if full is None else full
        off = self.offsets(full)
        total = int(off[-1].item())
        col = torch.empty(max(total, 1), device=self.dev, dtype=torch.int32)
        val = torch.empty(max(total, 1), device=self.dev, dtype=torch.int16)
        _lib.call("reidmi_rr_pack", _lib.ptr(ecol), _lib.ptr(eval_), _lib.ptr(nnz), nnz.numel(), cap, _lib.ptr(off),
                  _lib.ptr(col), _lib.ptr(val), self.st)
        return full, col[:total], val[:total], off

    def _scratch(self, name, nbytes):
        if nbytes <= 0:
            return None
        t = self._ws.get(name)
        if t is None or t.numel() < nbytes:
            t = self._ws[name] = torch.empty(nbytes, device=self.dev, dtype=torch.uint8)
        return t

    def _batches(self, lo, hi, row_bytes):
        step = max(1, int(self.ell_bytes // max(row_bytes, 1)))
        return [(a, min(a + step, hi)) for a in range(lo, hi, step)]

    def _cat(self, parts):
        if not parts:
            z = torch.zeros(0, device=self.dev, dtype=torch.int32)
            return z, z, torch.zeros(0, device=self.dev, dtype=torch.int16)
        if len(parts) == 1:
            return parts[0]
        return tuple(torch.cat([p[k] for p in parts]) for k in range(3))

    def v_rows(self, R, rmax, lo, hi):
        """R3 over rows lo..hi: ELL batches of width vcap (the k-reciprocal bound), packed to CSR."""
        ws = self._scratch("v", self.v_ws_bytes)
        parts = []
        for a, b in self._batches(lo, hi, self.vcap * 6):
            n = b - a
            ecol = torch.empty((n, self.vcap), device=self.dev, dtype=torch.int32)
            evl = torch.empty((n, self.vcap), device=self.dev, dtype=torch.int16)
            nnz = torch.zeros(n, device=self.dev, dtype=torch.int32)
            _lib.call("reidmi_rr_v_rows", _lib.ptr(self.feat), self.N, self.D, self.D, _lib.ptr(self.sqn),
                      _lib.ptr(rmax), _lib.ptr(R), self.K, a, b, self.k1, _lib.ptr(ecol), _lib.ptr(evl), _lib.ptr(nnz),
                      _lib.ptr(ws), self.v_ws_bytes, _lib.ptr(self.flags), self.st)
            parts.append(self._pack(ecol, evl, nnz, self.vcap)[:3])
        return self._cat(parts)

    def qe_rows(self, R, V, lo, hi):
        """R4 over rows lo..hi: rows assembled on chip go through an ELL of width qcap; rows
        beyond it (dense neighbourhoods, k2 > 32) are counted, then written straight into the
        CSR by reidmi_rr_qe_deferred."""
        off, col, val = V
        fast = self.k2e <= 32
        parts = []
        for a, b in self._batches(lo, hi, self.qcap * 6 if fast else 4):
            n = b - a
            w = n if fast else 1
            ecol = torch.empty((w, self.qcap), device=self.dev, dtype=torch.int32)
            evl = torch.empty((w, self.qcap), device=self.dev, dtype=torch.int16)
            nnz = torch.zeros(n, device=self.dev, dtype=torch.int32)
            dlist = torch.empty(n, device=self.dev, dtype=torch.int32)
            dcount = torch.zeros(1, device=self.dev, dtype=torch.int32)
            _lib.call("reidmi_rr_qe_rows", _lib.ptr(R), self.K, self.k2e, a, b, _lib.ptr(off), _lib.ptr(col),
                      _lib.ptr(val), _lib.ptr(ecol), _lib.ptr(evl), _lib.ptr(nnz), _lib.ptr(dlist), _lib.ptr(dcount),
                      self.st)
            nd = int(dcount.item())
            full = nnz
            if nd:
                ws = self._scratch("qe", self.qe_ws_bytes)
                full = nnz.clone()
                _lib.call("reidmi_rr_qe_deferred", _lib.ptr(R), self.K, self.k1, self.k2e, a, self.N, _lib.ptr(off),
                          _lib.ptr(col), _lib.ptr(val), _lib.ptr(dlist), nd, 0, None, None, None, _lib.ptr(full),
                          _lib.ptr(ws), self.qe_ws_bytes, _lib.ptr(self.flags), self.st)
            cnt, qcol, qval, qoff = self._pack(ecol, evl, nnz, self.qcap, full)
            if nd:
                _lib.call("reidmi_rr_qe_deferred", _lib.ptr(R), self.K, self.k1, self.k2e, a, self.N, _lib.ptr(off),
                          _lib.ptr(col), _lib.ptr(val), _lib.ptr(dlist), nd, 1, _lib.ptr(qoff), _lib.ptr(qcol),
                          _lib.ptr(qval), None, _lib.ptr(ws), self.qe_ws_bytes, _lib.ptr(self.flags), self.st)
            parts.append((cnt, qcol, qval))
        return self._cat(parts)

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
            L = _lib.load()
            bb = int(L.reidmi_rr_jaccard_bounds_bytes(N, G))
            bounds = torch.empty((bb + 7) // 8, device=self.dev, dtype=torch.int64)
            cr = int(max(1, min(65535, qhi - qlo, self.chunk_rows * N // max(G, 1))))
            _lib.call("reidmi_rr_jaccard_rows", _lib.ptr(self.feat), N, self.D, self.D, _lib.ptr(self.sqn),
                      _lib.ptr(rmax), Q, qlo, qhi, _lib.ptr(off), _lib.ptr(col), _lib.ptr(val), _lib.ptr(coff),
                      _lib.ptr(irow), _lib.ptr(ival), self.lam_h, self.lam_f, _lib.ptr(out), G,
                      _lib.ptr(self._chunk_buf(cr, G)), cr, _lib.ptr(bounds), bb, self.st)
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
    # R1 + R2 (reranking.py:36-48): several ranks split the one-GPU triangle form's tiles
    tri = stages.rank_rows_tri_sharded(lo, hi) if W > 1 and hasattr(stages, "rank_rows_tri_sharded") else None
    R_loc, rmax_loc = tri if tri is not None else stages.rank_rows(lo, hi)
    R = rd.gather_rows(R_loc, N)
    rmax = rd.gather_rows(rmax_loc, N)
    V = _gather_csr(stages, *stages.v_rows(R, rmax, lo, hi), N)  # R3 (reranking.py:51-71)
    if stages.k2 != 1 and stages.k2e >= 2:  # (k2 capped at N = 1 row: the mean is V itself)
        Vq = _gather_csr(stages, *stages.qe_rows(R, V, lo, hi), N)  # R4 (reranking.py:73-78)
    else:
        Vq = V
    qlo, qhi = rd.shard(Q, rank, W)
    out = stages.jaccard_rows(rmax, Vq, qlo, qhi)                 # R5-R7 (reranking.py:80-100)
    stages.check()
    return out


def re_ranking_sharded(probFea, galFea, k1, k2, lambda_value, chunk_bytes=None, stats=None):
    """Sharded re_ranking: probFea / galFea are the FULL query and gallery features on this
    rank's GPU (all-gathered after a sharded embed).  Returns this rank's query rows
    shard(Q, rank, W) of the re-ranked (Q, G) distance as a device tensor; with one process
    it equals re_ranking_device bit for bit, without the N x N buffers."""
    q = _as_dev_f32(probFea)
    Q = q.shape[0]
    feat = torch.cat([q, _as_dev_f32(galFea)]).contiguous()
    stages = HipStages(feat, Q, k1, k2, lambda_value, chunk_bytes)
    out = staged_rerank(stages, feat.shape[0], Q)
    if stats is not None:  # R2 path counters of this rank (rows, rows sent to the exact fallback, form)
        stats.update(stages.stats)
    return out
