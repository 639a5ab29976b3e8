"""Oracle: CPU restatement of the reference retrieval back end (+ fp32 encoders).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker or the timed CPU baseline.  The
product package (multimodal-reid_amd/) never imports it and has no CPU fallback.

Parity status:
  * eval_func, re_ranking stages R2-R7: pinned bit-exact to fixtures made by the
    reference itself (tests/golden/make_goldens.py).
  * euclidean_distance / F.normalize: the reference uses torch CPU BLAS whose
    accumulation order is not reproducible; pinned within 2e-6 abs.
  * encoders (oracle/vit_ref.py): fp32 torch restatement pinned to the reference
    modules' fp32 outputs on synthetic weights.
  * test-time transforms (transforms_oracle.c): Pillow's bilinear resize + ToTensor +
    Normalize, pinned bit-exact to fixtures made with Pillow 12.2 itself
    (tests/golden/make_transform_goldens.py).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_u16p = np.ctypeslib.ndpointer(np.uint16, flags="C_CONTIGUOUS")
_i64 = ctypes.c_int64


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def set_threads(n):
    """Worker threads of the C restatement's parallel loops (results do not depend on it)."""
    lib().orc_set_threads(int(n))


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "build", "liboracle.so")
        src = os.path.join(HERE, "reid_oracle.c")
        if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
            build()
        L = ctypes.CDLL(path)
        L.orc_l2norm.argtypes = [_f32p, _f32p, _i64, _i64]
        L.orc_distmat.argtypes = [_f32p, _f32p, _i64, _i64, _i64, _f32p]
        L.orc_topk_rows.argtypes = [_f32p, _i64, _i64, _i64, _i32p]
        L.orc_eval_rows.argtypes = [_f32p, _i64, _i64, _i64p, _i64p, _i64p, _i64p, _i32p, _i64p, _f64p, _i64p]
        L.orc_rerank_from_dist.argtypes = [_f32p, _i64, _i64, ctypes.c_int, ctypes.c_int, ctypes.c_uint16,
                                           ctypes.c_float, _f32p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p]
        L.orc_rr_rank_rows.argtypes = [_f32p, _i64, _i64, _i64, _i32p, _f32p]
        L.orc_rr_v_rows.argtypes = [_f32p, _f32p, _i32p, _i64, _i64, _i64, _i64, ctypes.c_int, _u16p]
        L.orc_rr_qe_rows.argtypes = [_i32p, _i64, ctypes.c_int, _i64, _i64, _u16p, _i64, _u16p]
        L.orc_rr_jaccard_rows.argtypes = [_f32p, _f32p, _i64, _i64, _i64, _u16p, _i64, ctypes.c_uint16,
                                          ctypes.c_float, _f32p]
        L.orc_np_expf.argtypes = [ctypes.c_float]
        L.orc_np_expf.restype = ctypes.c_float
        L.orc_f2h.argtypes = [ctypes.c_float]
        L.orc_f2h.restype = ctypes.c_uint16
        L.orc_pairwise_f32.argtypes = [_f32p, _i64]
        L.orc_pairwise_f32.restype = ctypes.c_float
        L.orc_pairwise_f64.argtypes = [_f64p, _i64]
        L.orc_pairwise_f64.restype = ctypes.c_double
        _u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
        _i = ctypes.c_int
        L.orc_pil_resize_rgb.argtypes = [_u8p, _i, _i, _i, _i, _u8p]
        L.orc_to_tensor_normalize.argtypes = [_u8p, _i, _i, _f32p, _f32p, _f32p]
        L.orc_resize_vertical_first.argtypes = [_i, _i, _i, _i]
        _LIB = L
    return _LIB


def _c(a, dt):
    return np.ascontiguousarray(np.asarray(a), dtype=dt)


def pil_resize(img, oh, ow):
    """PIL.Image.resize((ow, oh), BILINEAR) of an HxWx3 uint8 image (transforms_oracle.c)."""
    img = _c(img, np.uint8)
    out = np.empty((oh, ow, 3), np.uint8)
    lib().orc_pil_resize_rgb(img, img.shape[0], img.shape[1], oh, ow, out)
    return out


def to_tensor_normalize(img, mean=(0.5, 0.5, 0.5), std=(0.5, 0.5, 0.5)):
    """ToTensor() -> Normalize(mean, std) of an HxWx3 uint8 image -> float32 [3, H, W]."""
    img = _c(img, np.uint8)
    out = np.empty((3,) + img.shape[:2], np.float32)
    lib().orc_to_tensor_normalize(img, img.shape[0], img.shape[1], _c(mean, np.float32), _c(std, np.float32), out)
    return out


def eval_transform(img, oh=256, ow=128, mean=(0.5, 0.5, 0.5), std=(0.5, 0.5, 0.5)):
    """data_prepare.py:257-261: Resize -> ToTensor -> Normalize."""
    return to_tensor_normalize(pil_resize(img, oh, ow), mean, std)


def l2norm(x):
    x = _c(x, np.float32)
    y = np.empty_like(x)
    lib().orc_l2norm(x, y, x.shape[0], x.shape[1])
    return y


def distmat(q, g):
    q, g = _c(q, np.float32), _c(g, np.float32)
    out = np.empty((q.shape[0], g.shape[0]), np.float32)
    lib().orc_distmat(q, g, q.shape[0], g.shape[0], q.shape[1], out)
    return out


def topk_rows(dist, k):
    dist = _c(dist, np.float32)
    out = np.empty((dist.shape[0], k), np.int32)
    lib().orc_topk_rows(dist, dist.shape[0], dist.shape[1], k, out)
    return out


def eval_rows(dist, q_pids, g_pids, q_camids, g_camids):
    dist = _c(dist, np.float32)
    Q, G = dist.shape
    valid = np.empty(Q, np.int32)
    first = np.empty(Q, np.int64)
    ap = np.empty(Q, np.float64)
    nkept = np.empty(Q, np.int64)
    lib().orc_eval_rows(dist, Q, G, _c(q_pids, np.int64), _c(g_pids, np.int64), _c(q_camids, np.int64),
                        _c(g_camids, np.int64), valid, first, ap, nkept)
    return valid, first, ap, nkept


def eval_func(distmat_, q_pids, g_pids, q_camids, g_camids, max_rank=50):
    """evaluate.py:29-88 restated: per-query part in C, the aggregation (82-88) here."""
    Q, G = distmat_.shape
    if G < max_rank:
        max_rank = G
    valid, first, ap, nkept = eval_rows(distmat_, q_pids, g_pids, q_camids, g_camids)
    all_cmc, all_ap = [], []
    for q in range(Q):
        if not valid[q]:
            continue
        cmc = (np.arange(nkept[q]) >= first[q]).astype(np.int32)
        all_cmc.append(cmc[:max_rank])
        all_ap.append(ap[q])
    assert len(all_cmc) > 0, "Error: all query identities do not appear in gallery"
    all_cmc = np.asarray(all_cmc).astype(np.float32)
    all_cmc = all_cmc.sum(0) / float(len(all_ap))
    return all_cmc, np.mean(all_ap)


def rerank_from_dist(D, num_query, k1, k2, lambda_value, debug=False):
    """re_ranking(..., local_distmat=D, only_local=True) restated (reranking.py:29-100)."""
    D = _c(D, np.float32)
    N = D.shape[0]
    Q = num_query
    final = np.empty((Q, N - Q), np.float32)
    K = min(max(k1 + 1, k2), N)
    lam_h = np.float16(1 - lambda_value).view(np.uint16)
    lam_f = np.float32(lambda_value)
    if debug:
        rank = np.empty((N, K), np.int32)
        vqe = np.empty((N, N), np.uint16)
        jac = np.empty((Q, N), np.uint16)
        ptrs = [rank.ctypes.data, vqe.ctypes.data, jac.ctypes.data]
    else:
        ptrs = [None, None, None]
    lib().orc_rerank_from_dist(D, N, Q, k1, k2, int(lam_h), float(lam_f), final, *ptrs)
    if debug:
        return final, rank, vqe, jac
    return final


def re_ranking(probFea, galFea, k1, k2, lambda_value):
    """Full reference path: distance from features (oracle arithmetic) then R2-R7."""
    feat = np.concatenate([np.asarray(probFea, np.float32), np.asarray(galFea, np.float32)])
    return rerank_from_dist(distmat(feat, feat), len(probFea), k1, k2, lambda_value)


class RerankStages:
    """Staged re_ranking (R2-R7 over row ranges, orc_rr_*) with the exchange formats of the
    product's multimodal_reid_amd.reranking.staged_rerank: torch CPU tensors, V / V_qe rows as
    CSR (nnz, col int32, fp16 bits as int16).  Rows are kept dense inside (small N only)."""

    def __init__(self, feat, num_query, k1, k2, lambda_value):
        import torch
        self.torch = torch
        self.feat = np.ascontiguousarray(np.asarray(feat, np.float32))
        self.N = self.feat.shape[0]
        self.Q = num_query
        self.k1, self.k2 = k1, k2
        self.K = min(max(k1 + 1, k2), self.N)
        self.k2e = min(k2, self.K)
        self.lam_h = np.float16(1 - lambda_value).view(np.uint16)
        self.lam_f = np.float32(lambda_value)

    def _rows(self, lo, hi):
        return distmat(self.feat[lo:hi], self.feat)

    def rank_rows(self, lo, hi):
        R = np.zeros((hi - lo, self.K), np.int32)
        rmax = np.zeros(hi - lo, np.float32)
        if hi > lo:
            lib().orc_rr_rank_rows(self._rows(lo, hi), hi - lo, self.N, self.K, R, rmax)
        return self.torch.from_numpy(R), self.torch.from_numpy(rmax)

    def offsets(self, nnz):
        off = np.zeros(nnz.numel() + 1, np.int64)
        off[1:] = np.cumsum(nnz.numpy().astype(np.int64))
        return self.torch.from_numpy(off)

    def _to_csr(self, dense):
        nz = (dense & 0x7fff) != 0
        nnz = nz.sum(1).astype(np.int32)
        r, c = np.nonzero(nz)
        return (self.torch.from_numpy(nnz), self.torch.from_numpy(c.astype(np.int32)),
                self.torch.from_numpy(dense[r, c].view(np.int16).copy()))

    def _dense(self, V):
        off, col, val = (t.numpy() for t in V)
        d = np.zeros((self.N, self.N), np.uint16)
        rows = np.repeat(np.arange(self.N), np.diff(off))
        d[rows, col] = val.view(np.uint16)
        return d

    def v_rows(self, R, rmax, lo, hi):
        Vr = np.zeros((hi - lo, self.N), np.uint16)
        if hi > lo:
            lib().orc_rr_v_rows(self._rows(lo, hi), _c(rmax.numpy(), np.float32), _c(R.numpy(), np.int32), self.N,
                                self.K, lo, hi, self.k1, Vr)
        return self._to_csr(Vr)

    def qe_rows(self, R, V, lo, hi):
        Vq = np.zeros((hi - lo, self.N), np.uint16)
        if hi > lo:
            lib().orc_rr_qe_rows(_c(R.numpy(), np.int32), self.K, self.k2, lo, hi, self._dense(V), self.N, Vq)
        return self._to_csr(Vq)

    def jaccard_rows(self, rmax, Vq, qlo, qhi):
        out = np.zeros((qhi - qlo, self.N - self.Q), np.float32)
        if qhi > qlo:
            lib().orc_rr_jaccard_rows(self._rows(qlo, qhi), _c(rmax.numpy(), np.float32), self.Q, qlo, qhi,
                                      self._dense(Vq), self.N, int(self.lam_h), float(self.lam_f), out)
        return self.torch.from_numpy(out)

    def check(self):
        pass
