"""Drop-in for the reference's reranking.py:

    re_ranking(probFea, galFea, k1, k2, lambda_value, local_distmat=None, only_local=False)
        -> np.ndarray float32 (num_query, num_gallery)                  reranking.py:29-100

k-reciprocal encoding + Jaccard re-ranking (Zhong et al., CVPR'17) on the GPU through
libreidmi (rerank.hip).  Given the same original distances it reproduces the reference's
numpy arithmetic bit for bit (float32 exp/pairwise sums, float16 V / Jaccard), with ties in
the initial ranking ordered by index (np.argsort(kind="stable")).  The reference's dense
N x N float16 V / V_qe become sparse row lists, so MSMT17-size galleries fit.
"""
import numpy as np
import torch

from . import _lib
from .evaluate import _as_dev_f32, euclidean_distance_device

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
