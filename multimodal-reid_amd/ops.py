"""Small device ops around the hot path (libreidmi kernels, torch tensors in/out)."""
import torch

from . import _lib


def cosine_distance_device(qf, gf):
    """evaluate.py:16-26 on the GPU: arccos(clip(cos, -1+1e-5, 1-1e-5)) as (Q,G) fp32."""
    Q, D = qf.shape
    G = gf.shape[0]
    out = torch.empty((Q, G), device=qf.device, dtype=torch.float32)
    ws = torch.empty(Q + G, device=qf.device, dtype=torch.float32)
    _lib.call("reidmi_cosine_f32", _lib.ptr(qf), Q, qf.stride(0), _lib.ptr(gf), G, gf.stride(0), D, _lib.ptr(out),
              out.stride(0), _lib.ptr(ws), _lib.stream())
    return out


def class_mean_normalize_device(feats, counts):
    """zero_shot_learning.py:42-48: per class normalise rows, mean, normalise."""
    feats = feats.to(torch.float32).contiguous()
    off = torch.zeros(len(counts) + 1, dtype=torch.int64)
    off[1:] = torch.cumsum(torch.as_tensor(counts, dtype=torch.int64), 0)
    off = off.to(feats.device)
    out = torch.empty(len(counts), feats.shape[1], device=feats.device, dtype=torch.float32)
    _lib.call("reidmi_class_mean_normalize", _lib.ptr(feats), _lib.ptr(off), len(counts), feats.shape[1],
              _lib.ptr(out), _lib.stream())
    return out
