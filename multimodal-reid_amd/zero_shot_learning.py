"""Drop-in for the reference's zero_shot_learning.py eval driver (the hot path):

    inference(model, bottleneck, bottleneck_proj, zeroshot_weights, loader, loader_augment,
              multimodal, model_type) -> (embeddings, targets, camera_ids, sequence_ids)
                                                                 zero_shot_learning.py:61-134
    get_cmc_map(gallery_embeddings, query_embeddings, gallery_labels, query_labels,
                gallery_cams, query_cams) -> (cmc, mAP)          zero_shot_learning.py:137-153
    zeroshot_classifier(text_model, class_tokens) -> (n_cls, E)  zero_shot_learning.py:37-55

Differences from the reference that do not change results: both TTA passes of a batch run
back to back and the feature epilogue (average / concat / --mm softmax) is one HIP kernel;
embeddings stay fp32 on the GPU (the reference keeps fp16 then copies to the CPU).
``model`` is a model.CLIP / model.VisionTransformer (libreidmi).  Only model_type "vit"
exists here (the north-star path is the ViT tower).
"""
import numpy as np
import torch

from . import _lib
from .evaluate import R1_mAP_eval
from .loader import TtaView


def _vis(model):
    return getattr(model, "visual", model)


def embed_pair(model, images, images_aug=None, tta=None, zeroshot_weights=None, multimodal=False, out=None):
    """Feature rows for one batch: plain pass + augmented pass (an augmented image batch, or
    on-the-fly ``tta`` crop offsets applied to ``images_aug`` when given, else to ``images``),
    fused epilogue."""
    vis = _vis(model)
    B = images.shape[0]
    W, E = vis.width, vis.out_dim
    a12, ap = vis.encode_cls(images)
    b12, bp = vis.encode_cls(images if images_aug is None else images_aug, tta=tta)
    st = _lib.stream(vis.device)
    if multimodal:
        zs = zeroshot_weights.to(vis.device, torch.float32).contiguous()
        ncls = zs.shape[0]
        if out is None:
            out = torch.empty(B, W + ncls, device=vis.device, dtype=torch.float32)
        _lib.call("reidmi_feature_tta_mm", _lib.ptr(a12), _lib.ptr(ap), _lib.ptr(b12), _lib.ptr(bp), _lib.ptr(zs),
                  B, W, E, ncls, _lib.ptr(out), out.stride(0), st)
    else:
        if out is None:
            out = torch.empty(B, W + E, device=vis.device, dtype=torch.float32)
        _lib.call("reidmi_feature_tta_avg", _lib.ptr(a12), _lib.ptr(ap), _lib.ptr(b12), _lib.ptr(bp), B, W, E,
                  _lib.ptr(out), out.stride(0), st)
    return out


def inference(model, bottleneck, bottleneck_proj, zeroshot_weights, loader, loader_augment, multimodal,
              model_type):
    """zero_shot_learning.py:61-134.  Loaders yield (images, target, cams, seqs, indices);
    the i-th batches of the two loaders hold the same images (shuffle=False).  An augmented
    batch may be a loader.TtaView (the device loaders of loader.get_loader): its flip / pad /
    crop then run inside the encoder's im2col."""
    if model_type != "vit":
        raise NotImplementedError("libreidmi implements the ViT tower (north-star path) only")
    embeddings, targets, camera_ids, sequence_ids = [], [], [], []
    with torch.no_grad():
        for (images, target, cams, seqs, _), (images_aug, *_rest) in zip(loader, loader_augment):
            if isinstance(images_aug, TtaView):
                emb = embed_pair(model, images, images_aug.images, images_aug.offsets, zeroshot_weights, multimodal)
            else:
                emb = embed_pair(model, images, images_aug, None, zeroshot_weights, multimodal)
            embeddings.append(emb)
            targets.append(torch.as_tensor(target))
            camera_ids.append(torch.as_tensor(cams))
            sequence_ids.append(torch.as_tensor(seqs))
    return (torch.cat(embeddings, dim=0), torch.cat(targets, dim=0), torch.cat(camera_ids, dim=0),
            torch.cat(sequence_ids, dim=0))


def get_cmc_map(gallery_embeddings, query_embeddings, gallery_labels, query_labels, gallery_cams, query_cams,
                reranking=False, sharded=False):
    """zero_shot_learning.py:137-153 (R1_mAP_eval with max_rank=50, feat_norm=True);
    ``reranking=True`` selects R1_mAP_eval's k-reciprocal branch (evaluate.py:124-127).
    ``sharded=True`` (torch.distributed process group, torchrun, one process per GPU): the
    arguments are THIS rank's shards (its loaders' images, e.g. contiguous shards in rank
    order); R1_mAP_eval all-gathers them and every rank returns the CMC/mAP of the whole split,
    bit-identical to one process over the concatenated shards (evaluate.R1_mAP_eval).  Default:
    one process's data, no collective (distributed.py states the contract)."""
    evaluator = R1_mAP_eval(len(query_labels), max_rank=50, feat_norm=True, reranking=reranking, sharded=sharded)
    evaluator.reset()
    evaluator.update((torch.cat((query_embeddings.float(), gallery_embeddings.float()), dim=0),
                      torch.cat((torch.as_tensor(query_labels), torch.as_tensor(gallery_labels)), dim=0),
                      torch.cat((torch.as_tensor(query_cams), torch.as_tensor(gallery_cams)), dim=0)))
    return evaluator.compute()


def zeroshot_classifier(text_model, class_tokens, augmented_template=True):
    """zero_shot_learning.py:37-55.  Augmented templates (:39-49): per class, encode its
    template token rows, L2-normalise, mean over templates, L2-normalise; ``class_tokens``
    is a list of int64 [n_templates, 77] arrays.  Plain (:50-54): one token row per class
    ([n_cls, 77]), encoded and L2-normalised.  (The CLIP BPE vocabulary is not available
    offline, so callers pass token ids.)"""
    from .ops import class_mean_normalize_device
    if augmented_template:
        rows = [torch.as_tensor(np.asarray(t)).reshape(-1, np.asarray(t).shape[-1]) for t in class_tokens]
        counts = [r.shape[0] for r in rows]
        tokens = torch.cat(rows, 0)
    else:
        tokens = torch.as_tensor(np.asarray(class_tokens))
        counts = [1] * tokens.shape[0]
    feats = text_model.encode_text(tokens)
    return class_mean_normalize_device(feats, counts)
