"""Weight-format boundary of the drop-in (load time, host side; not timed).

    model_adaptor(model, height, width, weights=None, model_type="vit", training_mode="coop",
                  vision_stride_size=12) -> (model, bottleneck, bottleneck_proj)   utils.py:169-262
    load_clip(state_dict, height, width, ...) -> model.CLIP                       maple.py:1044-1098
    load_model(model, classnames, templates, weights, ...) -> (zeroshot_weights, model)
                                                                   zero_shot_learning.py:15-58
    resize_pos_embed                                                              utils.py:111-125

CLIP-ReID checkpoints store the towers under ``image_encoder.*`` / ``text_encoder.*``
(utils.py:211-214, zero_shot_learning.py:31-34); OpenAI CLIP state dicts under
``visual.*`` and top-level text keys.  Checkpoints are read with
``torch.load(weights_only=True)`` only (no pickle or TorchScript code is executed; the
reference tries ``torch.jit.load`` first, utils.py:171-175 — a TorchScript archive is
refused here: re-save its ``state_dict()`` with ``torch.save``).
BNNeck (utils.py:128-142) is constructed and loaded but, as in the reference's eval
(zero_shot_learning.py:91-92), never applied.
"""
import numpy as np
import torch

from .model import CLIP, TextTransformer, VisionTransformer, resize_pos_embed  # noqa: F401


def load_checkpoint(path):
    """State dict of a checkpoint file, weights-only (utils.py:17-55,171-175 semantics:
    a ``state_dict`` entry is unwrapped, a DataParallel ``module.`` prefix stripped)."""
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and "state_dict" in sd:
        sd = sd["state_dict"]
    if not isinstance(sd, dict):
        raise ValueError(f"{path}: not a state dict")
    return {k[7:] if k.startswith("module.") else k: v for k, v in sd.items()}


class BNNeck:
    """utils.py:128-142 (BatchNorm1d, eval mode): y = (x - mean) / sqrt(var + eps) * w + b."""

    def __init__(self, width, proj):
        self.proj = proj
        self.width = width
        self.params = None

    def load_state_dict(self, sd, strict=False):
        key = "bottleneck_proj" if self.proj else "bottleneck"
        p = {k.split(".")[-1]: v for k, v in sd.items() if k.split(".")[0] == key}
        self.params = p or None

    def eval(self):
        return self


def model_adaptor(model, height, width, weights=None, model_type="vit", training_mode="coop",
                  vision_stride_size=12, device=None):
    """Build the libreidmi vision tower from a CLIP-ReID checkpoint (``image_encoder.*``
    keys) exactly as utils.py:169-262 re-shapes the model: stride-12 patches, grid
    height//12 x width//12, positional embedding bicubic-resized when its grid differs.
    ``model`` may be None or a model.CLIP whose text tower is kept."""
    if model_type != "vit":
        raise NotImplementedError("libreidmi implements the ViT towers (north-star path)")
    sd = load_checkpoint(weights) if isinstance(weights, str) else weights
    if sd is None:
        raise ValueError("model_adaptor: a checkpoint (path or state dict) is required")
    vis = {k[len("image_encoder."):]: v for k, v in sd.items() if k.startswith("image_encoder.")}
    if not vis:
        vis = {k[len("visual."):]: v for k, v in sd.items() if k.startswith("visual.")}
    visual = VisionTransformer(vis, height=height, width=width, stride=vision_stride_size, device=device)
    bottleneck = BNNeck(visual.width, False)
    bottleneck_proj = BNNeck(visual.out_dim, True)
    bneck = {k: v for k, v in sd.items() if "bottleneck" in k}
    if bneck:
        bottleneck.load_state_dict(bneck)
        bottleneck_proj.load_state_dict(bneck)
    text = getattr(model, "text", None)
    return CLIP(visual, text), bottleneck, bottleneck_proj


def load_clip(state_dict, height=256, width=128, stride=12, device=None, text=True):
    """CLIP from an OpenAI-layout state dict (``visual.*`` + text keys), maple.build_model style."""
    vis = {k[len("visual."):]: v for k, v in state_dict.items() if k.startswith("visual.")}
    visual = VisionTransformer(vis, height=height, width=width, stride=stride, device=device) if vis else None
    tx = None
    if text and "token_embedding.weight" in state_dict:
        txt = {k: v for k, v in state_dict.items() if not k.startswith("visual.")}
        tx = TextTransformer(txt, device=device)
    return CLIP(visual, tx)


def text_encoder_overlay(base_text_sd, weights):
    """zero_shot_learning.py:28-35: the CLIP text tower's state dict with the checkpoint's
    ``text_encoder.*`` entries laid over it (prefix stripped, each cast to the base entry's
    dtype, strict=False: keys the checkpoint lacks keep the base values; a ``text_encoder.*`` key
    the tower does not have raises KeyError, as the reference's dtype lookup does, :34).
    ``weights``: a checkpoint path (weights-only load) or state dict, or None."""
    sd = dict(base_text_sd)
    if weights is None:
        return sd
    ck = load_checkpoint(weights) if isinstance(weights, str) else weights
    for key, v in ck.items():
        if key.startswith("text_encoder."):
            k = key[len("text_encoder."):]
            base = sd[k]  # KeyError for a key the tower lacks (zero_shot_learning.py:34)
            dt = base.dtype if isinstance(base, torch.Tensor) else torch.from_numpy(np.asarray(base)).dtype
            sd[k] = (v if isinstance(v, torch.Tensor) else torch.from_numpy(np.asarray(v))).to(dt)
    return sd


def load_model(model, classnames, templates, weights, augmented_template=True, tokenize=None, device=None):
    """zero_shot_learning.py:15-58 (coop mode): the CLIP text tower with the CLIP-ReID
    checkpoint's ``text_encoder.*`` overlay (text_encoder_overlay), then the zero-shot
    classifier over the class names' templates (zeroshot_classifier: augmented templates ->
    per-class normalise / mean / normalise; plain -> one template per class, normalised).
    ``model``: what ``clip.load(model_name)`` returns in the reference — here an OpenAI-layout
    state dict (``clip.load`` downloads weights, which this environment cannot) or a model.CLIP
    whose text tower's source state dict is kept (``model.text.source_state_dict``).
    ``templates[classname]``: a list of sentences (augmented) or one sentence (plain);
    ``tokenize``: clip.tokenize's role (tokenizer.tokenize with the BPE vocabulary, which is not
    shipped: parity unpinned) — or pass token ids directly as the templates' values.
    Returns (zeroshot_weights [n_cls, E] fp32 on the GPU, model.CLIP)."""
    from .zero_shot_learning import zeroshot_classifier
    if isinstance(model, CLIP):
        base = getattr(model.text, "source_state_dict", None)
        if base is None:
            raise ValueError("load_model: the CLIP model's text tower keeps no source state dict; pass the state dict")
        visual = model.visual
    else:
        base = {k: v for k, v in model.items() if not k.startswith("visual.")}
        visual = None
    text = TextTransformer(text_encoder_overlay(base, weights), device=device)
    text.source_state_dict = base

    def ids(t):
        if isinstance(t, (str, list)) and (isinstance(t, str) or (t and isinstance(t[0], str))):
            if tokenize is None:
                raise ValueError("load_model: sentences need a tokenizer (tokenizer.tokenize with the CLIP BPE "
                                 "vocabulary); or pass token ids")
            return np.asarray(tokenize(t if isinstance(t, list) else [t]))
        return np.asarray(t)

    if augmented_template:
        zw = zeroshot_classifier(text, [ids(templates[c]) for c in classnames], augmented_template=True)
    else:
        zw = zeroshot_classifier(text, np.concatenate([ids(templates[c]).reshape(1, -1) for c in classnames]),
                                 augmented_template=False)
    return zw, CLIP(visual, text)
