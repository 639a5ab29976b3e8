"""Prompt learners of the eval path (T3), device tensors + libreidmi's prompt_build kernel:

    PromptLearner(num_class, clip_model, dataset_name, tokenized_prompts, cls_ctx=None)
        .forward(label) -> [B, 77, W]            coop.py:62-110 (prefix 4 | cls_ctx 5 | suffix 68)
    VLPromptLearner(n_cls, clip_model, dataset_name, tokenized_prompts, ctx=None)
        .forward(label) -> [B, 77, W]            maple.py:21-90 (prefix 5 | ctx 4 | suffix 68)

The prompts feed TextEncoder(prompts, tokenized_prompts) (text_encoder.py:14-24; model.py).
The reference tokenises its context string ("A photo of X X X X X person." / "... vehicle.")
with clip.tokenize; the BPE vocabulary is not available offline, so callers pass that
string's token row (``tokenized_prompts``, int64 [1, 77]).  ``cls_ctx`` / ``ctx`` are the
learned context vectors (a checkpoint's ``prompt_learner.cls_ctx`` / ``prompt_learner.ctx``);
without them they are drawn N(0, 0.02) like the reference's initialisation.
"""
import numpy as np
import torch

from . import _lib


def _ctx_string(dataset_name):
    """coop.py:65-68 / maple.py:27-30."""
    if dataset_name in ("market1501", "dukemtmc", "msmt17", "personx"):
        return "A photo of X X X X X person."
    return "A photo of X X X X X vehicle."


class _Learner:
    n_prefix = n_ctx = 0

    def __init__(self, n_cls, clip_model, dataset_name, tokenized_prompts, ctx, seed):
        text = getattr(clip_model, "text", clip_model)
        self.text = text
        self.device = text.device
        self.ctx_init = _ctx_string(dataset_name)
        if tokenized_prompts is None:
            raise NotImplementedError(f"tokenized_prompts (the token row of {self.ctx_init!r}) is required: "
                                      "the CLIP BPE vocabulary is not available offline")
        tok = torch.as_tensor(np.asarray(tokenized_prompts), dtype=torch.int64).reshape(1, -1).to(self.device)
        self.tokenized_prompts = tok
        emb = text.token_embedding(tok)[0].float()  # [77, W]
        P, C = self.n_prefix, self.n_ctx
        self.token_prefix = emb[:P].contiguous()
        self.token_suffix = emb[P + C:].contiguous()
        W = emb.shape[1]
        if ctx is None:
            g = torch.Generator().manual_seed(seed)
            ctx = torch.randn(n_cls, C, W, generator=g) * 0.02
        self.ctx = torch.as_tensor(np.asarray(ctx) if not isinstance(ctx, torch.Tensor) else ctx,
                                   dtype=torch.float32).to(self.device).contiguous()
        if tuple(self.ctx.shape) != (n_cls, C, W):
            raise ValueError(f"context vectors must be [{n_cls}, {C}, {W}], got {tuple(self.ctx.shape)}")
        self.n_cls = n_cls

    def forward(self, label):
        label = torch.as_tensor(label, dtype=torch.int64).reshape(-1).to(self.device).contiguous()
        B = label.shape[0]
        W = self.ctx.shape[2]
        L = self.n_prefix + self.n_ctx + self.token_suffix.shape[0]
        out = torch.empty(B, L, W, device=self.device, dtype=torch.float32)
        bad = torch.zeros(1, device=self.device, dtype=torch.int32)
        _lib.call("reidmi_prompt_build", _lib.ptr(self.token_prefix), self.n_prefix, _lib.ptr(self.ctx), self.n_ctx,
                  _lib.ptr(label), self.n_cls, _lib.ptr(self.token_suffix), self.token_suffix.shape[0], B, W,
                  _lib.ptr(out), _lib.ptr(bad), _lib.stream(self.device))
        if int(bad.item()):
            raise IndexError(f"label out of range for {self.n_cls} classes")
        return out

    __call__ = forward


class PromptLearner(_Learner):
    """coop.PromptLearner (coop.py:62-110): 3 context words + SOS in the prefix, 5 class
    tokens per identity (``cls_ctx``), the rest of the template as suffix."""
    n_prefix, n_ctx = 4, 5

    def __init__(self, num_class, clip_model, dataset_name="market1501", tokenized_prompts=None, cls_ctx=None, seed=0):
        super().__init__(num_class, clip_model, dataset_name, tokenized_prompts, cls_ctx, seed)
        self.num_class = num_class
        self.n_cls_ctx = self.n_ctx

    @property
    def cls_ctx(self):
        return self.ctx


class VLPromptLearner(_Learner):
    """maple.VLPromptLearner (maple.py:21-90): SOS + 4 context words in the prefix, 4 class
    context vectors per identity (``ctx``), the rest of the template as suffix."""
    n_prefix, n_ctx = 5, 4

    def __init__(self, n_cls, clip_model, dataset_name="market1501", tokenized_prompts=None, ctx=None, seed=0):
        super().__init__(n_cls, clip_model, dataset_name, tokenized_prompts, ctx, seed)

    def construct_prompts(self, ctx, prefix, suffix, label=None):
        """maple.py:57-78 on device tensors (shape op; forward() uses the HIP kernel)."""
        if label is not None:
            prefix, suffix = prefix[label], suffix[label]
        prefix = prefix.expand(ctx.size(0), -1, -1)
        suffix = suffix.expand(ctx.size(0), -1, -1)
        return torch.cat([prefix, ctx, suffix], dim=1)
