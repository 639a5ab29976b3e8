"""Stand-in for OpenAI `clip` (absent offline).  Fixture-generation harness only."""
import torch

TOKENS = {}       # text -> int64 [77] token row, filled by make_goldens.py
LOAD_HOOK = None  # callable(name) -> model, installed by make_goldens.py


def tokenize(texts, context_length=77, truncate=False):
    if isinstance(texts, str):
        texts = [texts]
    return torch.stack([torch.as_tensor(TOKENS[t], dtype=torch.int64) for t in texts])


def load(name, *args, **kwargs):
    if LOAD_HOOK is None:
        raise RuntimeError("clip.load is unavailable offline")
    return LOAD_HOOK(name), None


def available_models():
    return ["RN50", "ViT-B/16", "ViT-L/14"]
