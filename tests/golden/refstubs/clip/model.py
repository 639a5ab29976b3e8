"""clip.model blocks: the reference's custom_clip_model.py holds the same math."""
from custom_clip_model import LayerNorm, QuickGELU, ResidualAttentionBlock, Transformer, ModifiedResNet  # noqa: F401
