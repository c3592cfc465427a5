"""Drop-in for source/gpt2_cross-att/model.py (gated cross-attention bridge)."""
import _gvl_path  # noqa: F401
from gvl.cross_att import (GPT, MLP, Block, CausalSelfAttention, CrossAttention,  # noqa: F401
                           GPTConfig, Vision_projector, pool_clip_197_to_33_avg_with_cls)
