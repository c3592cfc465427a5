"""Drop-in for source/gpt2_cross-att/model.py (gated cross-attention bridge)."""
import os as _os
import sys as _sys

_PKG = _os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
if _PKG not in _sys.path:  # the gvl package (gpt2-vision-language_amd/)
    _sys.path.insert(0, _PKG)
from gvl.cross_att import (GPT, MLP, Block, CausalSelfAttention, CrossAttention,  # noqa: F401
                           GPTConfig, Vision_projector, pool_clip_197_to_33_avg_with_cls)
