"""Drop-in for the `model_BLIP` module that source/gpt2_linear/train.py:9 imports."""
import os as _os
import sys as _sys

_PKG = _os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
if _PKG not in _sys.path:  # the gvl package (gpt2-vision-language_amd/)
    _sys.path.insert(0, _PKG)
from gvl.caption import (MLP, Block, CausalSelfAttention, GPT_previous, GPTConfig,  # noqa: F401
                         Linear_Bridge, pool_clip_197_to_33_avg_with_cls)
from gvl.caption import LinearCaption as GPT_Caption  # noqa: F401
