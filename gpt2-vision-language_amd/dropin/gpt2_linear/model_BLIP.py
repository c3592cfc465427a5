"""Drop-in for the `model_BLIP` module that source/gpt2_linear/train.py:9 imports."""
import _gvl_path  # noqa: F401
from gvl.caption import (MLP, Block, CausalSelfAttention, GPT_previous, GPTConfig,  # noqa: F401
                         Linear_Bridge, pool_clip_197_to_33_avg_with_cls)
from gvl.caption import LinearCaption as GPT_Caption  # noqa: F401
