"""Drop-in for the `model_BLIP` module that source/gpt2_q_former/train.py:9 imports."""
import _gvl_path  # noqa: F401
from gvl.caption import (MLP, BLIP2Bridge, Block, CausalSelfAttention, GPT_previous,  # noqa: F401
                         GPTConfig, QFormerLayer, pool_clip_197_to_33_avg_with_cls)
from gvl.caption import QFormerCaption as GPT_Caption  # noqa: F401
