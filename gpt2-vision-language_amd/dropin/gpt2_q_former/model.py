"""Drop-in for source/gpt2_q_former/model.py (BLIP-2-style Q-Former bridge)."""
import _gvl_path  # noqa: F401
from gvl.caption import (MLP, BLIP2Bridge, Block, CausalSelfAttention, GPT_previous,  # noqa: F401
                         GPTConfig, QFormerLayer, pool_clip_197_to_33_avg_with_cls)
from gvl.caption import QFormerCaption as GPT_Caption  # noqa: F401
