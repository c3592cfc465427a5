"""Drop-in for the model classes defined inline in source/gpt2/train_gpt2.py:21-144.
Replace those class definitions in the training script with
    from model import CausalSelfAttention, MLP, Block, GPTConfig, GPT
after putting this directory first on sys.path."""
import os as _os
import sys as _sys

_PKG = _os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
if _PKG not in _sys.path:  # the gvl package (gpt2-vision-language_amd/)
    _sys.path.insert(0, _PKG)
from gvl.gpt2 import GPT, MLP, Block, CausalSelfAttention, GPTConfig  # noqa: F401
