"""Drop-in for the model classes defined inline in source/gpt2/train_gpt2.py:21-144.
Replace those class definitions in the training script with
    from model import CausalSelfAttention, MLP, Block, GPTConfig, GPT
after putting this directory first on sys.path."""
import _gvl_path  # noqa: F401
from gvl.gpt2 import GPT, MLP, Block, CausalSelfAttention, GPTConfig  # noqa: F401
