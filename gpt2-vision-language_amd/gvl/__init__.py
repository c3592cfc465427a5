"""gvl — MI355X-native hot path of theophile-lt/gpt2-vision-language.

Drop-in module APIs:
    gvl.gpt2       -> source/gpt2/train_gpt2.py model classes (GPT, GPTConfig, Block, ...)
    gvl.caption    -> source/gpt2_linear/model.py and source/gpt2_q_former/model.py
    gvl.cross_att  -> source/gpt2_cross-att/model.py
Runtime:
    gvl.optim (fused AdamW + clip), gvl.dist (bucketed RCCL all-reduce), gvl.train (the
    grad-accumulation DP step), gvl.generate (greedy decode), gvl.kernels (C-ABI wrappers).
All compute goes through libgvl.so (include/gvl.h); importing a module that needs it on a
machine without the built library raises at first use, there is no fallback.
"""
import os as _os

__version__ = "0.1.0"
PACKAGE_DIR = _os.path.dirname(_os.path.abspath(__file__))


def library_path():
    from . import _lib
    return _lib.LIB_PATH


def load_library():
    from . import _lib
    return _lib.load()
