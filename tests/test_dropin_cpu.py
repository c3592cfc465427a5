"""The drop-in shims expose exactly the names the reference's train scripts import
(SURVEY.md §8b): `from model import ...` / `from model_BLIP import ...` resolve to gvl."""
import importlib
import os
import sys

import pytest

from tests.conftest import PKG

WANT = {
    "gpt2": ["CausalSelfAttention", "MLP", "Block", "GPTConfig", "GPT"],
    "gpt2_linear": ["GPTConfig", "GPT_previous", "GPT_Caption", "pool_clip_197_to_33_avg_with_cls",
                    "Linear_Bridge"],
    "gpt2_q_former": ["GPTConfig", "GPT_previous", "GPT_Caption",
                      "pool_clip_197_to_33_avg_with_cls", "BLIP2Bridge", "QFormerLayer"],
    "gpt2_cross-att": ["GPT", "GPTConfig", "pool_clip_197_to_33_avg_with_cls", "CrossAttention",
                       "Vision_projector"],
}


@pytest.mark.parametrize("d", sorted(WANT))
def test_dropin_names(d):
    path = os.path.join(PKG, "dropin", d)
    mods = ["model"] + (["model_BLIP"] if d in ("gpt2_linear", "gpt2_q_former") else [])
    sys.path.insert(0, path)
    try:
        for name in mods:
            sys.modules.pop(name, None)
            m = importlib.import_module(name)
            for sym in WANT[d]:
                assert hasattr(m, sym), (d, name, sym)
            if d == "gpt2_q_former":
                from gvl.caption import BLIP2Bridge
                assert m.GPT_Caption.bridge_cls is BLIP2Bridge
            sys.modules.pop(name, None)
    finally:
        sys.path.remove(path)
        sys.modules.pop("_gvl_path", None)
