"""Shared test helpers: recipe weights, fixture comparison, model builders."""
from __future__ import annotations

import numpy as np
import torch

from oracle import models as OM
from oracle import weights as W

TINY = dict(block_size=64, vocab_size=512, n_layer=2, n_head=2, n_embd=128)


def recipe_params(keys_shapes, dtype=torch.float32, device="cpu"):
    """Parameter dict from the deterministic recipe, tied wte/lm_head as ONE tensor."""
    ks = [(k, tuple(s)) for k, s in keys_shapes if not k.endswith(".attn.bias")]
    vals = W.make_state(ks)
    P = {k: torch.from_numpy(v.copy()).to(dtype).to(device) for k, v in vals.items()}
    for k in list(P):
        if k.endswith("lm_head.weight"):
            kb = k[: -len("lm_head.weight")] + "transformer.wte.weight"
            if kb in P:
                P[kb] = P[k]
    if "gpt.transformer.wte.weight" in P:  # caption aliases
        P["wte.weight"] = P["gpt.transformer.wte.weight"]
        P["wpe.weight"] = P["gpt.transformer.wpe.weight"]
    return P


def margins_out(name, rec):
    """Write a parity test's measured errors as JSON under $GVL_MARGINS_DIR (default
    gpurun_out/parity_margins; the GPU session copies them into profiles/)."""
    import json
    import os
    d = os.environ.get("GVL_MARGINS_DIR", os.path.join("gpurun_out", "parity_margins"))
    try:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, f"{name}.json"), "w") as f:
            json.dump(rec, f, indent=1, default=float)
    except OSError:
        pass


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    den = max(np.abs(b).max(), 1e-30)
    return float(np.abs(a - b).max() / den)


def check_summary(fx, name, t, rtol):
    """Compare tensor t against the fixture summary of `name` (full or sampled + sums)."""
    a = t.detach().to(torch.float64).cpu().numpy().reshape(-1)
    if name + "#full" in fx:
        e = rel_err(a, fx[name + "#full"])
        assert e < rtol, f"{name}: rel err {e:.3g} >= {rtol}"
    else:
        idx = fx[name + "#idx"]
        e = rel_err(a[idx], fx[name + "#val"])
        assert e < rtol, f"{name}: sampled rel err {e:.3g} >= {rtol}"
    sq = float(fx[name + "#sq"])
    e2 = abs((a * a).sum() - sq) / max(sq, 1e-30)
    assert e2 < 2 * rtol, f"{name}: sum-of-squares rel err {e2:.3g}"


def fixture_name(kind, key):
    """Oracle canonical key for the tied embedding is lm_head.weight."""
    if kind == "gpt" and key == "transformer.wte.weight":
        return "lm_head.weight"
    return key


def named_trainable(kind, meta):
    keys = [k for k, _ in meta[f"{kind}_keys"]]
    if kind == "cross":
        return list(meta["cross_trainable"])
    if kind == "gpt":
        return [k for k in keys if not k.endswith(".attn.bias") and k != "lm_head.weight"]
    return [k for k in keys if k.startswith("bridge.")]


def lr_caption(it, max_lr=1e-3, min_lr=1e-4, warm=5, max_steps=80):
    return OM.O.get_lr(it, max_lr, min_lr, warm, max_steps)


def lr_lm(it):
    return OM.O.get_lr(it, 6e-4, 6e-5, 715, 19073)


def lr_cross(it):
    return OM.O.get_lr(it, 1e-3, 1e-5, 20, 925)
