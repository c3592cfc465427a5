"""Checkpoint save / resume loop of the train scripts.

Reference behaviour restated (source/gpt2/train_gpt2.py:307-328 resume, :363-391 rolling and
best, :495-508 final; gpt2_linear/train.py:170-216 the same as functions):
  * one dict per file: model, optimizer, config, step, val_loss, ddp_world_size, ts;
  * rolling `model_last.pt` every `save_every` steps and at the last step (step > 0), written
    to `.model_last_step_{step:06d}.tmp` first and moved with os.replace (atomic);
  * `model_best.pt` whenever the validation loss improves; `model_final.pt` at the end;
  * resume: if model_last.pt exists, load the model then the optimizer state and continue
    at step + 1 (the order configure_optimizers -> load_state_dict of train_gpt2.py:320-322,
    which gvl.optim.AdamW honours: moments and fp32 masters move into its arenas).

Loading never unpickles code: torch.load(weights_only=True) with GPTConfig allow-listed
under every name the reference pickles it as (`__main__.GPTConfig` — the train scripts
define it in the script itself — and the model modules' own names).
"""
from __future__ import annotations

import os
import time

import torch

from .gpt2 import GPTConfig

# (class, pickled path) pairs the weights_only unpickler may build
_CONFIG_NAMES = ["__main__.GPTConfig", "model.GPTConfig", "model_BLIP.GPTConfig",
                 "train_gpt2.GPTConfig"]


def _safe_globals():
    from . import cross_att
    pairs = [(GPTConfig, n) for n in _CONFIG_NAMES]
    pairs.append((GPTConfig, f"{GPTConfig.__module__}.GPTConfig"))
    pairs.append((cross_att.GPTConfig, f"{cross_att.GPTConfig.__module__}.GPTConfig"))
    return pairs


def load_checkpoint(path, map_location=None):
    """torch.load(path, weights_only=True) accepting the reference's GPTConfig pickles.
    A reference checkpoint whose config is the cross-att GPTConfig (it has img_embd)
    round-trips as gvl.gpt2.GPTConfig; `restore_config` rebuilds the right class."""
    with torch.serialization.safe_globals(_safe_globals()):
        return torch.load(path, map_location=map_location, weights_only=True)


def restore_config(cfg):
    """Rebuild a GPTConfig-like object loaded under the pretrain name into the class whose
    fields it carries (cross-att adds img_embd)."""
    if cfg is None:
        return None
    fields = dict(vars(cfg))
    if "img_embd" in fields:
        from .cross_att import GPTConfig as XConfig
        return XConfig(**fields)
    return GPTConfig(**fields)


class CheckpointManager:
    """The reference train loops' checkpointing (file names, dict layout, atomic rolling
    save, best tracking, final save, resume).  Only the master process writes."""

    def __init__(self, ckpt_dir, raw_model, optimizer, *, ddp_world_size: int = 1,
                 master: bool = True, save_every: int = 2500, ts: str | None = None):
        self.dir = ckpt_dir
        self.model = raw_model
        self.opt = optimizer
        self.world = ddp_world_size
        self.master = master
        self.save_every = save_every
        self.ts = ts or time.strftime("%Y%m%d-%H%M%S")
        self.best_val = float("inf")
        self.best_step = 0
        self.last_path = os.path.join(ckpt_dir, "model_last.pt")
        self.best_path = os.path.join(ckpt_dir, "model_best.pt")
        self.final_path = os.path.join(ckpt_dir, "model_final.pt")
        if master:
            os.makedirs(ckpt_dir, exist_ok=True)

    def state(self, step, val_loss):
        """The checkpoint dict (train_gpt2.py:365-373)."""
        return {
            "model": self.model.state_dict(),
            "optimizer": self.opt.state_dict(),
            "config": getattr(self.model, "config", None),
            "step": step,
            "val_loss": None if val_loss is None else float(val_loss),
            "ddp_world_size": self.world,
            "ts": self.ts,
        }

    def save_rolling(self, step, val_loss):
        """Atomic model_last.pt: write a step-named .tmp, then os.replace."""
        if not self.master:
            return None
        tmp = os.path.join(self.dir, f".model_last_step_{step:06d}.tmp")
        torch.save(self.state(step, val_loss), tmp)
        os.replace(tmp, self.last_path)
        return self.last_path

    def maybe_save_rolling(self, step, last_step, val_loss):
        """train_gpt2.py:363: step > 0 and (step % SAVE_EVERY == 0 or last_step)."""
        if step > 0 and (step % self.save_every == 0 or last_step):
            return self.save_rolling(step, val_loss)
        return None

    def save_best(self, step, val_loss):
        """model_best.pt when val_loss improves (train_gpt2.py:378-391)."""
        if not self.master or not (float(val_loss) < self.best_val):
            return None
        self.best_val = float(val_loss)
        self.best_step = step
        torch.save(self.state(step, self.best_val), self.best_path)
        return self.best_path

    def save_final(self, step, val_loss=None):
        if not self.master:
            return None
        torch.save(self.state(step, val_loss), self.final_path)
        return self.final_path

    def resume(self, map_location=None) -> int:
        """Load model_last.pt if present into the model, then the optimizer; returns the step
        to start from (step + 1, or 0)."""
        if not os.path.isfile(self.last_path):
            return 0
        ckpt = load_checkpoint(self.last_path, map_location=map_location)
        self.model.load_state_dict(ckpt["model"])
        self.opt.load_state_dict(ckpt["optimizer"])
        return int(ckpt.get("step", 0)) + 1  # best_val restarts at inf, as in the reference
