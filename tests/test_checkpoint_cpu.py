"""Checkpoint loop (gvl.checkpoint) on CPU: the reference's file names, dict layout, atomic
rolling save, best tracking and resume (train_gpt2.py:307-328, :363-391, :495-508), and
weights_only loading of a checkpoint whose config is pickled as `__main__.GPTConfig` (the
reference train script defines GPTConfig in the script itself)."""
import dataclasses
import os
import sys

import torch

import gvl.gpt2 as g2
from gvl.checkpoint import CheckpointManager, load_checkpoint, restore_config
from tests.helpers import TINY


def _model():
    torch.manual_seed(0)
    return g2.GPT(g2.GPTConfig(**TINY))


def _opt(m):
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        return m.configure_optimizers(0.1, 1e-3, "cpu")  # torch AdamW on CPU (reference)


def _fake_step(m, opt, seed):
    g = torch.Generator().manual_seed(seed)
    opt.zero_grad()
    for p in m.parameters():
        p.grad = torch.randn(p.shape, generator=g) * 1e-2
    opt.step()


def test_rolling_best_final_and_resume(tmp_path):
    m = _model()
    opt = _opt(m)
    mgr = CheckpointManager(str(tmp_path), m, opt, save_every=2, ts="T")
    for step in range(5):
        _fake_step(m, opt, step)
        mgr.maybe_save_rolling(step, step == 4, val_loss=10.0 - step)
        mgr.save_best(step, 10.0 - step if step != 3 else 99.0)
    mgr.save_final(4, 6.0)
    names = sorted(os.listdir(tmp_path))
    assert names == ["model_best.pt", "model_final.pt", "model_last.pt"]  # no .tmp left
    last = load_checkpoint(mgr.last_path)
    assert set(last) == {"model", "optimizer", "config", "step", "val_loss", "ddp_world_size", "ts"}
    assert last["step"] == 4 and last["val_loss"] == 6.0 and last["ts"] == "T"
    assert isinstance(last["config"], g2.GPTConfig) and last["config"].n_embd == TINY["n_embd"]
    best = load_checkpoint(mgr.best_path)
    assert best["step"] == 4 and mgr.best_step == 4  # step 3 (val 99) did not replace it
    # resume into a fresh model + optimizer, in the reference's order
    m2 = _model()
    opt2 = _opt(m2)
    start = CheckpointManager(str(tmp_path), m2, opt2).resume()
    assert start == 5
    for (n, p), q in zip(m.named_parameters(), m2.parameters()):
        assert torch.equal(p, q), n
    _fake_step(m, opt, 77)
    _fake_step(m2, opt2, 77)
    for (n, p), q in zip(m.named_parameters(), m2.parameters()):
        assert torch.equal(p, q), n


def test_loads_reference_style_main_config(tmp_path):
    """A dict whose config was pickled as __main__.GPTConfig loads with weights_only=True."""
    main = sys.modules["__main__"]

    @dataclasses.dataclass
    class GPTConfig:  # the reference's script-level dataclass (train_gpt2.py:76-83)
        block_size: int = 1024
        vocab_size: int = 50257
        n_layer: int = 12
        n_head: int = 12
        n_embd: int = 768
    GPTConfig.__module__ = "__main__"
    GPTConfig.__qualname__ = "GPTConfig"
    had = hasattr(main, "GPTConfig")
    old = getattr(main, "GPTConfig", None)
    main.GPTConfig = GPTConfig
    try:
        path = str(tmp_path / "ref.pt")
        torch.save({"model": {"w": torch.ones(2)}, "config": GPTConfig(vocab_size=50304),
                    "step": 7}, path)
    finally:
        if had:
            main.GPTConfig = old
        else:
            del main.GPTConfig
    ck = load_checkpoint(path)
    cfg = restore_config(ck["config"])
    assert isinstance(cfg, g2.GPTConfig) and cfg.vocab_size == 50304 and ck["step"] == 7
