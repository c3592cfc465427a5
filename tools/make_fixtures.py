"""Generate golden fixtures from the REFERENCE model code (runs only in the build
container, where /root/reference exists; the reference never travels).

Loads (read-only, at run time):
  * source/gpt2/train_gpt2.py classes by AST-extracting the ClassDefs of lines 21-144
    (the script itself is top-level code with missing deps);
  * source/gpt2_linear/model.py, source/gpt2_q_former/model.py,
    source/gpt2_cross-att/model.py via importlib.
Weights come from the library-independent recipe in oracle/weights.py; bridges run in
eval() (dropout off) but still take gradients; cross_gate is non-zero.

Writes tests/golden/*.npz (+ meta.json).  Usage: python tools/make_fixtures.py [--full]
"""
from __future__ import annotations

import argparse
import ast
import importlib.util
import inspect
import json
import math
import os
import sys
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import weights as W  # noqa: E402

REF = "/root/reference/source"
OUT = os.path.join(ROOT, "tests", "golden")

TINY = dict(block_size=64, vocab_size=512, n_layer=2, n_head=2, n_embd=128)
N_SAMPLE = 256


def load_gpt2_classes():
    path = os.path.join(REF, "gpt2", "train_gpt2.py")
    src = open(path).read()
    tree = ast.parse(src)
    keep = [n for n in tree.body if isinstance(n, ast.ClassDef)
            and n.name in ("CausalSelfAttention", "MLP", "Block", "GPTConfig", "GPT")]
    mod = ast.Module(body=keep, type_ignores=[])
    ns = dict(torch=torch, nn=nn, F=F, math=math, inspect=inspect, dataclass=dataclass)
    exec(compile(mod, path, "exec"), ns)
    return ns


def load_module(sub, name):
    path = os.path.join(REF, sub, "model.py")
    spec = importlib.util.spec_from_file_location(name, path)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def set_recipe(model, salt=0):
    sd = model.state_dict()
    vals = W.make_state([(k, tuple(v.shape)) for k, v in sd.items()
                         if not k.endswith(".attn.bias")], salt)
    # GPT_Caption's alias entries share storage with the decoder's embeddings
    for alias, src in (("wte.weight", "gpt.transformer.wte.weight"),
                       ("wpe.weight", "gpt.transformer.wpe.weight")):
        if alias in vals and src in vals:
            vals[alias] = vals[src]
    new = {}
    for k, v in sd.items():
        if k in vals:
            new[k] = torch.from_numpy(vals[k].copy()).to(v.dtype)
        else:
            new[k] = v
    # tied: keep wte == lm_head (recipe already aliases lm_head -> wte)
    model.load_state_dict(new, strict=True)
    return model


def summarize(name, t, out):
    a = t.detach().to(torch.float64).numpy().reshape(-1)
    out[name + "#sum"] = np.array(a.sum())
    out[name + "#sq"] = np.array((a * a).sum())
    if a.size <= 20000:
        out[name + "#full"] = a.astype(np.float32)
    else:
        idx = (W.make_ids(N_SAMPLE, a.size, W.key_seed(name)) % a.size).astype(np.int64)
        out[name + "#idx"] = idx
        out[name + "#val"] = a[idx].astype(np.float32)


def inputs_lm(B, T, V, seed):
    ids = torch.from_numpy(W.make_ids(B * T + 1, V, seed))
    return ids[:-1].view(B, T).clone(), ids[1:].view(B, T).clone()


def inputs_caption(B, L, D, T, V, seed):
    z = torch.from_numpy(W.make_normal_like(B * L * D, seed)).view(B, L, D)
    ids = torch.from_numpy(W.make_ids(B * (T + 1), V, seed + 7)).view(B, T + 1)
    lens = torch.tensor([max(2, T - 3 * (b % 8)) for b in range(B)])
    x, y = ids[:, :-1].clone(), ids[:, 1:].clone()
    mask = torch.arange(T).unsqueeze(0) < lens.unsqueeze(1)
    return z, x, y, mask


def run_train(model, loss_of, n_steps, lr_of, fused_ok=False):
    opt = model.configure_optimizers(weight_decay=0.1, learning_rate=lr_of(0), device="cpu")
    losses, norms = [], []
    for it in range(n_steps):
        opt.zero_grad()
        loss = loss_of(model)
        loss.backward()
        norm = torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        for g in opt.param_groups:
            g["lr"] = lr_of(it)
        opt.step()
        losses.append(float(loss))
        norms.append(float(norm))
    return losses, norms


def lr_caption(it, max_lr=1e-3, min_lr=1e-4, warm=5, max_steps=80):
    if it < warm:
        return max_lr * (it + 1) / warm
    ratio = (it - warm) / (max_steps - warm)
    return min_lr + 0.5 * (1 + math.cos(math.pi * ratio)) * (max_lr - min_lr)


def lr_lm(it, max_lr=6e-4, min_lr=6e-5, warm=715, max_steps=19073):
    if it < warm:
        return max_lr * (it + 1) / warm
    ratio = (it - warm) / (max_steps - warm)
    return min_lr + 0.5 * (1 + math.cos(math.pi * ratio)) * (max_lr - min_lr)


def greedy(fn, prompt, n):
    x = prompt
    toks, margins = [], []
    with torch.no_grad():
        for _ in range(n):
            last = fn(x)[:, -1, :]
            t2 = torch.topk(last, 2, dim=-1)
            margins.append(t2.values[:, 0] - t2.values[:, 1])
            nxt = torch.argmax(last, dim=-1, keepdim=True)
            toks.append(nxt)
            x = torch.cat([x, nxt], 1)
    return torch.cat(toks, 1), torch.stack(margins, 1)


def init_sums(model):
    return {k: float(v.double().sum()) for k, v in model.state_dict().items()}


def fixture_gpt(g2, meta):
    cfg = g2["GPTConfig"](**TINY)
    torch.manual_seed(0)
    model = g2["GPT"](cfg)
    meta["gpt_init_sums_seed0"] = init_sums(model)
    meta["gpt_keys"] = [[k, list(v.shape)] for k, v in model.state_dict().items()]
    set_recipe(model)
    x, y = inputs_lm(2, 48, TINY["vocab_size"], 101)
    out = {"x": x.numpy(), "y": y.numpy()}
    logits, loss = model(x, y)
    out["logits"] = logits.detach().numpy()
    out["loss"] = np.array(float(loss))
    loss.backward()
    for n, p in model.named_parameters():
        summarize("grad:" + n, p.grad, out)
    model.zero_grad()
    losses, norms = run_train(model, lambda m: m(x, y)[1], 3, lr_lm)
    out["train_losses"] = np.array(losses)
    out["train_norms"] = np.array(norms)
    for n, p in model.named_parameters():
        summarize("step3:" + n, p.data, out)
    set_recipe(model)
    toks, margins = greedy(lambda s: model(s)[0], x[:1, :8], 16)
    out["greedy_prompt"] = x[:1, :8].numpy()
    out["greedy_tokens"] = toks.numpy()
    out["greedy_margins"] = margins.numpy()
    np.savez(os.path.join(OUT, "gpt_tiny.npz"), **out)


def fixture_caption(mod, kind, meta, m_vis):
    cfg = mod.GPTConfig(**TINY)
    torch.manual_seed(0)
    lm = mod.GPT_previous(cfg)
    model = mod.GPT_Caption(enc_dim=TINY["n_embd"], lm=lm, m_vis_tokens=m_vis)
    meta[f"{kind}_init_sums_seed0"] = init_sums(model)
    meta[f"{kind}_keys"] = [[k, list(v.shape)] for k, v in model.state_dict().items()]
    set_recipe(model)
    model.eval()  # dropout off; gradients still flow
    B, T = 2, 24
    z_raw, x, y, mask = inputs_caption(B, 257, TINY["n_embd"], T, TINY["vocab_size"], 202)
    labels = y.masked_fill(~mask, -100)
    z = mod.pool_clip_197_to_33_avg_with_cls(z_raw)
    out = {"z_raw": z_raw.numpy(), "z": z.numpy(), "x": x.numpy(), "y": y.numpy(),
           "mask": mask.numpy(), "labels": labels.numpy()}
    logits, loss = model(z, x, labels=labels)
    out["logits"] = logits.detach().numpy()
    out["loss"] = np.array(float(loss))
    loss.backward()
    for n, p in model.named_parameters():
        if p.requires_grad:
            summarize("grad:" + n, p.grad, out)
    model.zero_grad()
    losses, norms = run_train(model, lambda m: m(z, x, labels=labels)[1], 3, lr_caption)
    out["train_losses"] = np.array(losses)
    out["train_norms"] = np.array(norms)
    for n, p in model.named_parameters():
        if p.requires_grad:
            summarize("step3:" + n, p.data, out)
    set_recipe(model)
    model.eval()
    toks, margins = greedy(lambda s: model(z[:1], s)[0], x[:1, :3], 16)
    out["greedy_prompt"] = x[:1, :3].numpy()
    out["greedy_tokens"] = toks.numpy()
    out["greedy_margins"] = margins.numpy()
    np.savez(os.path.join(OUT, f"{kind}_tiny.npz"), **out)


def fixture_cross(mod, meta):
    cfg = mod.GPTConfig(**TINY, img_embd=TINY["n_embd"])
    torch.manual_seed(0)
    model = mod.GPT(cfg)
    meta["cross_init_sums_seed0"] = init_sums(model)
    meta["cross_keys"] = [[k, list(v.shape)] for k, v in model.state_dict().items()]
    meta["cross_trainable"] = [n for n, p in model.named_parameters() if p.requires_grad]
    set_recipe(model)
    B, T = 2, 24
    z_raw, x, y, mask = inputs_caption(B, 197, TINY["n_embd"], T, TINY["vocab_size"], 303)
    z = mod.pool_clip_197_to_33_avg_with_cls(z_raw)
    out = {"z_raw": z_raw.numpy(), "z": z.numpy(), "x": x.numpy(), "y": y.numpy(),
           "mask": mask.numpy()}
    logits, loss = model(x, z=z, targets=y, target_mask=mask)
    out["logits"] = logits.detach().numpy()
    out["loss"] = np.array(float(loss))
    loss.backward()
    for n, p in model.named_parameters():
        if p.requires_grad:
            summarize("grad:" + n, p.grad, out)
    model.zero_grad()
    losses, norms = run_train(model, lambda m: m(x, z=z, targets=y, target_mask=mask)[1], 3,
                              lambda it: lr_caption(it, 1e-3, 1e-5, 20, 925))
    out["train_losses"] = np.array(losses)
    out["train_norms"] = np.array(norms)
    for n, p in model.named_parameters():
        if p.requires_grad:
            summarize("step3:" + n, p.data, out)
    set_recipe(model)
    toks, margins = greedy(lambda s: model(s, z=z[:1])[0], x[:1, :3], 16)
    out["greedy_prompt"] = x[:1, :3].numpy()
    out["greedy_tokens"] = toks.numpy()
    out["greedy_margins"] = margins.numpy()
    # unmasked-loss variant too
    _, loss_plain = model(x, z=z, targets=y)
    out["loss_unmasked"] = np.array(float(loss_plain))
    np.savez(os.path.join(OUT, "cross_tiny.npz"), **out)


def fixture_ops(lin_mod):
    out = {}
    torch.manual_seed(1234)
    # causal / non-causal SDPA fwd+bwd
    for name, (B, H, Tq, Tk, causal) in {"sdpa_causal": (2, 2, 80, 80, True),
                                         "sdpa_cross": (2, 2, 31, 33, False),
                                         "sdpa_self32": (2, 2, 32, 32, False)}.items():
        q = torch.randn(B, H, Tq, 64, requires_grad=True)
        k = torch.randn(B, H, Tk, 64, requires_grad=True)
        v = torch.randn(B, H, Tk, 64, requires_grad=True)
        o = F.scaled_dot_product_attention(q, k, v, is_causal=causal)
        do = torch.randn_like(o)
        o.backward(do)
        for t, nm in ((q, "q"), (k, "k"), (v, "v"), (o, "o"), (do, "do")):
            out[f"{name}:{nm}"] = t.detach().numpy()
        for t, nm in ((q, "dq"), (k, "dk"), (v, "dv")):
            out[f"{name}:{nm}"] = t.grad.numpy()
    # pool at side 16 (uniform windows) and side 14 (overlapping windows)
    for side in (16, 14):
        tok = torch.randn(2, 1 + side * side, 96)
        out[f"pool{side}:in"] = tok.numpy()
        out[f"pool{side}:out"] = lin_mod.pool_clip_197_to_33_avg_with_cls(tok).numpy()
    # layernorm, gelus
    x = torch.randn(37, 128)
    w, b = torch.randn(128), torch.randn(128)
    out["ln:x"], out["ln:w"], out["ln:b"] = x.numpy(), w.numpy(), b.numpy()
    out["ln:y"] = F.layer_norm(x, (128,), w, b, 1e-5).numpy()
    g = torch.randn(4096) * 3
    out["gelu:x"] = g.numpy()
    out["gelu:tanh"] = nn.GELU(approximate="tanh")(g).numpy()
    out["gelu:erf"] = nn.GELU()(g).numpy()
    # CE with ignore_index and masked mean
    lg = torch.randn(40, 512)
    tg = torch.randint(0, 512, (40,))
    tg[::7] = -100
    out["ce:logits"], out["ce:targets"] = lg.numpy(), tg.numpy()
    out["ce:loss"] = np.array(float(F.cross_entropy(lg, tg, ignore_index=-100)))
    mk = torch.rand(40) > 0.3
    tg2 = torch.randint(0, 512, (40,))
    per = F.cross_entropy(lg, tg2, reduction="none") * mk
    out["ce:targets2"], out["ce:mask"] = tg2.numpy(), mk.numpy()
    out["ce:masked_loss"] = np.array(float(per.sum() / mk.sum().clamp_min(1)))
    # AdamW (2 steps, two groups) + clip
    p1 = torch.randn(64, 32)
    p2 = torch.randn(32)
    ps = [p1.clone().requires_grad_(True), p2.clone().requires_grad_(True)]
    opt = torch.optim.AdamW([{"params": [ps[0]], "weight_decay": 0.1},
                             {"params": [ps[1]], "weight_decay": 0.0}], lr=1e-3,
                            betas=(0.9, 0.95), eps=1e-8)
    grads = [torch.randn(64, 32) * 0.5, torch.randn(32) * 0.5]
    norms = []
    for it in range(2):
        opt.zero_grad()
        ps[0].grad = grads[0].clone() * (it + 1)
        ps[1].grad = grads[1].clone() * (it + 1)
        norms.append(float(torch.nn.utils.clip_grad_norm_(ps, 1.0)))
        opt.step()
    out["adam:p1"], out["adam:p2"] = p1.numpy(), p2.numpy()
    out["adam:g1"], out["adam:g2"] = grads[0].numpy(), grads[1].numpy()
    out["adam:p1_after"], out["adam:p2_after"] = ps[0].detach().numpy(), ps[1].detach().numpy()
    out["adam:norms"] = np.array(norms)
    np.savez(os.path.join(OUT, "ops.npz"), **out)


def fixture_full(g2, qf_mod, meta):
    """Full-size 124M scalars (weights regenerate from the recipe on the GPU box)."""
    out = {}
    cfg = g2["GPTConfig"](vocab_size=50304)
    model = set_recipe(g2["GPT"](cfg))
    x, y = inputs_lm(1, 1024, 50257, 404)
    logits, loss = model(x, y)
    loss.backward()
    norm = torch.sqrt(sum((p.grad.double() ** 2).sum() for p in model.parameters()))
    out["lm_loss"] = np.array(float(loss))
    out["lm_gradnorm"] = np.array(float(norm))
    out["lm_x"], out["lm_y"] = x.numpy(), y.numpy()
    out["lm_last_logits"] = logits[0, -1].detach().numpy()
    del model, logits
    cfg = qf_mod.GPTConfig(vocab_size=50304, block_size=1024)
    lm = qf_mod.GPT_previous(cfg)
    model = set_recipe(qf_mod.GPT_Caption(enc_dim=768, lm=lm, m_vis_tokens=32))
    model.eval()
    z_raw, x, yy, mask = inputs_caption(2, 257, 768, 31, 50257, 505)
    labels = yy.masked_fill(~mask, -100)
    z = qf_mod.pool_clip_197_to_33_avg_with_cls(z_raw)
    _, loss = model(z, x, labels=labels)
    loss.backward()
    norm = torch.sqrt(sum((p.grad.double() ** 2).sum() for p in model.parameters()
                          if p.grad is not None))
    out["qf_loss"] = np.array(float(loss))
    out["qf_gradnorm"] = np.array(float(norm))
    out["qf_x"], out["qf_labels"] = x.numpy(), labels.numpy()
    out["qf_z_seed"] = np.array(505)
    np.savez(os.path.join(OUT, "full124m.npz"), **out)


# ------------------------------------------------------------------ round-2 fixtures
N_SAMPLE_FULL = 512
CAP_B = 16


def sample_tensor(key, t, out, name):
    """Values of t at a key-determined index sample (the same sample for every quantity
    of one parameter, so grads, params and updates line up), plus sum of squares."""
    a = t.detach().to(torch.float64).numpy().reshape(-1)
    out[name + "#sq"] = np.array((a * a).sum())
    if a.size <= 4096:
        out[name + "#full"] = a.astype(np.float32)
    else:
        idx = (W.make_ids(N_SAMPLE_FULL, a.size, W.key_seed(key)) % a.size).astype(np.int64)
        out[name + "#idx"] = idx.astype(np.int32)
        out[name + "#val"] = a[idx].astype(np.float32)


def round_bf16_(model):
    """Give the reference model the bf16-valued weights the GPU model holds (fp32 math):
    'identical inputs' for the decode parity (train_gpt2.py:440-449)."""
    with torch.no_grad():
        for p in model.parameters():
            p.copy_(p.to(torch.bfloat16).float())
    return model


class _Bf16Weights:
    """Run the enclosed forward/backward on bf16-rounded copies of the (fp32 master)
    weights, restoring the masters afterwards: the mixed-precision loop gvl trains with
    (bf16 compute weights, fp32 master weights + moments), with the reference's own model
    code and autograd computing every loss and gradient."""

    def __init__(self, model, on):
        self.model, self.on = model, on

    def __enter__(self):
        if self.on:
            self.saved = [p.detach().clone() for p in self.model.parameters()]
            with torch.no_grad():
                for p in self.model.parameters():
                    p.copy_(p.to(torch.bfloat16).float())
        return self

    def __exit__(self, *exc):
        if self.on:
            with torch.no_grad():
                for p, s in zip(self.model.parameters(), self.saved):
                    p.copy_(s)


def train_ref(model, micro_batches, loss_of, n_steps, lr, out, pre, names, mp=False):
    """The reference optimizer step (train_gpt2.py:457-476 / gpt2_linear/train.py:292-322):
    zero_grad; per micro-step loss/accum + backward; clip_grad_norm_(1.0); lr; AdamW.
    mp=True: the same loop in mixed precision (_Bf16Weights), masters starting at the
    bf16-rounded initial weights — identical inputs to the GPU model at every step."""
    if mp:
        round_bf16_(model)
    opt = model.configure_optimizers(weight_decay=0.1, learning_rate=lr, device="cpu")
    params = dict(model.named_parameters())
    accum = len(micro_batches)
    losses, norms = [], []
    for step in range(n_steps):
        opt.zero_grad()
        la = 0.0
        with _Bf16Weights(model, mp):
            for mb in micro_batches:
                loss = loss_of(model, mb) / accum
                la += float(loss.detach())
                loss.backward()
        if step == 0:
            for n in names:
                sample_tensor(n, params[n].grad, out, f"{pre}grad:{n}")
        norm = torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        for g in opt.param_groups:
            g["lr"] = lr
        opt.step()
        losses.append(la)
        norms.append(float(norm))
        for n in names:
            sample_tensor(n, params[n].data, out, f"{pre}step{step + 1}:{n}")
    with torch.no_grad(), _Bf16Weights(model, mp):
        out[pre + "loss_after"] = np.array(float(loss_of(model, micro_batches[0])))
    out[pre + "losses"] = np.array(losses)
    out[pre + "norms"] = np.array(norms)


def fixture_full_train(g2, lin, qf, xa, meta):
    """Full-size (124M) training-step parity: 2 optimizer steps of the reference loop.
    LM: 2 accumulated micro-steps of B=1x1024 each (CFG2's accumulation path at B=1);
    linear / Q-Former / cross-att caption models at B=16 (~350 loss rows, so bf16 rounding
    of single logits averages out as in the B=128 training batches).  lr fixed at each config's
    max_lr (at warmup step 0 the LM update, 8.4e-7, is below bf16 resolution)."""
    out = {}
    cfg = g2["GPTConfig"](vocab_size=50304)
    model = set_recipe(g2["GPT"](cfg))
    mbs = [inputs_lm(1, 1024, 50257, s) for s in (404, 405)]
    for i, (x, y) in enumerate(mbs):
        out[f"lm_x{i}"], out[f"lm_y{i}"] = x.numpy(), y.numpy()
    names = [n for n, p in model.named_parameters() if p.requires_grad]
    meta["full_lm_trainable"] = names
    train_ref(model, mbs, lambda m, b: m(b[0], b[1])[1], 2, 6e-4, out, "lm_", names)
    print("lm", out["lm_losses"], out["lm_norms"], out["lm_loss_after"], flush=True)
    model = set_recipe(g2["GPT"](cfg))
    train_ref(model, mbs, lambda m, b: m(b[0], b[1])[1], 2, 6e-4, out, "mp_lm_", names, mp=True)
    print("mp lm", out["mp_lm_losses"], out["mp_lm_norms"], out["mp_lm_loss_after"], flush=True)
    del model
    for kind, mod in (("linear", lin), ("qformer", qf)):
        lm = mod.GPT_previous(mod.GPTConfig(vocab_size=50304, block_size=1024))
        model = set_recipe(mod.GPT_Caption(enc_dim=768, lm=lm, m_vis_tokens=32))
        model.eval()  # dropout off; gradients still flow
        z_raw, x, yy, mask = inputs_caption(CAP_B, 257, 768, 31, 50257, 606)
        labels = yy.masked_fill(~mask, -100)
        z = mod.pool_clip_197_to_33_avg_with_cls(z_raw)
        out[f"{kind}_x"], out[f"{kind}_labels"] = x.numpy(), labels.numpy()
        names = [n for n, p in model.named_parameters() if p.requires_grad]
        meta[f"full_{kind}_trainable"] = names
        for pre, mp in ((f"{kind}_", False), (f"mp_{kind}_", True)):
            lm = mod.GPT_previous(mod.GPTConfig(vocab_size=50304, block_size=1024))
            model = set_recipe(mod.GPT_Caption(enc_dim=768, lm=lm, m_vis_tokens=32))
            model.eval()
            train_ref(model, [(z, x, labels)], lambda m, b: m(b[0], b[1], labels=b[2])[1], 2,
                      1e-3, out, pre, names, mp=mp)
            print(pre, out[pre + "losses"], out[pre + "norms"], out[pre + "loss_after"],
                  flush=True)
        del model, lm
    model = set_recipe(xa.GPT(xa.GPTConfig(vocab_size=50304, block_size=1024)))
    z_raw, x, yy, mask = inputs_caption(CAP_B, 257, 768, 31, 50257, 707)
    z = xa.pool_clip_197_to_33_avg_with_cls(z_raw)
    out["cross_x"], out["cross_y"], out["cross_mask"] = x.numpy(), yy.numpy(), mask.numpy()
    names = [n for n, p in model.named_parameters() if p.requires_grad]
    meta["full_cross_trainable"] = names
    for pre, mp in (("cross_", False), ("mp_cross_", True)):
        model = set_recipe(xa.GPT(xa.GPTConfig(vocab_size=50304, block_size=1024)))
        train_ref(model, [(z, x, yy, mask)],
                  lambda m, b: m(b[1], z=b[0], targets=b[2], target_mask=b[3])[1], 2, 1e-3, out,
                  pre, names, mp=mp)
        print(pre, out[pre + "losses"], out[pre + "norms"], out[pre + "loss_after"], flush=True)
    out["z_seeds"] = np.array([606, 707])
    out["cap_batch"] = np.array(CAP_B)
    np.savez_compressed(os.path.join(OUT, "full_train.npz"), **out)


def fixture_accum(g2, qf, meta):
    """Gradient accumulation over 4 micro-steps (the CFG2/CFG3 micro-loop, train_gpt2.py:
    460-469) and 2 optimizer steps, tiny configs: GPT and the Q-Former caption model
    (mixed-precision loop: bf16 compute weights, fp32 masters — train_ref(mp=True))."""
    out = {}
    cfg = g2["GPTConfig"](**TINY)
    model = set_recipe(g2["GPT"](cfg))
    mbs = [inputs_lm(2, 48, TINY["vocab_size"], 900 + i) for i in range(4)]
    for i, (x, y) in enumerate(mbs):
        out[f"gpt_x{i}"], out[f"gpt_y{i}"] = x.numpy(), y.numpy()
    names = [n for n, p in model.named_parameters() if p.requires_grad]
    train_ref(model, mbs, lambda m, b: m(b[0], b[1])[1], 2, 1e-3, out, "gpt_", names, mp=True)
    lm = qf.GPT_previous(qf.GPTConfig(**TINY))
    model = set_recipe(qf.GPT_Caption(enc_dim=TINY["n_embd"], lm=lm, m_vis_tokens=32))
    model.eval()
    mbs = []
    for i in range(4):
        z_raw, x, yy, mask = inputs_caption(2, 257, TINY["n_embd"], 24, TINY["vocab_size"], 950 + i)
        labels = yy.masked_fill(~mask, -100)
        mbs.append((qf.pool_clip_197_to_33_avg_with_cls(z_raw), x, labels))
        out[f"qformer_x{i}"], out[f"qformer_labels{i}"] = x.numpy(), labels.numpy()
    names = [n for n, p in model.named_parameters() if p.requires_grad]
    train_ref(model, mbs, lambda m, b: m(b[0], b[1], labels=b[2])[1], 2, 1e-3, out, "qformer_",
              names, mp=True)
    out["qformer_z_seeds"] = np.array([950 + i for i in range(4)])
    np.savez_compressed(os.path.join(OUT, "accum_tiny.npz"), **out)


def fixture_edge(lin, qf, xa, meta):
    """Reference edge cases: use_cls_only (M=1; Q-Former cross-attention over Tk=1),
    2-D patch_tokens, M+T > block_size truncation (gpt2_linear/model.py:181-196), and the
    cross-att GPT with z=None (gpt2_cross-att/model.py:159-165)."""
    out = {}
    z_raw, x, yy, mask = inputs_caption(2, 257, TINY["n_embd"], 24, TINY["vocab_size"], 202)
    labels = yy.masked_fill(~mask, -100)
    ids_long = torch.from_numpy(W.make_ids(2 * 41, TINY["vocab_size"], 808)).view(2, 41)
    x_long, y_long = ids_long[:, :-1].clone(), ids_long[:, 1:].clone()
    out["x_long"], out["y_long"] = x_long.numpy(), y_long.numpy()
    for kind, mod in (("linear", lin), ("qformer", qf)):
        z = mod.pool_clip_197_to_33_avg_with_cls(z_raw)
        cases = {
            "cls": (dict(use_cls_only=True), lambda m: m(z, x, labels=labels)),
            "patch2d": (dict(), lambda m: m(z[:, 0], x, labels=labels)),
            "trunc": (dict(), lambda m: m(z, x_long, labels=y_long)),
        }
        for case, (kw, fn) in cases.items():
            lm = mod.GPT_previous(mod.GPTConfig(**TINY))
            model = set_recipe(mod.GPT_Caption(enc_dim=TINY["n_embd"], lm=lm, m_vis_tokens=32, **kw))
            model.eval()
            logits, loss = fn(model)
            loss.backward()
            pre = f"{kind}_{case}_"
            out[pre + "loss"] = np.array(float(loss))
            out[pre + "logits_shape"] = np.array(logits.shape)
            out[pre + "logits_sq"] = np.array(float((logits.double() ** 2).sum()))
            for n, p in model.named_parameters():
                if p.requires_grad:
                    sample_tensor(n, p.grad, out, pre + "grad:" + n)
            print(pre, float(loss), tuple(logits.shape), flush=True)
    model = set_recipe(xa.GPT(xa.GPTConfig(**TINY, img_embd=TINY["n_embd"])))
    logits, loss = model(x, z=None, targets=yy)
    out["cross_noz_loss"] = np.array(float(loss))
    out["cross_noz_logits_sq"] = np.array(float((logits.double() ** 2).sum()))
    out["x"], out["y"], out["labels"] = x.numpy(), yy.numpy(), labels.numpy()
    out["z_seed"] = np.array(202)
    np.savez_compressed(os.path.join(OUT, "edge_tiny.npz"), **out)


def fixture_greedy(g2, lin, qf, xa, meta):
    """Greedy decode of the reference models on the bf16-valued weights the GPU model
    holds (fp32 math): tiny configs of all four models and the full-size 124M LM, linear,
    Q-Former and cross-att models.  16 new tokens each, with top-1/top-2 margins."""
    out = {}

    def run(pre, fn, prompt):
        toks, margins = greedy(fn, prompt, 16)
        out[pre + "prompt"] = prompt.numpy()
        out[pre + "tokens"] = toks.numpy()
        out[pre + "margins"] = margins.numpy()
        print(pre, toks.tolist(), np.round(margins.numpy(), 3).tolist(), flush=True)

    for size, cfg_kw, B_lm in (("tiny", TINY, None), ("full", dict(vocab_size=50304), None)):
        V = cfg_kw.get("vocab_size")
        D = cfg_kw.get("n_embd", 768)
        model = round_bf16_(set_recipe(g2["GPT"](g2["GPTConfig"](**cfg_kw))))
        x, _ = inputs_lm(1, 24, min(V, 50257), 1111)
        run(f"{size}_gpt_", lambda s: model(s)[0], x[:, :8])
        z_raw, xc, _, _ = inputs_caption(1, 257, D, 8, min(V, 50257), 1212)
        for kind, mod in (("linear", lin), ("qformer", qf)):
            c = dict(cfg_kw)
            c.setdefault("block_size", 1024)
            lm = mod.GPT_previous(mod.GPTConfig(**c))
            m = round_bf16_(set_recipe(mod.GPT_Caption(enc_dim=D, lm=lm, m_vis_tokens=32)))
            m.eval()
            z = mod.pool_clip_197_to_33_avg_with_cls(z_raw)
            run(f"{size}_{kind}_", lambda s: m(z, s)[0], xc[:, :3])
        c = dict(cfg_kw)
        if size == "tiny":
            c["img_embd"] = D
        m = round_bf16_(set_recipe(xa.GPT(xa.GPTConfig(**c))))
        z = xa.pool_clip_197_to_33_avg_with_cls(z_raw)
        run(f"{size}_cross_", lambda s: m(s, z=z)[0], xc[:, :3])
        del model, m
    out["z_seed"] = np.array(1212)
    np.savez_compressed(os.path.join(OUT, "greedy.npz"), **out)


BENCH_CAP_B = 128   # bench.py caption batch
BENCH_LM_B = 16     # bench.py LM micro-batch (configs[1])


def _grads_out(model, names, out, pre):
    params = dict(model.named_parameters())
    sq = 0.0
    for n in names:
        g = params[n].grad
        sample_tensor(n, g, out, f"{pre}grad:{n}")
        sq += float((g.double() ** 2).sum())
    out[pre + "gradnorm"] = np.array(np.sqrt(sq))


def fixture_bench_shapes(g2, lin, qf, xa, meta):
    """One forward+backward of the reference at EXACTLY the bench's shapes (round 3): the
    caption models at B=128 (8,064 / 3,968 / 4,096-row GEMMs, the four-wave kernels' routing)
    and the LM at one B=16 x 1024 micro-step (M = 16,384 dX GEMMs, K = 16,384 batched weight
    gradients).  The reference runs on the bf16-valued recipe weights in fp32 math (the
    `mp` loop of train_ref), so the comparison isolates the GPU path's compute error; the
    loss at the fp32 recipe weights is stored too (`loss_fp32w`, the north-star 1e-4 bar)."""
    out = {}
    torch.set_grad_enabled(True)
    for kind, mod in (("qformer", qf), ("linear", lin)):
        lm = mod.GPT_previous(mod.GPTConfig(vocab_size=50304, block_size=1024))
        model = set_recipe(mod.GPT_Caption(enc_dim=768, lm=lm, m_vis_tokens=32))
        model.eval()
        z_raw, x, yy, mask = inputs_caption(BENCH_CAP_B, 257, 768, 31, 50257, 1313)
        labels = yy.masked_fill(~mask, -100)
        z = mod.pool_clip_197_to_33_avg_with_cls(z_raw)
        with torch.no_grad():
            out[f"{kind}_loss_fp32w"] = np.array(float(model(z, x, labels=labels)[1]))
        round_bf16_(model)
        _, loss = model(z, x, labels=labels)
        loss.backward()
        names = [n for n, p in model.named_parameters() if p.requires_grad]
        meta[f"bench_{kind}_trainable"] = names
        out[f"{kind}_loss"] = np.array(float(loss))
        _grads_out(model, names, out, f"{kind}_")
        out[f"{kind}_x"], out[f"{kind}_labels"] = x.numpy(), labels.numpy()
        print(kind, float(loss), out[f"{kind}_loss_fp32w"], out[f"{kind}_gradnorm"], flush=True)
        del model, lm, loss
    model = set_recipe(xa.GPT(xa.GPTConfig(vocab_size=50304, block_size=1024)))
    z_raw, x, yy, mask = inputs_caption(BENCH_CAP_B, 257, 768, 31, 50257, 1414)
    z = xa.pool_clip_197_to_33_avg_with_cls(z_raw)
    with torch.no_grad():
        out["cross_loss_fp32w"] = np.array(float(model(x, z=z, targets=yy, target_mask=mask)[1]))
    round_bf16_(model)
    _, loss = model(x, z=z, targets=yy, target_mask=mask)
    loss.backward()
    names = [n for n, p in model.named_parameters() if p.requires_grad]
    meta["bench_cross_trainable"] = names
    out["cross_loss"] = np.array(float(loss))
    _grads_out(model, names, out, "cross_")
    out["cross_x"], out["cross_y"], out["cross_mask"] = x.numpy(), yy.numpy(), mask.numpy()
    print("cross", float(loss), out["cross_loss_fp32w"], out["cross_gradnorm"], flush=True)
    del model, loss
    out["z_seeds"] = np.array([1313, 1414])
    out["cap_batch"] = np.array(BENCH_CAP_B)
    # LM: one micro-step of the bench's B=16 x 1024 (the x, y windows regenerate on the box
    # from the recipe id stream, seed 4040)
    cfg = g2["GPTConfig"](vocab_size=50304)
    model = set_recipe(g2["GPT"](cfg))
    x, y = inputs_lm(BENCH_LM_B, 1024, 50257, 4040)
    with torch.no_grad():
        out["lm_loss_fp32w"] = np.array(float(model(x, y)[1]))
    round_bf16_(model)
    _, loss = model(x, y)
    loss.backward()
    names = [n for n, p in model.named_parameters() if p.requires_grad]
    meta["bench_lm_trainable"] = names
    out["lm_loss"] = np.array(float(loss))
    _grads_out(model, names, out, "lm_")
    out["lm_seed"] = np.array(4040)
    out["lm_batch"] = np.array(BENCH_LM_B)
    print("lm", float(loss), out["lm_loss_fp32w"], out["lm_gradnorm"], flush=True)
    np.savez_compressed(os.path.join(OUT, "bench_shapes.npz"), **out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--full", action="store_true", help="also the 124M scalar fixtures")
    ap.add_argument("--only", default="",
                    help="comma list of round-2 sets to (re)generate alone: "
                         "full_train,accum,edge,greedy")
    args = ap.parse_args()
    os.makedirs(OUT, exist_ok=True)
    torch.set_num_threads(os.cpu_count() or 8)
    meta = {"torch": torch.__version__, "tiny_config": TINY, "generator": "tools/make_fixtures.py",
            "reference": "theophile-lt/gpt2-vision-language @ /root/reference"}
    g2 = load_gpt2_classes()
    lin = load_module("gpt2_linear", "ref_gpt2_linear_model")
    qf = load_module("gpt2_q_former", "ref_gpt2_q_former_model")
    xa = load_module("gpt2_cross-att", "ref_gpt2_cross_att_model")
    if args.only:
        mpath = os.path.join(OUT, "meta.json")
        with open(mpath) as f:
            meta = json.load(f)
        sets = {"full_train": lambda: fixture_full_train(g2, lin, qf, xa, meta),
                "accum": lambda: fixture_accum(g2, qf, meta),
                "edge": lambda: fixture_edge(lin, qf, xa, meta),
                "greedy": lambda: fixture_greedy(g2, lin, qf, xa, meta),
                "bench_shapes": lambda: fixture_bench_shapes(g2, lin, qf, xa, meta)}
        for name in args.only.split(","):
            sets[name]()
        with open(mpath, "w") as f:
            json.dump(meta, f, indent=1)
        return
    fixture_ops(lin)
    fixture_gpt(g2, meta)
    fixture_caption(lin, "linear", meta, m_vis=32)
    fixture_caption(qf, "qformer", meta, m_vis=32)
    fixture_cross(xa, meta)
    if args.full:
        fixture_full(g2, qf, meta)
    with open(os.path.join(OUT, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    for fn in sorted(os.listdir(OUT)):
        print(fn, os.path.getsize(os.path.join(OUT, fn)))


if __name__ == "__main__":
    main()
