"""Functional CPU fp32 restatement of the reference models (TEST INFRASTRUCTURE).

Parameters are a dict keyed exactly like the reference state_dicts;
dropout is off (the parity setting).  Autograd on these functions gives the
reference gradients.
"""
from __future__ import annotations

import torch

from . import ops as O


def _ln(P, k, x):
    return O.layernorm(x, P[k + ".weight"], P[k + ".bias"])


def _lin(P, k, x, bias=True):
    return O.linear(x, P[k + ".weight"], P.get(k + ".bias") if bias else None)


def self_attention(P, pre, x, H):
    """CausalSelfAttention.forward (train_gpt2.py:33-43)."""
    C = x.shape[-1]
    qkv = _lin(P, pre + "c_attn", x)
    q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
    y = O.attention(O.split_heads(q, H), O.split_heads(k, H), O.split_heads(v, H), causal=True)
    return _lin(P, pre + "c_proj", O.merge_heads(y))


def block(P, pre, x, H):
    """Block.forward (train_gpt2.py:71-74): pre-LN residual attention + tanh-GELU MLP."""
    x = x + self_attention(P, pre + "attn.", _ln(P, pre + "ln_1", x), H)
    h = O.gelu_tanh(_lin(P, pre + "mlp.c_fc", _ln(P, pre + "ln_2", x)))
    return x + _lin(P, pre + "mlp.c_proj", h)


def embed(P, pre, idx):
    """wte(idx) + wpe(arange(T)) (train_gpt2.py:114-117)."""
    T = idx.shape[1]
    return P[pre + "transformer.wte.weight"][idx] + P[pre + "transformer.wpe.weight"][:T]


def decoder(P, pre, x, n_layer, H):
    for i in range(n_layer):
        x = block(P, f"{pre}transformer.h.{i}.", x, H)
    return _ln(P, pre + "transformer.ln_f", x)


def gpt_forward(P, idx, n_layer, H, targets=None, pre=""):
    """GPT.forward (train_gpt2.py:111-125) -> (logits, loss|None)."""
    x = decoder(P, pre, embed(P, pre, idx), n_layer, H)
    logits = x @ P[pre + "lm_head.weight"].t()
    loss = None if targets is None else O.cross_entropy(logits, targets)
    return logits, loss


# ------------------------------------------------------------------ bridges
def mha(P, pre, q_in, kv_in, H):
    """nn.MultiheadAttention(batch_first) eval forward (packed in_proj rows [q; k; v])."""
    C = q_in.shape[-1]
    W, b = P[pre + "in_proj_weight"], P[pre + "in_proj_bias"]
    q = O.linear(q_in, W[:C], b[:C])
    k = O.linear(kv_in, W[C:2 * C], b[C:2 * C])
    v = O.linear(kv_in, W[2 * C:], b[2 * C:])
    y = O.attention(O.split_heads(q, H), O.split_heads(k, H), O.split_heads(v, H), causal=False)
    return _lin(P, pre + "out_proj", O.merge_heads(y))


def qformer_layer(P, pre, q, v, H):
    """QFormerLayer.forward (gpt2_q_former/model.py:133-145), dropout off."""
    q2 = _ln(P, pre + "ln1", q)
    q = q + mha(P, pre + "self_attn.", q2, q2, H)
    q = q + mha(P, pre + "cross_attn.", _ln(P, pre + "ln2_q", q), _ln(P, pre + "ln2_v", v), H)
    h = O.gelu_erf(_lin(P, pre + "mlp.0", _ln(P, pre + "ln3", q)))
    return q + _lin(P, pre + "mlp.2", h)


def bridge(P, kind, z, H, n_layers=2):
    """Linear_Bridge (gpt2_linear/model.py:127-129) or BLIP2Bridge (gpt2_q_former:159-168)."""
    x = _lin(P, "bridge.vis_proj", z)
    if kind == "linear":
        return x
    q = P["bridge.query_tokens"].unsqueeze(0).expand(z.shape[0], -1, -1)
    for i in range(n_layers):
        q = qformer_layer(P, f"bridge.layers.{i}.", q, x, H)
    return q


def caption_forward(P, kind, patch_tokens, ids, n_layer, H, block_size, labels=None):
    """GPT_Caption.forward (gpt2_linear/model.py:175-211)."""
    if patch_tokens.dim() == 2:
        patch_tokens = patch_tokens.unsqueeze(1)
    img = bridge(P, kind, patch_tokens, H)
    M = img.shape[1]
    T = ids.shape[1]
    if M + T > block_size:
        T = block_size - M
        ids = ids[:, :T]
        labels = None if labels is None else labels[:, :T]
    txt = P["gpt.transformer.wte.weight"][ids] + P["gpt.transformer.wpe.weight"][:T]
    x = decoder(P, "gpt.", torch.cat([img, txt], dim=1), n_layer, H)
    logits = x @ P["gpt.lm_head.weight"].t()
    loss = None
    if labels is not None:
        loss = O.cross_entropy(logits[:, M:M + T], labels)
    return logits, loss


def cross_att_forward(P, idx, z, n_layer, H, targets=None, target_mask=None):
    """cross-att GPT.forward (gpt2_cross-att/model.py:152-186)."""
    x = embed(P, "", idx)
    zp = None if z is None else _lin(P, "transformer.vis_proj.z_proj", z)
    for i in range(n_layer):
        pre = f"transformer.h.{i}."
        if zp is not None:
            xn = _ln(P, pre + "ln_x", x)
            C = x.shape[-1]
            q = _lin(P, pre + "xattn.q_proj", xn)
            kv = _lin(P, pre + "xattn.kv_proj", zp)
            y = O.attention(O.split_heads(q, H), O.split_heads(kv[..., :C], H),
                            O.split_heads(kv[..., C:], H), causal=False)
            y = _lin(P, pre + "xattn.c_proj", O.merge_heads(y))
            x = x + torch.tanh(P[pre + "cross_gate"]) * y
        x = block(P, pre, x, H)
    x = _ln(P, "transformer.ln_f", x)
    logits = x @ P["lm_head.weight"].t()
    loss = None
    if targets is not None:
        if target_mask is None:
            loss = O.cross_entropy(logits, targets)
        else:
            loss = O.masked_cross_entropy(logits, targets, target_mask)
    return logits, loss


def greedy(step_logits_fn, prompt, n_new):
    """Full-recompute greedy decode: next = argmax(logits[:, -1]) (first max on ties)."""
    x = prompt
    toks, margins = [], []
    for _ in range(n_new):
        last = step_logits_fn(x)[:, -1, :]
        top2 = torch.topk(last, 2, dim=-1)
        margins.append(top2.values[:, 0] - top2.values[:, 1])
        nxt = torch.argmax(last, dim=-1, keepdim=True)
        toks.append(nxt)
        x = torch.cat([x, nxt], dim=1)
    return torch.cat(toks, dim=1), torch.stack(margins, dim=1)


def trainable_keys(kind, keys):
    """Which parameters train in each setting."""
    if kind == "gpt":  # lm_head.weight is the canonical copy of the tied wte
        return [k for k in keys if not k.endswith(".attn.bias") and k != "transformer.wte.weight"]
    if kind in ("linear", "qformer"):
        return [k for k in keys if k.startswith("bridge.")]
    if kind == "cross":
        return [k for k in keys if ".xattn." in k or k.endswith("cross_gate")
                or k.startswith("transformer.vis_proj.")]
    raise ValueError(kind)


def decay_split(P, keys):
    """configure_optimizers grouping: >=2-D decays, <2-D does not (train_gpt2.py:131-132)."""
    return [k for k in keys if P[k].dim() >= 2], [k for k in keys if P[k].dim() < 2]


def train_steps(P, kind, keys, loss_of, n_steps, lr_of, wd=0.1, max_norm=1.0):
    """The optimizer loop of train_gpt2.py:457-476 in fp32: zero_grad, fwd/bwd, clip,
    AdamW (decoupled decay on >=2-D params). Mutates P (trainable entries). Returns losses."""
    dk, nk = decay_split(P, keys)
    state = {k: (torch.zeros_like(P[k]), torch.zeros_like(P[k])) for k in keys}
    losses = []
    tied = [k for k in P if k.endswith("lm_head.weight")]
    for it in range(n_steps):
        for k in keys:
            P[k] = P[k].detach().requires_grad_(True)
        # keep tie: wte aliases lm_head
        for k in tied:
            kb = k[: -len("lm_head.weight")] + "transformer.wte.weight"
            if kb in P:
                P[kb] = P[k]
        loss = loss_of(P, it)
        grads = torch.autograd.grad(loss, [P[k] for k in keys])
        losses.append(float(loss))
        _, coef = O.clip_coef(grads, max_norm)
        lr = lr_of(it)
        with torch.no_grad():
            for k, g in zip(keys, grads):
                p = P[k].detach().clone()
                m, v = state[k]
                O.adamw_update(p, g * coef, m, v, it + 1, lr, wd=(wd if k in dk else 0.0))
                P[k] = p
        for k in tied:
            kb = k[: -len("lm_head.weight")] + "transformer.wte.weight"
            if kb in P:
                P[kb] = P[k]
    return losses
