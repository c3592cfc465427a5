"""KV-cached incremental decoding and sampling.

The reference re-runs the whole sequence through forward() for every new token
(train_gpt2.py:440-449 top-k sampling; gpt2_linear/data.py:111-127 temperature + top-p
caption decoding).  Here a prompt is prefilled once into a per-layer KV cache and every new
token costs one row through each block:

  * cache: one packed bf16 [B, Tmax, 3C] tensor per layer — the c_attn GEMM of a new token
    writes its q|k|v row straight into cache[:, t] (ldc = Tmax*3C), so nothing is copied;
  * attention of the new row: gvl_attn_decode over cache[:, :t+1] (k and v as strided views);
  * caption models prefill [bridge(z) | prompt embeddings] (positions on text only,
    gpt2_linear/model.py:197-200); the cross-att model projects z once and caches every
    layer's kv_proj(z_proj) (gpt2_cross-att/model.py:160-165, :49-57);
  * the next token comes from gvl_sample (temperature / top-k / top-p, inverse CDF of a
    uniform drawn from the caller's torch.Generator) or its greedy form (top_k = 1, u = 0:
    the first maximum, torch.argmax's tie-break).

Everything runs on the libgvl kernels; no autograd (inference only).
"""
from __future__ import annotations

import torch

from . import functional as Fn
from . import kernels as K
from .functional import bf

BF16 = torch.bfloat16


def _block_params(blk):
    a, m = blk.attn, blk.mlp
    return dict(ln1=(bf(blk.ln_1.weight), bf(blk.ln_1.bias)), attn=(bf(a.c_attn.weight), bf(a.c_attn.bias)),
                aproj=(bf(a.c_proj.weight), bf(a.c_proj.bias)), ln2=(bf(blk.ln_2.weight), bf(blk.ln_2.bias)),
                fc=(bf(m.c_fc.weight), bf(m.c_fc.bias)), mproj=(bf(m.c_proj.weight), bf(m.c_proj.bias)),
                H=a.n_head)


def _cross_params(blk):
    xa = blk.xattn
    return dict(ln=(bf(blk.ln_x.weight), bf(blk.ln_x.bias)), q=(bf(xa.q_proj.weight), bf(xa.q_proj.bias)),
                kv=(bf(xa.kv_proj.weight), bf(xa.kv_proj.bias)), c=(bf(xa.c_proj.weight), bf(xa.c_proj.bias)),
                gate=bf(blk.cross_gate), H=xa.n_head)


class KVDecoder:
    """Prefill + one-token steps for gvl.gpt2.GPT, gvl.caption.GPT_Caption (its frozen
    decoder) and gvl.cross_att.GPT.  Batch B; the cache holds the prefix + max_new tokens."""

    def __init__(self, model, batch: int, max_new: int):
        from . import caption, cross_att
        self.model = model
        self.kind = ("caption" if isinstance(model, caption.GPT_Caption) else
                     "cross" if isinstance(model, cross_att.GPT) else "gpt")
        dec = model.gpt if self.kind == "caption" else model
        tr = dec.transformer
        self.wte, self.wpe = bf(tr.wte.weight), bf(tr.wpe.weight)
        self.lnf = (bf(tr.ln_f.weight), bf(tr.ln_f.bias))
        self.head = bf(dec.lm_head.weight)
        self.blocks = [_block_params(b) for b in tr.h]
        self.cross = [_cross_params(b) for b in tr.h] if self.kind == "cross" else None
        self.block_size = dec.config.block_size
        C = self.wte.shape[1]
        self.C, self.B, self.max_new = C, batch, max_new
        self.Tmax = 0
        self.cache = None  # allocated by prefill: [B, prefix + max_new, 3C] per layer
        self.kvz = None
        self.t = 0        # positions in the cache
        self.txt0 = 0     # cache position of the first text token (caption prefix length)

    # ---------------------------------------------------------------- pieces
    def _ln(self, x2, wb):
        return K.layernorm_fwd(x2, wb[0], wb[1], stats=False)[0]

    def _cross(self, l, x2, S):
        """x + tanh(g) * c_proj(attn(q_proj(ln_x x), kv_proj(z_proj))) for S new rows."""
        P = self.cross[l]
        kvz = self.kvz[l]
        q = K.linear(self._ln(x2, P["ln"]), *P["q"])
        C = self.C
        if S == 1:
            y = K.attn_decode(q, kvz[:, :, :C], kvz[:, :, C:], P["H"])
        else:
            y = K.attn_fwd(q.view(self.B, S, C), kvz[:, :, :C], kvz[:, :, C:], P["H"], False)[0]
            y = y.view(self.B * S, C)
        return K.linear(y, P["c"][0], P["c"][1], residual=x2, gate=P["gate"])

    def _mlp(self, x2, P):
        h = K.linear(self._ln(x2, P["ln2"]), *P["fc"], act=1)
        return K.linear(h, P["mproj"][0], P["mproj"][1], residual=x2)

    def _logits(self, x2):
        xf = self._ln(x2, self.lnf)
        wp, V = Fn.pad_vocab(self.head)
        lg = K.linear(xf, wp)
        return lg if wp is self.head else lg[:, :V]

    # ------------------------------------------------------------------ API
    @torch.no_grad()
    def prefill(self, x_emb):
        """x_emb [B, S, C]: the whole prefix (image tokens + prompt embeddings).  Returns the
        logits of the last position [B, V]."""
        B, S, C = x_emb.shape
        self.Tmax = S + self.max_new
        self.cache = [torch.empty(B, self.Tmax, 3 * C, dtype=BF16, device=x_emb.device)
                      for _ in self.blocks]
        x2 = x_emb.to(BF16).reshape(B * S, C).contiguous()
        for l, P in enumerate(self.blocks):
            if self.cross is not None:
                x2 = self._cross(l, x2, S)
            qkv = K.linear(self._ln(x2, P["ln1"]), *P["attn"])
            q3 = qkv.view(B, S, 3 * C)
            self.cache[l][:, :S].copy_(q3)
            y = K.attn_fwd(q3[:, :, :C], q3[:, :, C:2 * C], q3[:, :, 2 * C:], P["H"], True)[0]
            x2 = K.linear(y.view(B * S, C), P["aproj"][0], P["aproj"][1], residual=x2)
            x2 = self._mlp(x2, P)
        self.t = S
        last = x2.view(B, S, C)[:, S - 1].contiguous()
        return self._logits(last)

    @torch.no_grad()
    def step(self, ids):
        """Append one token per sequence (ids [B]) and return the next logits [B, V]."""
        B, C, t = self.B, self.C, self.t
        if t >= self.Tmax:
            raise ValueError("KV cache full")
        pos = t - self.txt0
        if pos >= self.wpe.shape[0]:
            raise ValueError(f"position {pos} exceeds block_size {self.wpe.shape[0]}")
        Fn.check_index_range(ids, self.wte.shape[0], "token id")
        x = torch.empty(B, 1, C, dtype=BF16, device=ids.device)
        K.embedding_fwd(ids.view(B, 1), self.wte, self.wpe[pos:pos + 1], x, 1, 1, 0)
        x2 = x.view(B, C)
        for l, P in enumerate(self.blocks):
            if self.cross is not None:
                x2 = self._cross(l, x2, 1)
            row = self.cache[l][:, t]  # [B, 3C] view, row stride Tmax*3C
            K.linear(self._ln(x2, P["ln1"]), *P["attn"], out=row)
            cl = self.cache[l][:, :t + 1]
            y = K.attn_decode(row[:, :C], cl[:, :, C:2 * C], cl[:, :, 2 * C:], P["H"])
            x2 = K.linear(y, P["aproj"][0], P["aproj"][1], residual=x2)
            x2 = self._mlp(x2, P)
        self.t = t + 1
        return self._logits(x2)

    # ------------------------------------------------------- model-specific prefixes
    @torch.no_grad()
    def start(self, prompt_ids, z=None):
        """Prefill for the model kind: text-only (GPT), [bridge(z) | text] (caption), or text
        with the cached cross-attention keys/values of z (cross-att).  Returns logits [B, V]."""
        m = self.model
        self.kvz = None
        if self.kind == "caption":
            pt = z.unsqueeze(1) if z.dim() == 2 else z
            if m.use_cls_only:
                pt = pt[:, 0:1, :]
            img = m.bridge(pt).to(BF16)
            M = img.shape[1]
            emb = Fn.EmbedFn.apply(prompt_ids, self.wte, self.wpe, img)
            self.txt0 = M
            return self.prefill(emb)
        if self.kind == "cross" and z is not None:
            zp = m.transformer.vis_proj(z).to(BF16)
            Sz = zp.shape[1]
            z2 = zp.reshape(-1, self.C).contiguous()
            self.kvz = [K.linear(z2, *P["kv"]).view(self.B, Sz, 2 * self.C) for P in self.cross]
        elif self.kind == "cross":
            self.cross = None  # z=None: the gated cross-attention is skipped (model.py:159-165)
        self.txt0 = 0
        emb = Fn.EmbedFn.apply(prompt_ids, self.wte, self.wpe, None)
        return self.prefill(emb)


def sample_next(logits, *, greedy=False, temperature=1.0, top_k=0, top_p=1.0, generator=None):
    """Next token ids [B] from logits [B, V] on the gvl_sample kernel."""
    rows = logits.shape[0]
    if greedy:
        u = torch.zeros(rows, dtype=torch.float32, device=logits.device)
        return K.sample(logits, u, 1.0, 1, 1.0)
    u = torch.rand(rows, generator=generator, device=logits.device, dtype=torch.float32)
    return K.sample(logits, u, temperature, top_k, top_p)


@torch.no_grad()
def generate(model, prompt_ids, n_new, *, z=None, greedy=False, temperature=1.0, top_k=0,
             top_p=1.0, generator=None, return_logits=False):
    """KV-cached decode of n_new tokens after prompt_ids [B, P].  greedy: argmax (first max);
    else temperature / top-k / top-p sampling with `generator` (a CUDA torch.Generator).
    Returns the new ids [B, n_new] (and the per-step logits [B, n_new, V] if asked)."""
    B = prompt_ids.shape[0]
    dec = KVDecoder(model, B, n_new)
    logits = dec.start(prompt_ids, z)
    out, lg = [], []
    for i in range(n_new):
        if return_logits:
            lg.append(logits.float())
        nxt = sample_next(logits, greedy=greedy, temperature=temperature, top_k=top_k,
                          top_p=top_p, generator=generator)
        out.append(nxt)
        if i + 1 < n_new:
            logits = dec.step(nxt)
    ids = torch.stack(out, dim=1)
    return (ids, torch.stack(lg, dim=1)) if return_logits else ids
