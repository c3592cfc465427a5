"""Fused AdamW + gradient clipping over flat bf16 arenas (the reference's
torch.optim.AdamW(fused=True) + clip_grad_norm_, train_gpt2.py:140-143, :472, :476).

MI355X design: at the first step every trainable parameter (and its .grad) is re-pointed
into ONE contiguous bf16 arena per quantity (params, grads, exp_avg, exp_avg_sq), laid out
group by group (decay group first).  Then
  * the global grad norm is one streaming reduction over the grad arena, finished on the
    device together with the clip coefficient (no host sync);
  * AdamW is one streaming kernel per param group, applying the clip coefficient to the
    gradient on the fly (14 B of HBM traffic per parameter);
  * data-parallel gradient buckets are plain slices of the grad arena (gvl.dist).
Parameters keep their identity; `param.data` / `param.grad` become views of the arenas.
"""
from __future__ import annotations

import torch

from . import kernels as K

BF16 = torch.bfloat16
F32 = torch.float32
_ALIGN = 8  # elements: every segment starts 16-byte aligned


def _pad(n):
    return (n + _ALIGN - 1) // _ALIGN * _ALIGN


def arena_offsets(param_groups):
    """(offsets in param_groups order, per-group [start, end) segments, total) of the flat
    arenas: each parameter a 16-B aligned slot, group after group (decay group first)."""
    offs, seg = [], []
    total = 0
    for g in param_groups:
        start = total
        # parameters tagged with the same `_gvl_stack_key` (the cross-att blocks' kv_proj
        # weights / biases, which gvl.functional.CrossKVFn multiplies as ONE stacked matrix)
        # get consecutive arena slots at the first one's place, so the stack is a view of the
        # arena instead of a per-step torch.cat; the param_groups order (and so the optimizer
        # state_dict's parameter indices) is unchanged
        stacks = {}
        for p in g["params"]:
            k = getattr(p, "_gvl_stack_key", None)
            if k is not None:
                stacks.setdefault(k, []).append(p)
        placed = {}
        for p in g["params"]:
            if id(p) in placed:
                continue
            k = getattr(p, "_gvl_stack_key", None)
            for q in (stacks[k] if k is not None else [p]):
                placed[id(q)] = total
                total += _pad(q.numel())
        offs.extend(placed[id(p)] for p in g["params"])
        seg.append((start, total))
    return offs, seg, total


class AdamW(torch.optim.Optimizer):
    """torch.optim.AdamW drop-in (the reference's fused AdamW, train_gpt2.py:140-143).

    master_weights=True (default): fp32 master weights and fp32 moments in arenas, the
    model's bf16 parameters are compute copies rewritten by every step (mixed precision).
    False: bf16 parameters and bf16 moments updated in place — the reference's own GPU
    semantics (model.to(bfloat16) + fused AdamW), where an update below half a bf16 ulp of
    the weight (e.g. every LayerNorm gain at lr 6e-4) rounds away.
    """

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2,
                 master_weights: bool = True):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.master_weights = bool(master_weights)
        self._arena = None
        self._clip_coef = None
        self._step_count = 0

    # ---------------------------------------------------------------- arenas
    def _build(self):
        params = [p for g in self.param_groups for p in g["params"]]
        if not params:
            raise ValueError("gvl AdamW: no parameters")
        dev = params[0].device
        if dev.type != "cuda":
            raise RuntimeError("gvl AdamW runs on the ROCm device; use torch.optim.AdamW on CPU")
        for p in params:
            if p.dtype != BF16:
                raise TypeError("gvl AdamW expects bf16 parameters (the reference trains the "
                                "model after .to(torch.bfloat16))")
        offs, seg, total = arena_offsets(self.param_groups)
        total = max(total, _ALIGN)
        sdt = F32 if self.master_weights else BF16
        parena = torch.zeros(total, dtype=BF16, device=dev)
        garena = torch.zeros(total, dtype=BF16, device=dev)
        marena = torch.zeros(total, dtype=sdt, device=dev)
        varena = torch.zeros(total, dtype=sdt, device=dev)
        warena = torch.zeros(total, dtype=F32, device=dev) if self.master_weights else None
        for p, o in zip(params, offs):
            n = p.numel()
            st = self.state[p]
            view = parena[o:o + n].view_as(p)
            view.copy_(p.data)
            if warena is not None:
                mview = warena[o:o + n].view_as(p)
                # a resumed master copy (state 'master', see state_dict) beats the bf16 weight
                mview.copy_(st["master"].to(device=dev, dtype=F32).view_as(p) if "master" in st
                            else p.data.float())
                st["master"] = mview
            else:
                st.pop("master", None)  # a stale fp32-master snapshot must not be resaved
            p.data = view
            gview = garena[o:o + n].view_as(p)
            if p.grad is not None:
                gview.copy_(p.grad)
            p.grad = gview
            p._gvl_grad_sink = True  # gvl.functional may accumulate into this grad in place
            # state loaded before the first step (the reference resumes with
            # configure_optimizers -> load_state_dict -> train, train_gpt2.py:320-322)
            # moves into the arenas instead of being reset
            for key, arena in (("exp_avg", marena), ("exp_avg_sq", varena)):
                aview = arena[o:o + n].view_as(p)
                if key in st:
                    aview.copy_(st[key].to(device=dev, dtype=sdt).view_as(p))
                st[key] = aview
            if "step" in st:
                self._step_count = max(self._step_count, int(float(st["step"])))
            st["step"] = torch.tensor(float(self._step_count), dtype=torch.float32)
        self._arena = dict(p=parena, g=garena, m=marena, v=varena, w=warena, offs=offs, seg=seg,
                           params=params)
        # per group {lr, step} on the device, read by the AdamW kernel (capturable step)
        self._hyper = torch.zeros(len(self.param_groups), 2, dtype=torch.float32, device=dev)

    @property
    def grad_arena(self):
        if self._arena is None:
            self._build()
        return self._arena["g"]

    def arena_layout(self):
        """[(param, offset, numel)] sorted by arena offset (used by gvl.dist buckets).

        Offsets follow param_groups order except for parameters sharing a
        `_gvl_stack_key`, which take consecutive slots at the first one's position; sorting
        keeps the "arena order" contract GradBuckets relies on when it has no model."""
        if self._arena is None:
            self._build()
        a = self._arena
        return sorted(((p, o, p.numel()) for p, o in zip(a["params"], a["offs"])),
                      key=lambda e: e[1])

    def master_of(self, p):
        """fp32 master copy of parameter p (None with master_weights=False)."""
        if self._arena is None:
            self._build()
        return self.state[p].get("master")

    @torch.no_grad()
    def sync_master_from_params(self):
        """Re-seed the fp32 masters from the bf16 parameters (after the caller overwrote
        parameters directly, e.g. model.load_state_dict after the optimizer was built)."""
        if self._arena is not None and self._arena["w"] is not None:
            self._arena["w"].copy_(self._arena["p"].float())

    def _sync_grads(self):
        """Re-point any grad that autograd replaced (e.g. after set_to_none)."""
        a = self._arena
        for p, o in zip(a["params"], a["offs"]):
            n = p.numel()
            gview = a["g"][o:o + n].view_as(p)
            if p.grad is None:
                gview.zero_()
                p.grad = gview
            elif p.grad.data_ptr() != gview.data_ptr():
                gview.copy_(p.grad)
                p.grad = gview

    # -------------------------------------------------------------- API
    def zero_grad(self, set_to_none: bool = True):
        """Zero the grad arena in one memset; grads stay arena views (set_to_none ignored)."""
        if self._arena is None:
            self._build()
        from . import functional as F
        F.discard_pending()  # deferred gradients left by a backward that raised
        self._arena["g"].zero_()
        self._sync_grads()

    @torch.no_grad()
    def clip_grad_norm_(self, max_norm: float):
        """Global L2 norm of all grads + the clip coefficient, both on the device; the
        coefficient is applied by the next step() (fused).  Returns the norm (0-dim fp32)."""
        if self._arena is None:
            self._build()
        self._sync_grads()
        out = K.grad_norm(self._arena["g"], max_norm)
        self._clip_coef = out[1:2]
        return out[0]

    def stage_hyper(self):
        """Copy each group's current lr and the step count to the device block the AdamW
        kernel reads (pinned host buffer, stream-ordered, no host sync)."""
        vals = torch.tensor([[float(g["lr"]), float(self._step_count)] for g in self.param_groups],
                            dtype=torch.float32).pin_memory()
        self._hyper.copy_(vals, non_blocking=True)

    def advance(self):
        """Host side of one optimizer step: bump the step count and stage {lr, step}.
        step() does this itself; a replayed hipGraph (gvl.graph) calls it per replay."""
        self._step_count += 1
        self.stage_hyper()

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        if self._arena is None:
            self._build()
        self._sync_grads()
        if not torch.cuda.is_current_stream_capturing():
            self.advance()
        a = self._arena
        for gi, (g, (s0, s1)) in enumerate(zip(self.param_groups, a["seg"])):
            if s1 == s0:
                continue
            b1, b2 = g["betas"]
            if a["w"] is not None:
                K.adamw_master_dev(a["p"][s0:s1], a["w"][s0:s1], a["g"][s0:s1], a["m"][s0:s1],
                                   a["v"][s0:s1], s1 - s0, self._hyper[gi], b1, b2, g["eps"],
                                   g["weight_decay"], grad_scale=self._clip_coef)
            else:
                K.adamw_dev(a["p"][s0:s1], a["g"][s0:s1], a["m"][s0:s1], a["v"][s0:s1], s1 - s0,
                            self._hyper[gi], b1, b2, g["eps"], g["weight_decay"],
                            grad_scale=self._clip_coef)
        self._clip_coef = None
        return loss

    def state_dict(self):
        if self._arena is not None:
            for p in self._arena["params"]:
                self.state[p]["step"].fill_(self._step_count)
                if not self.master_weights:
                    self.state[p].pop("master", None)
        return super().state_dict()

    def load_state_dict(self, state_dict):
        # torch casts every state tensor to its param's dtype (bf16); keep the saved fp32
        # moments / masters at full precision instead (same param order as the groups)
        saved_ids = [i for g in state_dict["param_groups"] for i in g["params"]]
        mine = [p for g in self.param_groups for p in g["params"]]
        raw = {}
        for pid, p in zip(saved_ids, mine):
            st = state_dict["state"].get(pid, {})
            raw[p] = {k: v for k, v in st.items()
                      if k in ("exp_avg", "exp_avg_sq", "master") and torch.is_tensor(v)
                      and v.dtype == F32}
        super().load_state_dict(state_dict)
        for p, kv in raw.items():
            for k, v in kv.items():
                self.state[p][k] = v.to(device=p.device)
        if self._arena is None:
            # moved into the arenas by _build() (first zero_grad / step)
            steps = [int(float(st["step"])) for st in self.state.values() if "step" in st]
            self._step_count = max(steps, default=0)
            return
        a = self._arena
        steps = []
        for p, o in zip(a["params"], a["offs"]):
            n = p.numel()
            st = self.state[p]
            keys = [("exp_avg", a["m"]), ("exp_avg_sq", a["v"])]
            if a["w"] is not None:
                keys.append(("master", a["w"]))
            else:
                st.pop("master", None)
            for key, arena in keys:
                view = arena[o:o + n].view_as(p)
                if key in st and st[key].data_ptr() != view.data_ptr():
                    view.copy_(st[key].to(device=view.device, dtype=view.dtype).view_as(p))
                elif key == "master" and key not in st:
                    view.copy_(p.data.float())
                st[key] = view
            if "step" in st:
                steps.append(int(float(st["step"])))
        self._step_count = max(steps, default=0)


def clip_grad_norm_(optimizer_or_params, max_norm: float):
    """Drop-in for torch.nn.utils.clip_grad_norm_.  Given a gvl AdamW, computes the norm on
    the device and defers the scaling into the fused step; otherwise falls back to torch's
    utility on the given parameters (eager, not the hot path)."""
    if isinstance(optimizer_or_params, AdamW):
        return optimizer_or_params.clip_grad_norm_(max_norm)
    if isinstance(optimizer_or_params, torch.optim.Optimizer):
        optimizer_or_params = [p for g in optimizer_or_params.param_groups for p in g["params"]]
    return torch.nn.utils.clip_grad_norm_(optimizer_or_params, max_norm)


def get_lr(it, max_lr, min_lr, warmup_steps, max_steps):
    """Cosine schedule with linear warmup (train_gpt2.py:277-285)."""
    import math
    if it < warmup_steps:
        return max_lr * (it + 1) / warmup_steps
    if it > max_steps:
        return min_lr
    ratio = (it - warmup_steps) / (max_steps - warmup_steps)
    assert 0 <= ratio <= 1
    return min_lr + 0.5 * (1.0 + math.cos(math.pi * ratio)) * (max_lr - min_lr)
