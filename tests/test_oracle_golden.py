"""Pin the CPU restatement (oracle/) against golden fixtures produced by the reference's
own model code (tools/make_fixtures.py).  CPU only."""
import numpy as np
import pytest
import torch

from oracle import models as OM
from oracle import ops as O
from tests.helpers import (TINY, check_summary, fixture_name, lr_caption, lr_cross, lr_lm,
                           named_trainable, recipe_params, rel_err)

RT = 2e-5  # fp32 restatement vs fp32 reference


def _t(a):
    return torch.from_numpy(np.asarray(a))


def test_ops_sdpa(golden):
    fx = golden("ops")
    for name, causal in (("sdpa_causal", True), ("sdpa_cross", False), ("sdpa_self32", False)):
        q, k, v = (_t(fx[f"{name}:{n}"]).requires_grad_(True) for n in "qkv")
        o = O.attention(q, k, v, causal)
        assert rel_err(o.detach().numpy(), fx[f"{name}:o"]) < RT
        o.backward(_t(fx[f"{name}:do"]))
        for t, n in ((q, "dq"), (k, "dk"), (v, "dv")):
            assert rel_err(t.grad.numpy(), fx[f"{name}:{n}"]) < 1e-4, (name, n)


@pytest.mark.parametrize("side", [16, 14])
def test_ops_pool(golden, side):
    fx = golden("ops")
    out = O.pool_clip(_t(fx[f"pool{side}:in"]))
    assert rel_err(out.numpy(), fx[f"pool{side}:out"]) < RT


def test_ops_ln_gelu_ce(golden):
    fx = golden("ops")
    y = O.layernorm(_t(fx["ln:x"]), _t(fx["ln:w"]), _t(fx["ln:b"]))
    assert rel_err(y.numpy(), fx["ln:y"]) < RT
    g = _t(fx["gelu:x"])
    assert rel_err(O.gelu_tanh(g).numpy(), fx["gelu:tanh"]) < RT
    assert rel_err(O.gelu_erf(g).numpy(), fx["gelu:erf"]) < RT
    loss = O.cross_entropy(_t(fx["ce:logits"]), _t(fx["ce:targets"]))
    assert abs(float(loss) - float(fx["ce:loss"])) / float(fx["ce:loss"]) < RT
    ml = O.masked_cross_entropy(_t(fx["ce:logits"]), _t(fx["ce:targets2"]), _t(fx["ce:mask"]))
    assert abs(float(ml) - float(fx["ce:masked_loss"])) / float(fx["ce:masked_loss"]) < RT


def test_ops_adamw_clip(golden):
    fx = golden("ops")
    p = [_t(fx["adam:p1"]).clone(), _t(fx["adam:p2"]).clone()]
    g = [_t(fx["adam:g1"]), _t(fx["adam:g2"])]
    st = [(torch.zeros_like(x), torch.zeros_like(x)) for x in p]
    norms = []
    for it in range(2):
        gi = [x * (it + 1) for x in g]
        nrm, coef = O.clip_coef(gi, 1.0)
        norms.append(float(nrm))
        for j in range(2):
            O.adamw_update(p[j], gi[j] * coef, st[j][0], st[j][1], it + 1, 1e-3,
                           wd=0.1 if j == 0 else 0.0)
    assert rel_err(norms, fx["adam:norms"]) < RT
    assert rel_err(p[0].numpy(), fx["adam:p1_after"]) < 1e-6
    assert rel_err(p[1].numpy(), fx["adam:p2_after"]) < 1e-6


def test_encode_caption_semantics():
    """_encode_caption (gpt2_linear/data.py:35-49): SURVEY.md A22's measured example."""
    x, y, m = O.encode_caption([1, 2, 3, 4, 5], 32, 50256)
    assert x[:6].tolist() == [1, 2, 3, 4, 5, 50256]
    assert y[:5].tolist() == [2, 3, 4, 5, 50256]
    assert int(m.sum()) == 5 and x.shape == (31,)
    x, y, m = O.encode_caption(list(range(40)), 32, 50256)
    assert int(m.sum()) == 31 and y[-1].item() == 50256
    x, y, m = O.encode_caption([], 32, 50256)
    assert int(m.sum()) == 1


def _grads_and_steps(kind, fx, meta, loss_of, lr_of):
    P = recipe_params(meta[f"{kind}_keys"])
    names = named_trainable(kind, meta)
    keys = [fixture_name(kind, n) for n in names]
    for k in keys:
        P[k] = P[k].clone().requires_grad_(True)
    if kind == "gpt":
        P["transformer.wte.weight"] = P["lm_head.weight"]
    loss = loss_of(P, 0)
    assert abs(float(loss) - float(fx["loss"])) / abs(float(fx["loss"])) < RT
    grads = torch.autograd.grad(loss, [P[k] for k in keys])
    for n, g in zip(names, grads):
        check_summary(fx, "grad:" + n, g, 2e-4)
    P2 = recipe_params(meta[f"{kind}_keys"])
    losses = OM.train_steps(P2, kind, keys, loss_of, 3, lr_of)
    assert rel_err(losses, fx["train_losses"]) < 1e-5
    for n, k in zip(names, keys):
        check_summary(fx, "step3:" + n, P2[k], 2e-4)


def test_gpt_tiny(golden, meta):
    fx = golden("gpt_tiny")
    x, y = _t(fx["x"]), _t(fx["y"])
    P = recipe_params(meta["gpt_keys"])
    logits, loss = OM.gpt_forward(P, x, 2, 2, y)
    assert rel_err(logits.numpy(), fx["logits"]) < RT
    _grads_and_steps("gpt", fx, meta, lambda P, it: OM.gpt_forward(P, x, 2, 2, y)[1], lr_lm)
    toks, _ = OM.greedy(lambda s: OM.gpt_forward(P, s, 2, 2)[0], _t(fx["greedy_prompt"]), 16)
    assert toks.tolist() == fx["greedy_tokens"].tolist()


@pytest.mark.parametrize("kind", ["linear", "qformer"])
def test_caption_tiny(golden, meta, kind):
    fx = golden(f"{kind}_tiny")
    z_raw = _t(fx["z_raw"])
    z = O.pool_clip(z_raw)
    assert rel_err(z.numpy(), fx["z"]) < RT
    x, labels = _t(fx["x"]), _t(fx["labels"])
    P = recipe_params(meta[f"{kind}_keys"])
    logits, loss = OM.caption_forward(P, kind, z, x, 2, 2, 64, labels)
    assert rel_err(logits.numpy(), fx["logits"]) < RT

    def loss_of(P, it):
        return OM.caption_forward(P, kind, z, x, 2, 2, 64, labels)[1]

    _grads_and_steps(kind, fx, meta, loss_of, lr_caption)
    toks, _ = OM.greedy(lambda s: OM.caption_forward(P, kind, z[:1], s, 2, 2, 64)[0],
                        _t(fx["greedy_prompt"]), 16)
    assert toks.tolist() == fx["greedy_tokens"].tolist()


def test_cross_tiny(golden, meta):
    fx = golden("cross_tiny")
    z = O.pool_clip(_t(fx["z_raw"]))
    assert rel_err(z.numpy(), fx["z"]) < RT
    x, y, m = _t(fx["x"]), _t(fx["y"]), _t(fx["mask"])
    P = recipe_params(meta["cross_keys"])
    logits, loss = OM.cross_att_forward(P, x, z, 2, 2, y, m)
    assert rel_err(logits.numpy(), fx["logits"]) < RT
    _, lu = OM.cross_att_forward(P, x, z, 2, 2, y)
    assert abs(float(lu) - float(fx["loss_unmasked"])) / float(fx["loss_unmasked"]) < RT

    def loss_of(P, it):
        return OM.cross_att_forward(P, x, z, 2, 2, y, m)[1]

    _grads_and_steps("cross", fx, meta, loss_of, lr_cross)
    toks, _ = OM.greedy(lambda s: OM.cross_att_forward(P, s, z[:1], 2, 2)[0],
                        _t(fx["greedy_prompt"]), 16)
    assert toks.tolist() == fx["greedy_tokens"].tolist()


def test_fast_paths_match_explicit_math():
    """oracle.ops.FAST_PATHS (bench.py's timed CPU baseline) computes the same values."""
    import torch
    from oracle import ops as O
    g = torch.Generator().manual_seed(3)
    q, k, v = (torch.randn(2, 3, 40, 64, generator=g) for _ in range(3))
    x = torch.randn(5, 7, 96, generator=g)
    w, b = torch.randn(96, generator=g), torch.randn(96, generator=g)
    lg = torch.randn(30, 50, generator=g)
    t = torch.randint(0, 50, (30,), generator=g)
    t[::4] = -100
    outs = []
    for fast in (False, True):
        O.FAST_PATHS = fast
        try:
            outs.append([O.attention(q, k, v, True), O.attention(q, k, v, False),
                         O.layernorm(x, w, b), O.gelu_tanh(x), O.gelu_erf(x),
                         O.cross_entropy(lg, t)])
        finally:
            O.FAST_PATHS = False
    for a, b_ in zip(*outs):
        assert torch.allclose(a, b_, rtol=1e-5, atol=1e-5)
