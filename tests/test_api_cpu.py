"""Drop-in API checks that need no GPU: module trees, state_dict layout, init recipe,
freezing semantics, optimizer grouping, and that the product path refuses CPU tensors."""
import pytest
import torch

from tests.helpers import TINY


def _seed_build(kind):
    import gvl.caption as cap
    import gvl.cross_att as xa
    import gvl.gpt2 as g2
    torch.manual_seed(0)
    if kind == "gpt":
        return g2.GPT(g2.GPTConfig(**TINY))
    if kind == "cross":
        return xa.GPT(xa.GPTConfig(**TINY, img_embd=TINY["n_embd"]))
    lm = cap.GPT_previous(g2.GPTConfig(**TINY))
    cls = cap.LinearCaption if kind == "linear" else cap.QFormerCaption
    return cls(enc_dim=TINY["n_embd"], lm=lm, m_vis_tokens=32)


@pytest.mark.parametrize("kind", ["gpt", "linear", "qformer", "cross"])
def test_state_dict_layout_and_init_match_reference(meta, kind):
    """Same keys, shapes and — under torch.manual_seed(0) — the same initial values as the
    reference classes (sums recorded from the reference by tools/make_fixtures.py)."""
    m = _seed_build(kind)
    sd = m.state_dict()
    want = meta[f"{kind}_keys"]
    assert [k for k, _ in want] == list(sd)
    assert [list(s) for _, s in want] == [list(v.shape) for v in sd.values()]
    ref = meta[f"{kind}_init_sums_seed0"]
    for k, v in sd.items():
        assert float(v.double().sum()) == pytest.approx(ref[k], rel=1e-6, abs=1e-6), k


def test_trainable_sets():
    cross = _seed_build("cross")
    tr = [n for n, p in cross.named_parameters() if p.requires_grad]
    assert all(".xattn." in n or n.endswith("cross_gate") or n.startswith("transformer.vis_proj")
               for n in tr)
    assert not any(".ln_x." in n for n in tr)
    for kind in ("linear", "qformer"):
        m = _seed_build(kind)
        tr = [n for n, p in m.named_parameters() if p.requires_grad]
        assert tr and all(n.startswith("bridge.") for n in tr)
        assert m.wte is m.gpt.transformer.wte and m.wpe is m.gpt.transformer.wpe
    g = _seed_build("gpt")
    assert g.transformer.wte.weight is g.lm_head.weight


def test_full_size_param_counts():
    """trainable counts of the full-size models."""
    import gvl.caption as cap
    import gvl.cross_att as xa
    import gvl.gpt2 as g2
    with torch.device("meta"):
        lm = cap.GPT_previous(g2.GPTConfig(vocab_size=50304))
        q = cap.QFormerCaption(enc_dim=768, lm=lm, m_vis_tokens=32)
        lm2 = cap.GPT_previous(g2.GPTConfig(vocab_size=50304))
        li = cap.LinearCaption(enc_dim=768, lm=lm2, m_vis_tokens=32)
        x = xa.GPT(xa.GPTConfig(vocab_size=50304))
        g = g2.GPT(g2.GPTConfig(vocab_size=50304))
    count = lambda m, tr: sum(p.numel() for p in m.parameters() if (p.requires_grad or not tr))
    assert count(q, True) == 19_521_792 and count(q, False) == 143_997_696
    assert count(li, True) == 590_592
    assert count(x, True) == 28_939_020 and count(x, False) == 153_433_356
    assert count(g, False) == 124_475_904


def test_optimizer_groups_cpu():
    g = _seed_build("gpt")
    opt = g.configure_optimizers(0.1, 6e-4, "cpu")
    assert isinstance(opt, torch.optim.AdamW)
    assert opt.param_groups[0]["weight_decay"] == 0.1 and opt.param_groups[1]["weight_decay"] == 0.0
    assert all(p.dim() >= 2 for p in opt.param_groups[0]["params"])
    assert all(p.dim() < 2 for p in opt.param_groups[1]["params"])


def test_product_path_has_no_cpu_fallback():
    from gvl import kernels as K
    x = torch.zeros(4, 8, dtype=torch.bfloat16)
    with pytest.raises((RuntimeError, ImportError)):
        K.gemm(x, x)


def test_lr_schedule_matches_oracle():
    from gvl.optim import get_lr
    from oracle.ops import get_lr as ref
    for it in (0, 1, 4, 5, 40, 79, 80, 81, 100):
        assert get_lr(it, 1e-3, 1e-4, 5, 80) == ref(it, 1e-3, 1e-4, 5, 80)


def test_caption_batch_semantics():
    """Synthetic caption batches follow _encode_caption (gpt2_linear/data.py:35-49)."""
    from gvl.train import caption_batch, caption_labels
    z, x, y, m = caption_batch(4, L=17, D=8, T=31, device="cpu")
    assert z.shape == (4, 17, 8) and x.shape == (4, 31) and y.shape == (4, 31)
    assert torch.equal(x[:, 1:], y[:, :-1])
    for b in range(4):
        n = int(m[b].sum())
        # first masked-out target is EOT-padding territory; y[n-1] is the first EOT
        assert y[b, n - 1].item() == 50256
        assert (y[b, n:] == 50256).all()
    lab = caption_labels(y, m)
    assert ((lab == -100) == ~m).all()


def test_residual_tape_hands_the_branch_gradient_over():
    """gvl.functional.ResTapFn (the Q-Former residual streams): identity forward; its backward
    stores the output gradient in the tape — the gradient of the unit's detached residual input
    that LayerNormFn(x, ..., tape) adds — and passes it on unchanged."""
    from gvl import functional as F
    tape = F.ResTape()
    x = torch.randn(3, 4, requires_grad=True)
    y = F.ResTapFn.apply(x * 2.0, tape)
    assert torch.equal(y, x * 2.0) and tape.d is None
    g = torch.randn(3, 4)
    y.backward(g)
    assert torch.equal(tape.d, g)
    assert torch.allclose(x.grad, 2.0 * g)


def test_backward_seed_is_cached_per_accumulation():
    """gvl.train seeds loss.backward() with one cached 1/accum scalar per (device, dtype, accum),
    so a captured step replays no fill kernel for it."""
    from gvl import train as T
    loss = torch.tensor(2.0, requires_grad=True)
    s4 = T._grad_seed(loss, 4)
    assert s4 is T._grad_seed(loss, 4) and float(s4) == 0.25
    assert float(T._grad_seed(loss, 1)) == 1.0
    (loss * 3.0).backward(s4)
    assert float(loss.grad) == 0.75
