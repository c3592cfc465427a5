"""The captured training step (gvl.graph.GraphedStep) on the MI355X.

* replaying the graph is the same computation as the eager step: after identical
  initialisation, 1 eager warm-up + 2 replays == 3 eager steps, bit for bit, for the LM
  (no dropout) — lr and the AdamW step count reach the kernel from the device block;
* with dropout on (Q-Former bridge in train mode) every replay re-keys the masks through
  the device step offset: consecutive replays on frozen weights give different losses,
  and a replay with the offset rewound reproduces the earlier loss exactly.
(HIP events recorded during capture cannot time replayed kernels on ROCm 7 —
hipEventElapsedTime returns hipErrorInvalidHandle, tools/probe_graph_events.py — so
bench.py times kernels with events in a separate eager pass.)
"""
import pytest
import torch

from tests.helpers import TINY, recipe_params

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def _gpt(cuda):
    import gvl.gpt2 as g2
    m = g2.GPT(g2.GPTConfig(**TINY))
    sd = m.state_dict()
    P = recipe_params([(k, tuple(v.shape)) for k, v in sd.items() if not k.endswith("attn.bias")])
    m.load_state_dict({k: (P[k] if k in P else v) for k, v in sd.items()})
    return m.to(cuda).to(BF).train()


def _batches(cuda, n=2, B=2, T=64, V=None):
    V = V or TINY["vocab_size"]
    g = torch.Generator().manual_seed(5)
    out = []
    for _ in range(n):
        ids = torch.randint(0, V, (B, T + 1), generator=g)
        out.append((ids[:, :-1].contiguous().to(cuda), ids[:, 1:].contiguous().to(cuda)))
    return out


def test_graphed_lm_step_matches_eager(cuda):
    from gvl.graph import GraphedStep
    from gvl.train import train_step
    lrs = [3e-4, 5e-4, 7e-4]
    loss_fn = lambda m, b: m(b[0], b[1])[1]  # noqa: E731

    m1 = _gpt(cuda)
    o1 = m1.configure_optimizers(0.1, 1e-3, "cuda")
    b1 = _batches(cuda)
    eager = [train_step(m1, o1, b1, loss_fn, lr) for lr in lrs]
    torch.cuda.synchronize()

    m2 = _gpt(cuda)
    o2 = m2.configure_optimizers(0.1, 1e-3, "cuda")
    b2 = _batches(cuda)
    gs = GraphedStep(m2, o2, b2, loss_fn, lrs[0], warmup=1)
    got = [float(gs(lr).loss) for lr in lrs[1:]]
    torch.cuda.synchronize()
    ref = [float(r.loss) for r in eager[1:]]
    print("eager", ref, "graph", got)
    assert got == ref
    for (n, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        assert torch.equal(p1, p2), n
    assert o2._step_count == 3
    # lifecycle: close() resets the graph (idempotent), a closed step refuses to replay,
    # and the weights it trained stay usable eagerly
    from gvl.graph import live_steps
    assert gs in live_steps()
    gs.close()
    gs.close()
    assert gs.closed and gs not in live_steps()
    with pytest.raises(RuntimeError):
        gs(lrs[0])
    assert torch.isfinite(train_step(m2, o2, b2, loss_fn, lrs[0]).loss).item()


def test_graphed_dropout_masks_advance(cuda):
    import gvl.caption as cap
    import gvl.gpt2 as g2
    from gvl import kernels as K
    from gvl.graph import GraphedStep
    lm = cap.GPT_previous(g2.GPTConfig(**TINY))
    m = cap.QFormerCaption(enc_dim=TINY["n_embd"], lm=lm, m_vis_tokens=32)
    m = m.to(cuda).to(BF).train()
    opt = m.configure_optimizers(0.1, 1e-3, "cuda")
    g = torch.Generator().manual_seed(3)
    z = torch.randn(4, 33, TINY["n_embd"], generator=g).to(cuda)
    x = torch.randint(0, TINY["vocab_size"], (4, 15), generator=g).to(cuda)
    lab = torch.randint(0, TINY["vocab_size"], (4, 15), generator=g).to(cuda)
    loss_fn = lambda mm, b: mm(b[0], b[1], labels=b[2])[1]  # noqa: E731
    gs = GraphedStep(m, opt, [(z, x, lab)], loss_fn, 0.0, warmup=1)
    off = K.seed_offset(cuda)
    start = int(off.item())
    # lr 0: decoupled decay p*(1 - lr*wd) and the Adam update vanish, so the weights stay
    # fixed and only the dropout masks move
    la = float(gs(0.0).loss)
    lb = float(gs(0.0).loss)
    assert int(off.item()) == start + 2
    assert la != lb
    off.fill_(start)
    la2 = float(gs(0.0).loss)
    assert la2 == la

