"""The data-parallel path on CPU with gloo, world_size 2: bucketed
gradient all-reduce over arena slices fired from post-accumulate-grad hooks, loss
all-reduce, and the DP equivalence invariant (2 ranks x B == 1 rank x 2B)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class ArenaSGD(torch.optim.SGD):
    """CPU stand-in exposing the gvl.optim.AdamW arena interface (flat grad arena whose
    slices are parameter .grad views) so gvl.dist.GradBuckets can be exercised with gloo."""

    def __init__(self, params, lr):
        super().__init__(params, lr=lr)
        ps = [p for g in self.param_groups for p in g["params"]]
        self._layout, off = [], 0
        for p in ps:
            self._layout.append((p, off, p.numel()))
            off += (p.numel() + 7) // 8 * 8
        self._g = torch.zeros(off)
        for p, o, n in self._layout:
            p.grad = self._g[o:o + n].view_as(p)

    def arena_layout(self):
        return self._layout

    @property
    def grad_arena(self):
        return self._g

    def zero_grad(self, set_to_none=True):
        self._g.zero_()


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(16, 64), torch.nn.GELU(), torch.nn.Linear(64, 64),
                               torch.nn.GELU(), torch.nn.Linear(64, 4))


def _data(rank, n=8):
    g = torch.Generator().manual_seed(100 + rank)
    return torch.randn(n, 16, generator=g), torch.randn(n, 4, generator=g)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gvl.dist import GradBuckets
    from gvl.train import train_step
    m = _model()
    opt = ArenaSGD(m.parameters(), lr=0.1)
    # tiny buckets: several per backward, cut from the arena's end
    bk = GradBuckets(opt, bucket_mb=4096 * 4 / (1024 * 1024))
    x, y = _data(rank)
    mbs = [(x[:4], y[:4]), (x[4:], y[4:])]
    res = train_step(m, opt, mbs, lambda mm, b: ((mm(b[0]) - b[1]) ** 2).mean(), lr=0.1,
                     buckets=bk, max_norm=1e9)
    q.put((rank, len(bk.buckets), float(res.loss), [p.detach().numpy().copy() for p in m.parameters()]))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(180)
def test_gloo_two_ranks_match_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=150) for _ in range(2)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    (_, nb0, l0, p0), (_, nb1, l1, p1) = out
    assert nb0 == nb1 and nb0 >= 2, "expected several buckets"
    assert l0 == pytest.approx(l1)
    p0 = [torch.from_numpy(a) for a in p0]
    p1 = [torch.from_numpy(a) for a in p1]
    for a, b in zip(p0, p1):
        assert torch.allclose(a, b), "ranks diverged after the step"
    # single process over the concatenated batch (2 micro-steps of 8): same update
    m = _model()
    opt = torch.optim.SGD(m.parameters(), lr=0.1)
    xs, ys = zip(*[_data(r) for r in range(2)])
    opt.zero_grad()
    # mean over ranks of per-rank mean-over-2-microsteps == mean over all 4 quarter batches
    chunks = [(xs[r][i * 4:(i + 1) * 4], ys[r][i * 4:(i + 1) * 4]) for r in range(2) for i in range(2)]
    loss_ref = sum(((m(a) - b) ** 2).mean() for a, b in chunks) / 4
    loss_ref.backward()
    opt.step()
    assert float(loss_ref) == pytest.approx(l0, rel=1e-6)
    for a, b in zip(m.parameters(), p0):
        assert torch.allclose(a.detach(), b, atol=1e-6), "DP step != single-process step"


class _FusedLinear(torch.autograd.Function):
    """CPU stand-in for a gvl fused unit: the weight gradient is accumulated IN PLACE into the
    arena view (.grad) and announced through gvl.functional's grad-ready hook, bypassing
    AccumulateGrad — exactly how GPTBlockFn & co. feed gvl.dist.GradBuckets."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return x @ w.t()

    @staticmethod
    def backward(ctx, dy):
        from gvl import functional as F
        x, w = ctx.saved_tensors
        w.grad.add_(dy.t() @ x)
        F._ready(w)
        return dy @ w, None


class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.a = torch.nn.Linear(16, 64)
        self.w = torch.nn.Parameter(torch.randn(64, 64) * 0.1)  # the fused-sink parameter
        self.b = torch.nn.Linear(64, 4)

    def forward(self, x):
        h = torch.nn.functional.gelu(self.a(x))
        h = torch.nn.functional.gelu(_FusedLinear.apply(h, self.w))
        return self.b(h)


def _worker_accum(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import gvl.dist as D
    from gvl.train import train_step
    calls = []
    real = D._avg

    def counting(t, pg, async_op):
        calls.append((len(seen), t.numel()))
        return real(t, pg, async_op)
    D._avg = counting
    seen = []
    m = _Net()
    opt = ArenaSGD(m.parameters(), lr=0.1)
    bk = D.GradBuckets(opt, bucket_mb=1024 * 4 / (1024 * 1024))
    x, y = _data(rank, 16)
    mbs = [(x[i * 4:(i + 1) * 4], y[i * 4:(i + 1) * 4]) for i in range(4)]

    def loss_fn(mm, b):
        seen.append(bk.sync)
        return ((mm(b[0]) - b[1]) ** 2).mean()
    res = train_step(m, opt, mbs, loss_fn, lr=0.1, buckets=bk, max_norm=1e9)
    q.put((rank, len(bk.buckets), seen, calls, float(res.loss),
           [p.detach().numpy().copy() for p in m.parameters()]))
    bk.remove()
    dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_gloo_buckets_with_fused_sinks_and_sync_toggle():
    """GradBuckets over the arena with a fused in-place-accumulating parameter, 4 micro-steps:
    sync is off for micro-steps 0-2 and on for 3 (train_gpt2.py:468), every bucket is reduced
    exactly once and only during the last micro-step, and the result equals one process over
    the concatenated batch."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_accum, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=150) for _ in range(2)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for rank, nb, seen, calls, loss, params in out:
        assert len(seen) == 4  # (sync is toggled after each forward, before its backward)
        assert nb >= 2 and len(calls) == nb + 1, (nb, calls)  # every bucket once + the loss
        assert all(step == 4 for step, _ in calls), "a bucket fired before the sync micro-step"
    assert out[0][4] == pytest.approx(out[1][4])
    m = _Net()
    opt = torch.optim.SGD(m.parameters(), lr=0.1)
    chunks = []
    for r in range(2):
        x, y = _data(r, 16)
        chunks += [(x[i * 4:(i + 1) * 4], y[i * 4:(i + 1) * 4]) for i in range(4)]
    opt.zero_grad()
    loss_ref = sum(((m(a) - b) ** 2).mean() for a, b in chunks) / 8
    # _FusedLinear needs an existing .grad to accumulate into (the arena view in gvl)
    m.w.grad = torch.zeros_like(m.w)
    loss_ref.backward()
    opt.step()
    assert float(loss_ref) == pytest.approx(out[0][4], rel=1e-6)
    for a, b in zip(m.parameters(), out[0][5]):
        assert torch.allclose(a.detach(), torch.from_numpy(b), atol=1e-6)


# ------------------------------------------------------------ overlap with backward (A12)
class _Res(torch.nn.Module):
    def __init__(self, d):
        super().__init__()
        self.lin = torch.nn.Linear(d, d)

    def forward(self, x):  # residual inside the block, like GPTBlockFn
        return x + torch.nn.functional.gelu(self.lin(x))


class _Stack(torch.nn.Module):
    """A decoder-shaped toy: input layer, `n` residual blocks, head — so bucket readiness
    and segment cuts follow the same module order as GPT.transformer.h."""

    def __init__(self, n=6, d=32):
        super().__init__()
        torch.manual_seed(0)
        self.inp = torch.nn.Linear(16, d)
        self.h = torch.nn.ModuleList([_Res(d) for _ in range(n)])
        self.head = torch.nn.Linear(d, 4)

    def forward(self, x):
        x = self.inp(x)
        for blk in self.h:
            x = blk(x)
        return self.head(x)


class GroupedArenaSGD(ArenaSGD):
    """Arena laid out like gvl.optim.AdamW: the >=2-D (decay) group first, then the biases,
    each group in module order."""

    def __init__(self, params, lr):
        ps = list(params)
        torch.optim.SGD.__init__(self, [{"params": [p for p in ps if p.dim() >= 2]},
                                        {"params": [p for p in ps if p.dim() < 2]}], lr=lr)
        order = [p for g in self.param_groups for p in g["params"]]
        self._layout, off = [], 0
        for p in order:
            self._layout.append((p, off, p.numel()))
            off += (p.numel() + 7) // 8 * 8
        self._g = torch.zeros(off)
        for p, o, n in self._layout:
            p.grad = self._g[o:o + n].view_as(p)


def _worker_overlap(rank, world, port, q, segmented):
    try:
        _overlap_body(rank, world, port, q, segmented)
    except BaseException as e:  # report instead of leaving the parent waiting
        q.put((rank, repr(e)))
        raise


def _overlap_body(rank, world, port, q, segmented):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import gvl.dist as D
    events = []
    real = D._avg

    def logging_avg(t, pg, async_op):
        events.append(("bucket", t.data_ptr()))
        return real(t, pg, async_op)
    D._avg = logging_avg
    m = _Stack()
    def mark(i):
        def hook(mod, a, out):
            out.register_hook(lambda g: events.append(("bwd", i)))
        return hook
    for i, blk in enumerate(m.h):
        blk.register_forward_hook(mark(i))
    opt = GroupedArenaSGD(m.parameters(), lr=0.1)
    # one bucket per ~block (32x32 weight + bias = 1056 params)
    bk = D.GradBuckets(opt, bucket_mb=1056 * 4 / (1024 * 1024), model=m)
    x, y = _data(rank, 8)
    bk.set_sync(True)
    if segmented:
        segs = D.BackwardSegments([m.h[2], m.h[4]])
        segs.arm(True)
        loss = ((m(x) - y) ** 2).mean()
        n = segs.backward(loss, between=lambda j: events.append(("between", j)))
        assert n == 3
    else:
        loss = ((m(x) - y) ** 2).mean()
        loss.backward()
    bk.wait()
    first_bucket_params = [n for n, p in m.named_parameters() if any(p is b for b in bk.buckets[0][1])]
    q.put((rank, events, [len(r) for r, _ in bk.buckets], first_bucket_params,
           [p.grad.clone().numpy() for p in m.parameters()]))
    dist.destroy_process_group()


@pytest.mark.timeout(180)
@pytest.mark.parametrize("segmented", [False, True])
def test_gloo_buckets_overlap_backward(segmented):
    """The first gradient bucket (the top block's weight AND bias, two arena runs of the
    decay-grouped arena) is all-reduced before the backward of the lowest blocks starts —
    eagerly, and through BackwardSegments (the captured DP step's segment order) — and the
    reduced gradients equal the mean over ranks."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_overlap, args=(r, 2, port, q, segmented)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=150) for _ in range(2)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=30)
    assert all(len(o) == 5 for o in out), out
    for rank, events, runs, first, grads in out:
        kinds = [e[0] if e[0] != "bwd" else f"bwd{e[1]}" for e in events]
        assert "head.weight" in first and "head.bias" in first, first
        assert runs[0] == 2, runs  # weight run + bias run of the grouped arena
        first_b = kinds.index("bucket")
        assert first_b < kinds.index("bwd0"), kinds
        assert first_b < kinds.index("bwd3"), kinds
        if segmented:
            assert kinds.index("between") < kinds.index("bwd3"), kinds
    # reduced gradients: identical on both ranks and equal to the mean of local gradients
    m = _Stack()
    ref = [torch.zeros_like(p) for p in m.parameters()]
    for r in range(2):
        m.zero_grad()
        x, y = _data(r, 8)
        ((m(x) - y) ** 2).mean().backward()
        for a, p in zip(ref, m.parameters()):
            a += p.grad / 2
    for g0, g1, r in zip(out[0][4], out[1][4], ref):
        assert torch.allclose(torch.from_numpy(g0), torch.from_numpy(g1))
        assert torch.allclose(torch.from_numpy(g0), r, atol=1e-6)


class _SharedInputLayer(torch.nn.Module):
    """A Q-Former-like layer: reads the running queries and a shared second input."""

    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(8, 8)
        self.b = torch.nn.Linear(8, 8)

    def forward(self, q, v):
        return q + torch.tanh(self.a(q) + self.b(v).mean(1, keepdim=True))


class _SharedInputBridge(torch.nn.Module):
    def __init__(self, n_layers):
        super().__init__()
        torch.manual_seed(3)
        self.proj = torch.nn.Linear(8, 8)
        self.q0 = torch.nn.Parameter(torch.randn(4, 8))
        self.layers = torch.nn.ModuleList([_SharedInputLayer() for _ in range(n_layers)])

    def forward(self, x):
        v = self.proj(x)
        q = self.q0.unsqueeze(0).expand(x.shape[0], -1, -1)
        for layer in self.layers:
            q = layer(q, v)
        return q


@pytest.mark.parametrize("n_layers", [2, 3, 4])
def test_backward_segments_shared_input_backpropagated_once(n_layers):
    """Every cut reads the projected image tokens v (gpt2_q_former/model.py:166-167).  The
    segmented backward must give the plain backward's gradients AND run the projection's
    backward exactly once — with >= 3 layers a per-segment backward of v used to deliver
    vis_proj's gradient in two graph tasks, so its DP bucket fired on the first partial."""
    import gvl.dist as D
    x = torch.randn(2, 5, 8, generator=torch.Generator().manual_seed(1))
    ref = _SharedInputBridge(n_layers)
    (ref(x) ** 2).sum().backward()
    m = _SharedInputBridge(n_layers)
    fired = []
    for name, p in m.named_parameters():
        p.register_post_accumulate_grad_hook(lambda p, name=name: fired.append(name))
    segs = D.BackwardSegments(list(m.layers)[1:])  # segment_cuts() of a Q-Former bridge
    assert len(segs.cuts) == n_layers - 1
    segs.arm(True)
    loss = (m(x) ** 2).sum()
    assert segs.backward(loss) == n_layers
    for (name, p), pr in zip(m.named_parameters(), ref.parameters()):
        assert torch.allclose(p.grad, pr.grad, atol=1e-6), name
        assert fired.count(name) == 1, (name, fired)


def test_destroy_process_group_closes_live_steps():
    """gvl.dist.destroy_process_group (the reference scripts' teardown, train_gpt2.py:523)
    closes every live captured step bound to the group before the communicator goes, in that
    order, whatever the caller's garbage-collection order (host logic; GraphedStep itself
    needs a GPU: tests/test_gpu_dp.py::test_segmented_graph_step_matches_eager)."""
    import gvl.dist as D
    import gvl.graph as G
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    order = []

    class FakeStep:  # the part of GraphedStep the teardown relies on
        pg = None

        def close(self):
            order.append(("close", dist.is_initialized()))
            G._LIVE.discard(self)

    st = FakeStep()
    G._LIVE.add(st)
    try:
        assert st in G.live_steps()
        D.destroy_process_group()
    finally:
        G._LIVE.discard(st)
        if dist.is_initialized():
            dist.destroy_process_group()
    assert order == [("close", True)]  # closed while the group was still alive
    assert not dist.is_initialized() and st not in G.live_steps()


@pytest.mark.parametrize("stacked", [False, True])
def test_stacked_arena_layout_buckets(stacked):
    """gvl.optim.arena_offsets with `_gvl_stack_key` (the cross-att kv_proj stack): stacked
    parameters take consecutive slots, slots tile the arena without overlap, and GradBuckets
    built from the offset-sorted layout (no model: the arena order is the ready-order proxy)
    covers every parameter once, with runs that are exactly the union of their slots
    (arena_layout's order contract with stacked placement)."""
    from gvl.dist import GradBuckets
    from gvl.optim import _pad, arena_offsets
    torch.manual_seed(0)
    lins = [torch.nn.Linear(24, 16) for _ in range(5)]
    if stacked:
        for li in lins[1:4]:
            li.weight._gvl_stack_key = "kv_w"
            li.bias._gvl_stack_key = "kv_b"
    groups = [{"params": [li.weight for li in lins]}, {"params": [li.bias for li in lins]}]
    offs, seg, total = arena_offsets(groups)
    params = [p for g in groups for p in g["params"]]
    off_of = {id(p): o for p, o in zip(params, offs)}
    slots = sorted((o, o + _pad(p.numel())) for p, o in zip(params, offs))
    assert slots[0][0] == 0 and slots[-1][1] == total
    assert all(a[1] == b[0] for a, b in zip(slots, slots[1:]))  # tiled, no overlap
    if stacked:
        ow = [off_of[id(li.weight)] for li in lins[1:4]]
        assert all(b - a == _pad(lins[1].weight.numel()) for a, b in zip(ow, ow[1:]))

    class Opt:
        def __init__(self):
            self._g = torch.zeros(total)
            self._layout = sorted(((p, o, p.numel()) for p, o in zip(params, offs)),
                                  key=lambda e: e[1])

        def arena_layout(self):
            return self._layout

        @property
        def grad_arena(self):
            return self._g

    bk = GradBuckets(Opt(), bucket_mb=3 * 24 * 16 * 4 / 2**20)
    try:
        seen = [p for _, ps in bk.buckets for p in ps]
        assert len(seen) == len(params) and {id(p) for p in seen} == {id(p) for p in params}
        for runs, ps in bk.buckets:
            covered = sorted((off_of[id(p)], off_of[id(p)] + _pad(p.numel())) for p in ps)
            merged = []
            for a, b in covered:
                if merged and merged[-1][1] == a:
                    merged[-1][1] = b
                else:
                    merged.append([a, b])
            assert [tuple(r) for r in merged] == list(runs)
    finally:
        bk.remove()
