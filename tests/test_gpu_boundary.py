"""The drop-in boundary under the reference's own train-script usage (round-2 fixes):

  * torch DDP around a gvl model + gvl AdamW (train_gpt2.py:260-287, :457-476;
    gpt2_linear/train.py:118-123, :292-322): the reducer's hooks must fire, grads and
    params must equal the non-DDP run;
  * optimizer resume in the reference's order configure -> load_state_dict -> step
    (train_gpt2.py:314-322);
  * GPTConfig()'s default vocab of 50257 (train_gpt2.py:76-83);
  * out-of-range token ids / targets raise like nn.Embedding / F.cross_entropy.
"""
import copy
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

from tests.helpers import TINY, recipe_params

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def _tiny_gpt(cuda, **over):
    import gvl.gpt2 as g2
    cfg = dict(TINY, **over)
    m = g2.GPT(g2.GPTConfig(**cfg))
    sd = m.state_dict()
    P = recipe_params([(k, tuple(v.shape)) for k, v in sd.items()])
    m.load_state_dict({k: (P[k] if k in P else v) for k, v in sd.items()})
    return m.to(cuda).to(BF), P


def _batches(cuda, n, B=2, T=48, V=512, seed=0):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n):
        ids = torch.randint(0, V, (B * T + 1,), generator=g)
        out.append((ids[:-1].view(B, T).to(cuda), ids[1:].view(B, T).to(cuda)))
    return out


def _reference_loop(model, opt, mbs, n_steps, ddp):
    """train_gpt2.py:457-476 verbatim in structure (autocast, loss/accum, sync toggle on
    the last micro-step, torch clip_grad_norm_ over model.parameters(), lr, step)."""
    norms = []
    for _ in range(n_steps):
        model.train()
        opt.zero_grad()
        for i, (x, y) in enumerate(mbs):
            with torch.autocast(device_type="cuda", dtype=torch.bfloat16):
                _, loss = model(x, y)
            loss = loss / len(mbs)
            if ddp:
                model.require_backward_grad_sync = (i == len(mbs) - 1)
            loss.backward()
        norms.append(float(torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)))
        for g in opt.param_groups:
            g["lr"] = 1e-3
        opt.step()
    return norms


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_torch_ddp_wraps_gvl_model(cuda):
    """world_size-1 RCCL DDP(gvl GPT) + gvl AdamW == the same loop without DDP."""
    from torch.nn.parallel import DistributedDataParallel as DDP
    mbs = _batches(cuda, 3)
    plain, _ = _tiny_gpt(cuda)
    opt = plain.configure_optimizers(0.1, 1e-3, "cuda")
    norms_plain = _reference_loop(plain, opt, mbs, 2, ddp=False)
    grads_plain = torch.cat([p.grad.float().reshape(-1) for p in plain.parameters()])

    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1, device_id=cuda)
    try:
        model, _ = _tiny_gpt(cuda)
        model = DDP(model, device_ids=[0])
        calls = []

        def hook(state, bucket):  # the default all-reduce, counted
            calls.append(bucket.buffer().numel())
            fut = dist.all_reduce(bucket.buffer(), async_op=True).get_future()
            return fut.then(lambda f: f.value()[0])
        model.register_comm_hook(None, hook)
        raw = model.module
        opt2 = raw.configure_optimizers(0.1, 1e-3, "cuda")
        norms_ddp = _reference_loop(model, opt2, mbs, 2, ddp=True)
        grads_ddp = torch.cat([p.grad.float().reshape(-1) for p in raw.parameters()])
        n_params = sum(p.numel() for p in raw.parameters())
        # every parameter went through the reducer once per optimizer step (sync micro-step
        # only), i.e. AccumulateGrad fired for every gvl parameter under DDP
        assert sum(calls) >= 2 * n_params and sum(calls) < 3 * n_params, (sum(calls), n_params)
        err_g = float((grads_ddp - grads_plain).norm() / grads_plain.norm())
        pa = torch.cat([p.float().reshape(-1) for p in plain.parameters()])
        pb = torch.cat([p.float().reshape(-1) for p in raw.parameters()])
        err_p = float((pa - pb).abs().max() / pa.abs().max())
        print(f"DDP vs plain: norms {norms_ddp} vs {norms_plain}; grad rel-L2 {err_g:.2e}; "
              f"param max err {err_p:.2e}; reducer saw {sum(calls)} elements")
        np.testing.assert_allclose(norms_ddp, norms_plain, rtol=1e-2)
        assert err_g < 1e-2 and err_p < 1e-2
        # the arena identity survives the reducer's copy-back
        ga = opt2.grad_arena
        for p, off, n in opt2.arena_layout():
            assert p.grad.data_ptr() == ga[off:off + n].data_ptr()
    finally:
        dist.destroy_process_group()


def test_adamw_resume_in_reference_order(cuda):
    """configure_optimizers -> load_state_dict -> step continues exactly (train_gpt2.py:
    314-322), instead of restarting the moments and bias correction at zero."""
    from gvl.train import train_step
    mbs = _batches(cuda, 2, seed=3)
    loss_fn = lambda m, b: m(b[0], b[1])[1]
    ref, _ = _tiny_gpt(cuda)
    ropt = ref.configure_optimizers(0.1, 1e-3, "cuda")
    for _ in range(3):
        train_step(ref, ropt, mbs, loss_fn, 1e-3)
    a, _ = _tiny_gpt(cuda)
    aopt = a.configure_optimizers(0.1, 1e-3, "cuda")
    for _ in range(2):
        train_step(a, aopt, mbs, loss_fn, 1e-3)
    ckpt = copy.deepcopy({"model": a.state_dict(), "optimizer": aopt.state_dict()})
    b, _ = _tiny_gpt(cuda)
    b.load_state_dict(ckpt["model"])
    bopt = b.configure_optimizers(0.1, 1e-3, "cuda")
    bopt.load_state_dict(ckpt["optimizer"])
    assert bopt._step_count == 2
    train_step(b, bopt, mbs, loss_fn, 1e-3)
    for (n, p), q in zip(ref.named_parameters(), b.parameters()):
        assert torch.equal(p, q), n


def test_default_vocab_50257(cuda):
    """GPTConfig() trains with vocab 50257 (not a multiple of 8): tiny-width model with
    V=509 and the full default config, vs the CPU fp32 oracle on the same bf16 weights."""
    from oracle import models as OM
    for over, T in (({"vocab_size": 509}, 48), ({"vocab_size": 50257, "n_embd": 768, "n_head": 12,
                                                 "n_layer": 12, "block_size": 1024}, 64)):
        V = over["vocab_size"]
        model, P = _tiny_gpt(cuda, **over)
        x, y = _batches(cuda, 1, B=1, T=T, V=V, seed=5)[0]
        logits, loss = model(x, y)
        assert tuple(logits.shape) == (1, T, V)
        loss.backward()
        H, L = over.get("n_head", TINY["n_head"]), over.get("n_layer", TINY["n_layer"])
        Pb = {k: v.to(BF).float().requires_grad_(k == "lm_head.weight") for k, v in P.items()}
        Pb["transformer.wte.weight"] = Pb["lm_head.weight"]
        rl, rloss = OM.gpt_forward(Pb, x.cpu(), L, H, y.cpu())
        rloss.backward()
        e = abs(loss.item() - rloss.item()) / rloss.item()
        el = float((logits.float().cpu() - rl.detach()).abs().max() / rl.detach().abs().max())
        g = model.lm_head.weight.grad.float().cpu()
        rg = Pb["lm_head.weight"].grad
        eg = float((g - rg).norm() / rg.norm())
        print(f"V={V}: loss {loss.item():.6f} oracle {rloss.item():.6f} rel {e:.2e}; logits "
              f"{el:.2e}; wte grad rel-L2 {eg:.2e}")
        assert e < 2e-3 and el < 3e-2 and eg < 5e-2


def test_out_of_range_ids_raise(cuda):
    """Synchronous checks (the first gvl.functional.SYNC_CHECKS calls of a process) raise at
    the op, like nn.Embedding / F.cross_entropy; later ones are asynchronous and raise on a
    following call once the device verdict has landed (no host sync per micro-step)."""
    from gvl import functional as Fn
    Fn._ID_CHECKS[0] = 0
    Fn._ID_INFLIGHT.clear()
    model, _ = _tiny_gpt(cuda)
    x, y = _batches(cuda, 1)[0]
    bad = x.clone()
    bad[0, 3] = TINY["vocab_size"]
    with pytest.raises(IndexError):
        model(bad, y)
    neg = x.clone()
    neg[1, 0] = -1
    with pytest.raises(IndexError):
        model(neg)
    ybad = y.clone()
    ybad[0, 0] = TINY["vocab_size"] + 7
    with pytest.raises(IndexError):
        model(x, ybad)
    yign = y.clone()
    yign[0, :5] = -100  # ignore_index stays legal
    _, loss = model(x, yign)
    assert torch.isfinite(loss)
    # asynchronous mode: the bad id does not stall the op; it raises on a later call
    Fn._ID_CHECKS[0] = Fn.SYNC_CHECKS
    with pytest.raises(IndexError, match="asynchronously"):
        model(bad, y)  # (may already raise here: the target check polls the id verdict)
        torch.cuda.synchronize()
        model(x, y)
    model(x, y)  # the verdict queue is clear again
    torch.cuda.synchronize()
    Fn._poll_id_checks()


def test_checkpoint_manager_resume_with_arenas(cuda, tmp_path):
    """gvl.checkpoint round trip of a gvl-AdamW run (fp32 masters + moments in arenas):
    save at step 2, resume into a fresh model + optimizer, continue == uninterrupted."""
    from gvl.checkpoint import CheckpointManager
    from gvl.train import train_step
    mbs = _batches(cuda, 2, seed=9)
    loss_fn = lambda m, b: m(b[0], b[1])[1]
    ref, _ = _tiny_gpt(cuda)
    ropt = ref.configure_optimizers(0.1, 1e-3, "cuda")
    a, _ = _tiny_gpt(cuda)
    aopt = a.configure_optimizers(0.1, 1e-3, "cuda")
    mgr = CheckpointManager(str(tmp_path), a, aopt, save_every=2)
    for step in range(3):
        train_step(ref, ropt, mbs, loss_fn, 1e-3)
        if step < 2:
            train_step(a, aopt, mbs, loss_fn, 1e-3)
            mgr.maybe_save_rolling(step + 1, False, 5.0)
    b, _ = _tiny_gpt(cuda)
    bopt = b.configure_optimizers(0.1, 1e-3, "cuda")
    start = CheckpointManager(str(tmp_path), b, bopt).resume(map_location=cuda)
    assert start == 3
    train_step(b, bopt, mbs, loss_fn, 1e-3)
    for (n, p), q in zip(ref.named_parameters(), b.parameters()):
        assert torch.equal(p, q), n


def test_shard_loader_device_prefetch(cuda, tmp_path):
    """gvl.data.DataLoaderLite(device='cuda'): pinned async prefetch returns the same windows
    as the host path (train_gpt2.py:177-187)."""
    from gvl.data import DataLoaderLite
    rng = np.random.default_rng(0)
    for i, n in enumerate((900, 1300)):
        np.save(tmp_path / f"fw_train_{i:06d}.npy", rng.integers(0, 50257, n).astype(np.uint16))
    for rank in range(2):
        h = DataLoaderLite(2, 32, rank, 2, "train", data_root=str(tmp_path))
        d = DataLoaderLite(2, 32, rank, 2, "train", data_root=str(tmp_path), device=cuda)
        for _ in range(25):
            (hx, hy), (dx, dy) = h.next_batch(), d.next_batch()
            assert dx.is_cuda and torch.equal(hx, dx.cpu()) and torch.equal(hy, dy.cpu())


def test_cross_attention_module_forward(cuda):
    """CrossAttention is callable on its own (gpt2_cross-att/model.py:46-58): output and
    input / weight gradients vs an fp32 torch restatement on the same bf16-valued inputs."""
    import gvl.cross_att as xa
    import torch.nn.functional as F
    cfg = xa.GPTConfig(block_size=64, vocab_size=512, n_layer=2, n_head=2, n_embd=128)
    mod = xa.CrossAttention(cfg)
    sd = mod.state_dict()
    P = recipe_params([(k, tuple(v.shape)) for k, v in sd.items()])
    mod.load_state_dict(P)
    mod = mod.to(cuda).to(BF)
    g = torch.Generator().manual_seed(3)
    x = (torch.randn(2, 24, 128, generator=g)).to(BF)
    z = (torch.randn(2, 33, 128, generator=g)).to(BF)
    xg, zg = x.to(cuda).requires_grad_(True), z.to(cuda).requires_grad_(True)
    y = mod(xg, zg)
    dy = torch.randn(y.shape, generator=g).to(BF)
    y.backward(dy.to(cuda))
    # fp32 reference on the bf16-valued parameters / inputs
    W = {k: v.detach().float().cpu().requires_grad_(True) for k, v in mod.state_dict().items()}
    xr, zr = x.float().requires_grad_(True), z.float().requires_grad_(True)
    q = F.linear(xr, W["q_proj.weight"], W["q_proj.bias"])
    kv = F.linear(zr, W["kv_proj.weight"], W["kv_proj.bias"])
    k, v = kv.split(128, 2)
    sh = lambda t, n: t.view(2, n, 2, 64).transpose(1, 2)  # noqa: E731
    o = F.scaled_dot_product_attention(sh(q, 24), sh(k, 33), sh(v, 33), is_causal=False)
    yr = F.linear(o.transpose(1, 2).reshape(2, 24, 128), W["c_proj.weight"], W["c_proj.bias"])
    yr.backward(dy.float())
    rel = lambda a, b: float((a.float().cpu() - b).norm() / b.norm())  # noqa: E731
    errs = dict(y=rel(y.detach(), yr.detach()), dx=rel(xg.grad, xr.grad), dz=rel(zg.grad, zr.grad),
                dq_w=rel(mod.q_proj.weight.grad, W["q_proj.weight"].grad),
                dkv_w=rel(mod.kv_proj.weight.grad, W["kv_proj.weight"].grad),
                dc_w=rel(mod.c_proj.weight.grad, W["c_proj.weight"].grad))
    print("CrossAttention.forward rel-L2 vs fp32:", errs)
    assert max(errs.values()) < 2e-2, errs


def test_feature_shard_loader_feeds_caption_step(cuda, tmp_path):
    """Feature shards (gvl.features) -> pinned one-ahead device batches -> pooled z ->
    gvl.train.train_step of the tiny linear caption model; the pooled batch equals pooling
    the gathered rows."""
    import gvl.caption as cap
    import gvl.gpt2 as g2
    from gvl.features import CaptionFeatureDataset, CaptionFeatureLoader, FeatureShardWriter
    from gvl.train import train_step
    gen = torch.Generator().manual_seed(1)
    feats = torch.randn(12, 257, TINY["n_embd"], generator=gen)
    w = FeatureShardWriter(str(tmp_path), rows_per_shard=5)
    w.add(feats)
    w.close()
    caps = [[list(torch.randint(0, 511, (int(n),), generator=gen).tolist())]
            for n in torch.randint(3, 30, (12,), generator=gen)]
    ds = CaptionFeatureDataset(str(tmp_path), caps, max_len=25, eot=511, seed=0)
    loader = CaptionFeatureLoader(ds, 4, device=cuda, shuffle=True, seed=0)
    lm = cap.GPT_previous(g2.GPTConfig(**TINY))
    model = cap.LinearCaption(enc_dim=TINY["n_embd"], lm=lm, m_vis_tokens=32).to(cuda).to(BF)
    opt = model.configure_optimizers(0.1, 1e-3, "cuda")
    n = 0
    for z, x, y, m, lab in loader:
        assert z.shape == (4, 33, TINY["n_embd"]) and x.shape == (4, 24)
        r = train_step(model, opt, [(z, x, lab)], lambda mm, b: mm(b[0], b[1], labels=b[2])[1],
                       1e-3)
        assert torch.isfinite(r.loss)
        n += 1
    assert n == 3
    # pooled rows == pooling the rows the dataset holds (fp16 shards)
    idx = list(range(12))
    import random
    random.Random(0).shuffle(idx)
    z0 = cap.pool_clip_197_to_33_avg_with_cls(feats.to(torch.float16)[idx[:4]].float().to(cuda))
    z, *_ = next(iter(CaptionFeatureLoader(ds, 4, device=cuda, shuffle=True, seed=0)))
    assert torch.allclose(z.float(), z0.float(), atol=1e-6)


def test_deferred_wgrad_survives_failed_backward(cuda):
    """A backward that raises after blocks queued deferred weight gradients (their flush
    callback never runs) must not disturb later steps: the next optimizer step's gradients
    and updated parameters equal a clean run's, bit for bit (gvl/functional.py deferral is
    keyed per autograd graph task; zero_grad drops the stale queue)."""
    from gvl import functional as Fn
    from gvl.train import train_step
    mbs = _batches(cuda, 2, seed=13)
    loss_fn = lambda m, b: m(b[0], b[1])[1]
    ref, _ = _tiny_gpt(cuda)
    ropt = ref.configure_optimizers(0.1, 1e-3, "cuda")
    train_step(ref, ropt, mbs, loss_fn, 1e-3)
    m, _ = _tiny_gpt(cuda)
    opt = m.configure_optimizers(0.1, 1e-3, "cuda")
    opt.zero_grad()

    class Boom(RuntimeError):
        pass
    def boom(g):
        raise Boom()

    def hook(mod, a, out):
        out.register_hook(boom)
    h = m.transformer.h[0].register_forward_hook(hook)
    _, loss = m(*mbs[0])
    with pytest.raises(Boom):
        loss.backward()
    h.remove()
    assert Fn._PENDING, "the aborted backward should have left deferred entries"
    train_step(m, opt, mbs, loss_fn, 1e-3)
    assert not Fn._PENDING and not Fn._PENDING_B
    for (n, p), q in zip(ref.named_parameters(), m.parameters()):
        assert torch.equal(p.grad, q.grad), n
        assert torch.equal(p, q), n
