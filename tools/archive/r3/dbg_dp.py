"""Debug: 2 ranks on one GPU over gloo, gvl GPT (4 layers) + gvl AdamW + GradBuckets: after
accumulate(), which parameters' gradients differ between the ranks?"""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-vision-language_amd")]


def main(rank, port, variant):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    from tests.test_gpu_dp import LM_LOSS, _gpt, _lm_batches
    from gvl import _lib
    from gvl.dist import GradBuckets
    from gvl.train import accumulate
    _lib.load()
    dev = torch.device("cuda:0")
    m = _gpt(dev)
    opt = m.configure_optimizers(0.1, 1e-3, "cuda")
    mb, ov = variant
    import gvl.dist as D0
    log = []
    orig = D0.GradBuckets._on_grad
    nm = {id(p): n for n, p in m.named_parameters()}

    def traced(self, p):
        import traceback
        stk = traceback.extract_stack()
        src = stk[-2].name if len(stk) >= 2 else "C++"
        log.append((nm.get(id(p), "?"), src, self.sync, list(self._pending)))
        return orig(self, p)
    D0.GradBuckets._on_grad = traced
    bk = GradBuckets(opt, bucket_mb=mb, model=m, overlap_blocks=ov)
    mbs = _lm_batches(dev, 2, seed=100 + rank)
    import gvl.dist as D
    real = D._avg
    snaps = []

    import traceback

    def spy(t, pg, async_op):
        if rank == 0:
            st = [f"{f.name}:{f.lineno}" for f in traceback.extract_stack()[-8:-1]]
            print(f"reduce of {t.numel()} at ready-count {len(ready)}: {st}", flush=True)
        r = real(t, pg, async_op)
        torch.cuda.synchronize()
        snaps.append((t.data_ptr(), t.numel(), t.clone()))
        return r
    D._avg = spy
    from gvl import functional as F
    ready = []
    F.register_grad_ready_hook(lambda p: ready.append(names_of[id(p)]))
    names_of = {id(p): n for n, p in m.named_parameters()}
    accumulate(m, opt, mbs, LM_LOSS, bk)
    torch.cuda.synchronize()
    D._avg = real
    arena = opt.grad_arena
    base = arena.data_ptr()
    lay = {id(p): (o, n) for p, o, n in opt.arena_layout()}
    rows = []
    for pn, p in m.named_parameters():
        o, n = lay[id(p)]
        for ptr, cnt, snap in snaps:
            so = (ptr - base) // 2
            if so <= o and o + n <= so + cnt:
                sv = snap[o - so:o - so + n]
                cur = arena[o:o + n]
                ck = torch.tensor([float(sv.float().sum()), float(cur.float().sum())], dtype=torch.float64)
                allck = [torch.zeros_like(ck) for _ in range(2)]
                dist.all_gather(allck, ck)
                rows.append((pn, "changed" if not torch.equal(sv, cur) else "same",
                             "reduce-consistent" if allck[0][0] == allck[1][0] else "REDUCE-DIFFERS"))
    if rank == 0:
        pass
    bad = []
    for n, p in m.named_parameters():
        s = torch.tensor([float(p.grad.float().sum()), float(p.grad.float().norm())], dtype=torch.float64)
        o = [torch.zeros_like(s) for _ in range(2)]
        dist.all_gather(o, s)
        if not torch.equal(o[0], o[1]):
            bad.append(n)
    if rank == 0:
        print(f"variant bucket_mb={mb} overlap={ov}: {len(bk.buckets)} buckets, launch order "
              f"{bk.launch_log}; differing grads: {bad}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    for variant in [(1000.0, 0), (0.05, 4), (0.05, 0)]:
        import socket
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        mp.spawn(main, args=(port, variant), nprocs=2)
