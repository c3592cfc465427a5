"""Batched weight-gradient GEMMs of the LM step (gvl_gemm_batched, one persistent launch for
the 12 blocks' dW += dY^T X of one shape, fused bias column sums) against the hipBLASLt
yardstick (torch.bmm over the same transposed views, no accumulate, no bias), HIP events,
median of 5 x 10 launches.  python tools/wgrad_diag.py [K]  (K = tokens per micro-step,
default 16384 = B 16 x T 1024).  Last line: all 48 problems as ONE grouped launch
(gvl_gemm_grouped, the default LM flush since round 4) against the sum of the four batches."""
import os
import ctypes as C
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-vision-language_amd")]
from gvl import _lib  # noqa: E402
from gvl import kernels as K  # noqa: E402

_lib.load()
dev = torch.device("cuda:0")
KT = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
L = 12
SHAPES = [("c_attn", 2304, 768), ("attn.c_proj", 768, 768), ("c_fc", 3072, 768), ("mlp.c_proj", 768, 3072)]


def timeit(fn, reps=10, rounds=5):
    t = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        t.append(e0.elapsed_time(e1) * 1e3 / reps)
    return statistics.median(t)


torch.manual_seed(0)
ALL, tot_b, tot_fl = [], 0.0, 0.0
for name, M, N in SHAPES:
    dy = [(torch.rand(KT, M, device=dev) - 0.5).to(torch.bfloat16) for _ in range(L)]
    x = [(torch.rand(KT, N, device=dev) - 0.5).to(torch.bfloat16) for _ in range(L)]
    g = [torch.zeros(M, N, device=dev, dtype=torch.bfloat16) for _ in range(L)]
    db = [torch.zeros(M, device=dev, dtype=torch.bfloat16) for _ in range(L)]
    items = [(dy[i], x[i], g[i], True) for i in range(L)]
    fl = 2.0 * M * N * KT * L
    tb = timeit(lambda: K.gemm_batched(items, a_mn=True, b_mn=True, dbias=db))
    tn = timeit(lambda: K.gemm_batched(items, a_mn=True, b_mn=True))
    K.gemm_batched(items, a_mn=True, b_mn=True)
    buf = C.create_string_buffer(128)
    _lib.lib().gvl_gemm_batched_kernel_name(buf, 128)
    kname = buf.value.decode()
    DY, X = torch.stack(dy), torch.stack(x)
    ty = timeit(lambda: torch.bmm(DY.transpose(1, 2), X))
    print(f"{name:12s} M={M:5d} N={N:5d} K={KT} x{L}: gvl+dbias {tb:8.1f}us ({fl / tb / 1e6:6.0f} TF/s)  "
          f"gvl {tn:8.1f}us ({fl / tn / 1e6:6.0f} TF/s)  torch.bmm {ty:8.1f}us ({fl / ty / 1e6:6.0f} TF/s)  [{kname}]",
          flush=True)
    tot_b += tb
    tot_fl += fl
    ALL.append((dy, x, g, db))
    del items, DY, X
    torch.cuda.empty_cache()
gitems = [(f[0][i], f[1][i], f[2][i]) for i in range(L) for f in ALL]
gdb = [f[3][i] for i in range(L) for f in ALL]
assert K.gemm_grouped(gitems, dbias=gdb)
_lib.lib().gvl_gemm_batched_kernel_name(buf, 128)
tg = timeit(lambda: K.gemm_grouped(gitems, dbias=gdb))
print(f"grouped x{len(gitems)} (+dbias): {tg:8.1f}us ({tot_fl / tg / 1e6:6.0f} TF/s)  vs the four batches "
      f"{tot_b:8.1f}us ({tot_fl / tot_b / 1e6:6.0f} TF/s)  [{buf.value.decode()}]", flush=True)

# The tied lm_head's weight gradient (dW = dlogits^T x over the micro-step's tokens, 50304 x 768)
# alone, and grouped with the 36 c_attn / c_fc / mlp.c_proj problems (GVL_WGRAD_LM=1): whole
# rounds of CUs across all of them instead of per-batch partial last rounds.
if os.environ.get("GVL_WGRAD_LM", "0") == "1":
    V = 50304
    dl = (torch.rand(KT, V, device=dev) - 0.5).to(torch.bfloat16)
    xl = (torch.rand(KT, 768, device=dev) - 0.5).to(torch.bfloat16)
    gl = torch.zeros(V, 768, device=dev, dtype=torch.bfloat16)
    fl_lm = 2.0 * V * 768 * KT
    t_lm = timeit(lambda: K.gemm(dl, xl, a_mn=True, b_mn=True, out=gl, residual=gl))
    print(f"lm_head dW   M={V} N=768 K={KT}: {t_lm:8.1f}us ({fl_lm / t_lm / 1e6:6.0f} TF/s)", flush=True)
    sel = [0, 2, 3]  # c_attn, c_fc, mlp.c_proj
    fl_sel = sum(2.0 * SHAPES[s][1] * SHAPES[s][2] * KT * L for s in sel) + fl_lm
    blk = [(ALL[s][0][i], ALL[s][1][i], ALL[s][2][i]) for s in sel for i in range(L)]
    blk_db = [ALL[s][3][i] for s in sel for i in range(L)]
    tsep = {}
    for s in sel:
        items = [(ALL[s][0][i], ALL[s][1][i], ALL[s][2][i], True) for i in range(L)]
        tsep[s] = timeit(lambda: K.gemm_batched(items, a_mn=True, b_mn=True, dbias=ALL[s][3]))
    sep = sum(tsep.values()) + t_lm
    print(f"separate: batches {' + '.join(f'{tsep[s]:.1f}' for s in sel)} + lm_head {t_lm:.1f} = {sep:8.1f}us "
          f"({fl_sel / sep / 1e6:6.0f} TF/s)", flush=True)
    for order in ("lm_last", "lm_first"):
        its = blk + [(dl, xl, gl)] if order == "lm_last" else [(dl, xl, gl)] + blk
        dbs = blk_db + [None] if order == "lm_last" else [None] + blk_db
        for bn in ("auto", "256", "192"):
            if bn == "auto":
                os.environ.pop("GVL_W4X_GR_BN", None)
            else:
                os.environ["GVL_W4X_GR_BN"] = bn
            assert K.gemm_grouped(its, dbias=dbs)
            _lib.lib().gvl_gemm_batched_kernel_name(buf, 128)
            tg = timeit(lambda: K.gemm_grouped(its, dbias=dbs))
            print(f"grouped x{len(its)} {order} bn={bn}: {tg:8.1f}us ({fl_sel / tg / 1e6:6.0f} TF/s)  "
                  f"[{buf.value.decode()}]", flush=True)
    os.environ.pop("GVL_W4X_GR_BN", None)
