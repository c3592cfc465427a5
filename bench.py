"""bench.py — throughput of the MI355X-native GPT-2 hot path (BASELINE.json metric).

Default workload (configs[1]): GPT-2 124M LM pretrain optimizer step, micro-batch 16 x 1024,
gradient accumulation to 524,288 tokens per step across the job (32 micro-steps at N=1,
4 per rank at N=8, like train_gpt2.py:244-251), bf16, fused AdamW + clip, RCCL all-reduce.
A secondary line item times the Q-Former caption step (B=128 per GPU, accumulation 1,
SURVEY.md D6) — the north star's roofline target.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload lm|qformer|linear|cross]
    torchrun --nproc-per-node N bench.py --gpus N ...

Prints ONE JSON line (rank 0).  Inputs are synthetic (random tokens / N(0,1) CLIP tokens),
resident in HBM before timing; weights random-init with the reference's init recipe.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gpt2-vision-language_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_BF16_TFLOPS = 2516.6  # 256 CU x 4 SIMD x 1024 FLOP/clk (32x32x16 bf16 in 32 cyc) x 2.4 GHz
PEAK_HBM_GBS = 8000.0
METRIC = "training tokens/sec/node, GPT-2-124M seq1024; caption-step images/sec"
# algorithmic work
LM_FLOP_PER_TOKEN = 798.1e6
CAP_FLOP_PER_IMAGE = {"qformer": 35.16e9, "linear": 31.98e9, "cross": 21.04e9}


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # GVL_BENCH_ONE_DEVICE=1: rehearsal of the N > 1 path on a one-GPU box — every rank on
    # cuda:0, collectives over gloo (RCCL refuses two ranks on one device).  Never a bench line.
    one_device = os.environ.get("GVL_BENCH_ONE_DEVICE") == "1"
    if one_device:
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        if one_device:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    return world, rank, torch.device(f"cuda:{local}")


# --------------------------------------------------------------------------- models
def build_lm(dev):
    import gvl.gpt2 as g2
    torch.manual_seed(0)
    m = g2.GPT(g2.GPTConfig(vocab_size=50304))
    return m.to(dev).to(torch.bfloat16)


def build_caption(kind, dev):
    import gvl.caption as cap
    import gvl.cross_att as xa
    import gvl.gpt2 as g2
    torch.manual_seed(0)
    if kind == "cross":
        m = xa.GPT(xa.GPTConfig(vocab_size=50304))
    else:
        lm = cap.GPT_previous(g2.GPTConfig(vocab_size=50304, block_size=1024))
        cls = cap.QFormerCaption if kind == "qformer" else cap.LinearCaption
        m = cls(enc_dim=768, lm=lm, m_vis_tokens=32)
    return m.to(dev).to(torch.bfloat16)


# ------------------------------------------------------------------------- workloads
def run_lm(args, world, rank, dev, timer=None):
    from gvl.dist import GradBuckets
    from gvl.optim import get_lr
    from gvl.train import lm_batch, train_step
    B, T = args.micro_batch, 1024
    total = 524288
    accum = max(1, total // (B * T * world))
    model = build_lm(dev)
    model.train()
    opt = _quiet(lambda: model.configure_optimizers(0.1, 6e-4, "cuda"))
    buckets = GradBuckets(opt, bucket_mb=args.bucket_mb or 32.0, model=model) if world > 1 else None
    batches = [lm_batch(B, T, step=i, rank=rank, device=dev) for i in range(accum)]
    loss_fn = lambda m, b: m(b[0], b[1])[1]

    lr_fn = lambda it: get_lr(it, 6e-4, 6e-5, 715, 19073)  # noqa: E731

    def step(it):
        return train_step(model, opt, batches, loss_fn, lr_fn(it), buckets=buckets)

    step.graph_args = (model, opt, batches, loss_fn, lr_fn)
    step.buckets = buckets
    tokens_per_step = B * T * accum * world
    return step, tokens_per_step, dict(workload="gpt2-124m-lm-pretrain", micro_batch=B,
                                       seq_len=T, grad_accum=accum,
                                       global_batch=B * accum * world,
                                       tokens_per_step=tokens_per_step)


def run_caption(kind, args, world, rank, dev):
    from gvl.caption import pool_clip_197_to_33_avg_with_cls as pool
    from gvl.dist import GradBuckets
    from gvl.optim import get_lr
    from gvl.train import caption_batch, caption_labels, train_step
    B = args.caption_batch
    model = build_caption(kind, dev)
    model.train()
    opt = _quiet(lambda: model.configure_optimizers(0.1, 1e-3, "cuda"))
    # 8 MB buckets: the bridge's gradients become final only inside its own short backward
    # (after the frozen decoder's); with 32 MB the first bucket is issued 0.13 ms before the
    # end of the captured backward, with 8 MB 0.81 ms (profiles/r4/qformer_dp_overlap_r4e.txt)
    buckets = GradBuckets(opt, bucket_mb=args.bucket_mb or 8.0, model=model) if world > 1 else None
    z, x, y, m = caption_batch(B, rank=rank, device=dev)
    if kind == "cross":
        loss_fn = lambda mm, b: mm(b[1], z=pool(b[0]), targets=b[2], target_mask=b[3])[1]
    else:
        lab = caption_labels(y, m)
        loss_fn = lambda mm, b: mm(pool(b[0]), b[1], labels=lab)[1]

    lr_fn = lambda it: get_lr(it, 1e-3, 1e-4, 5, 80)  # noqa: E731

    def step(it):
        return train_step(model, opt, [(z, x, y, m)], loss_fn, lr_fn(it), buckets=buckets)

    step.graph_args = (model, opt, [(z, x, y, m)], loss_fn, lr_fn)
    step.buckets = buckets

    return step, B * world, dict(workload=f"{kind}-caption-step", micro_batch=B, seq_len=31,
                                 grad_accum=1, global_batch=B * world)


def run_pixels(args, world, rank, dev, steps, warmup):
    """BASELINE configs[3]: (B,3,224,224) pixels -> frozen CLIP ViT-L/14 (stock PyTorch-ROCm,
    bf16) -> fused pool -> linear-bridge caption step (gvl).  The caption step is the graphed
    train step fed from a static feature buffer; CLIP runs eagerly before it each step."""
    from gvl.clip import FLOP_PER_IMAGE, CLIPFeatureStage, synthetic_pixels
    from gvl.train import caption_batch, caption_labels
    B = args.caption_batch
    clip = CLIPFeatureStage().to(dev).to(torch.bfloat16)
    pixels = synthetic_pixels(B, device=dev)
    model = build_caption("linear", dev)
    model.train()
    opt = _quiet(lambda: model.configure_optimizers(0.1, 1e-3, "cuda"))
    _, x, y, m = caption_batch(B, rank=rank, device=dev)
    lab = caption_labels(y, m)
    zbuf = torch.empty(B, 33, 768, dtype=torch.bfloat16, device=dev)
    zbuf.copy_(clip.features(pixels))
    loss_fn = lambda mm, b: mm(b[0], b[1], labels=b[2])[1]  # noqa: E731
    from gvl.optim import get_lr
    lr_fn = lambda it: get_lr(it, 1e-3, 1e-4, 5, 80)  # noqa: E731
    if world == 1 and not args.no_graph:
        from gvl.graph import GraphedStep
        gs = GraphedStep(model, opt, [(zbuf, x, lab)], loss_fn, lr_fn(0), warmup=2)
        inner = lambda it: gs(lr_fn(it))  # noqa: E731
    else:
        from gvl.train import train_step
        inner = lambda it: train_step(model, opt, [(zbuf, x, lab)], loss_fn, lr_fn(it))  # noqa: E731

    def step(it):
        zbuf.copy_(clip.features(pixels))
        return inner(it)
    for i in range(warmup):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        clip.features(pixels)
    torch.cuda.synchronize()
    clip_ms = (time.perf_counter() - t0) / steps * 1e3
    t0 = time.perf_counter()
    r = None
    for i in range(steps):
        r = step(warmup + i)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    val = B / dt
    # the same step with the tower's encoder on libgvl (gvl/clip.py native=True, same weights;
    # reported beside the stock-tower value the north star names, not instead of it)
    clip.native = True
    for i in range(2):
        step(warmup + steps + i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        clip.features(pixels)
    torch.cuda.synchronize()
    nclip_ms = (time.perf_counter() - t0) / steps * 1e3
    t0 = time.perf_counter()
    for i in range(steps):
        step(warmup + steps + 2 + i)
    torch.cuda.synchronize()
    ndt = (time.perf_counter() - t0) / steps
    clip.native = False
    native = dict(value=round(B / ndt, 1), unit="images/s", ms_per_step=round(ndt * 1e3, 3),
                  clip_ms_per_batch=round(nclip_ms, 3),
                  step_mfma_frac=round(B / ndt * (FLOP_PER_IMAGE + CAP_FLOP_PER_IMAGE["linear"])
                                       / 1e12 / PEAK_BF16_TFLOPS, 4),
                  clip="ViT-L/14 encoder on libgvl (packed qkv GEMM, gvl flash attention, "
                       "bias+residual / bias+quick-GELU GEMM epilogues, gvl LayerNorm)")
    return dict(value=round(val, 1), unit="images/s", ms_per_step=round(dt * 1e3, 3),
                clip_ms_per_batch=round(clip_ms, 3), native_clip=native,
                step_mfma_frac=round(val * (FLOP_PER_IMAGE + CAP_FLOP_PER_IMAGE["linear"]) / 1e12
                                     / PEAK_BF16_TFLOPS, 4),
                loss=round(float(r.loss), 5),
                config=dict(workload="linear-caption-step-pixels", micro_batch=B,
                            image="3x224x224", clip="ViT-L/14 (stock PyTorch-ROCm, bf16, SDPA)",
                            pool="fused before the visual projection (gvl)", seq_len=31,
                            grad_accum=1, global_batch=B))


def _quiet(fn):
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        return fn()


def graphed(step, warmup):
    """Capture the step into hipGraphs (gvl.graph) after `warmup` eager steps: one graph at
    N=1; at N>1 the last micro-step's backward in segments, each its own graph, with the
    buckets a segment finalised all-reduced on RCCL's stream while the next segment runs."""
    from gvl.graph import GraphedStep
    model, opt, batches, loss_fn, lr_fn = step.graph_args
    gs = GraphedStep(model, opt, batches, loss_fn, lr_fn(0), warmup=warmup,
                     buckets=getattr(step, "buckets", None))
    return lambda it: gs(lr_fn(it))


def kernel_pass(step, first_it, steps, timer):
    """Per-GEMM HIP-event timing for the roofline line.  Events recorded while a hipGraph
    is captured cannot time its replayed kernels on ROCm 7 (hipEventElapsedTime ->
    hipErrorInvalidHandle; tools/probe_graph_events.py), so with graphs on, the same step
    (same kernels, shapes and data) runs eagerly for `steps` steps with an event pair
    around every GEMM launch on its stream; rocprofv3 sees both kinds of launch."""
    from gvl import kernels as K
    torch.cuda.synchronize()
    K.set_kernel_timer(timer)
    try:
        for i in range(steps):
            step(first_it + i)
    finally:
        K.set_kernel_timer(None)
    torch.cuda.synchronize()


def timed(step, steps, warmup, world, timer=None, graph=False, kernel_steps=1):
    """Time exactly `steps` steps (barrier + synchronize on both sides, max over ranks);
    then, outside the timed region, one eager kernel pass of `kernel_steps` steps with the
    per-GEMM dispatch timer (the roofline line)."""
    eager = step
    if graph:
        step = graphed(step, warmup)
    else:
        for i in range(warmup):
            step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = None
    for i in range(steps):
        r = step(warmup + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    loss, norm = float(r.loss), float(r.norm)  # read before the kernel pass moves the model
    if timer is not None:
        kernel_pass(eager, warmup + steps, kernel_steps, timer)
    return dt, (loss, norm)


TRAFFIC_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "pmc_traffic.json")


def pmc_record(workload, kernel):
    """The committed PMC passes of the same bench command for `kernel` (tools/pmc_traffic.sh:
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / MFMA-busy + GRBM in separate runs): HBM bytes per
    launch (FETCH_SIZE doubled per the gfx950 correction), MFMA-busy fraction and achieved
    clock; {} when not measured."""
    try:
        with open(TRAFFIC_FILE) as f:
            t = json.load(f)["workloads"][{"qformer": "qf"}.get(workload, workload)]
        return t[kernel]
    except (OSError, KeyError, ValueError):
        return {}


def pmc_traffic(workload, kernel):
    return pmc_record(workload, kernel).get("hbm_bytes")


def dominant_kernel(summary, workload="lm", steps=1, full=False):
    """Roofline of the GEMM instance with the largest total time.  Durations come from HIP
    events bound to each kernel's own dispatch (gvl.kernels.KernelTimer, dispatch=True):
    the interval rocprofv3's kernel trace reports for the same kernel name.  Also lists the
    top GEMM instances (per-step launches, average duration, fraction of peak).  Every GEMM
    is one of libgvl's own kernels (since ABI v10: no vendor-library route)."""
    name, s = max(summary.items(), key=lambda kv: kv[1]["ms"])
    avg_ms = s["ms"] / s["launches"]
    achieved = s["flops"] / (s["ms"] * 1e-3) / 1e12
    top = sorted(summary.items(), key=lambda kv: -kv[1]["ms"])[:6]
    table = [dict(kernel=k, launches_per_step=round(v["launches"] / steps, 2),
                  ms_per_step=round(v["ms"] / steps, 3),
                  avg_us=round(v["ms"] / v["launches"] * 1e3, 2),
                  frac=round(v["flops"] / (v["ms"] * 1e-3) / 1e12 / PEAK_BF16_TFLOPS, 4),
                  mfma_busy=pmc_record(workload, k).get("mfma_busy"),
                  clock_ghz=pmc_record(workload, k).get("clock_ghz"),
                  mfma_rate_frac=pmc_record(workload, k).get("mfma_rate_frac"),
                  traffic=pmc_record(workload, k).get("hbm_bytes"))
             for k, v in top]
    return dict(kernel=name, bound="mfma", achieved=round(achieved, 1), peak=PEAK_BF16_TFLOPS,
                unit="TFLOP/s", frac=round(achieved / PEAK_BF16_TFLOPS, 4),
                traffic=pmc_traffic(workload, name), traffic_unit="bytes/launch",
                mfma_busy=pmc_record(workload, name).get("mfma_busy"),
                clock_ghz=pmc_record(workload, name).get("clock_ghz"),
                mfma_rate_frac=pmc_record(workload, name).get("mfma_rate_frac"),
                launches=s["launches"], avg_launch_us=round(avg_ms * 1e3, 2),
                avg_flop_per_launch=s["flops"] / s["launches"],
                timing="hip events bound to the kernel dispatch (hipExtLaunchKernelGGL), "
                       "eager pass of the same step",
                all_gemm_frac=round(sum(v["flops"] for v in summary.values())
                                    / (sum(v["ms"] for v in summary.values()) * 1e-3) / 1e12
                                    / PEAK_BF16_TFLOPS, 4),
                gemm_ms_per_step=round(sum(v["ms"] for v in summary.values()) / steps, 3),
                top_gemms=table,
                # --gemm-table: every GEMM instance of the step (tools/qformer_budget.py)
                **({"all_gemms": [dict(kernel=k, launches_per_step=round(v["launches"] / steps, 2),
                                       avg_us=round(v["ms"] / v["launches"] * 1e3, 2),
                                       gflop_per_launch=round(v["flops"] / v["launches"] / 1e9, 3))
                                  for k, v in sorted(summary.items(), key=lambda kv: -kv[1]["ms"])]}
                   if full else {}))


# ---------------------------------------------------------------------- CPU baseline
def host_threads():
    """Threads this process may use: the affinity mask (the GPU box's share; os.cpu_count()
    there reports the whole machine), capped by OMP_NUM_THREADS when set."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(workload, seconds=15.0, max_steps=6):
    """The oracle (fp32 CPU restatement of the reference step, pinned to the reference's
    fixtures) on this host's cores: zero_grad -> fwd -> bwd -> clip -> AdamW, repeated for
    ~`seconds` of CPU work.  Sample: LM = BASELINE configs[0] itself (B=4 x T=1024);
    captions = the bench's own B=128 step (z (128,257,768) pooled, 31 text
    tokens), timed from its first step (one B=128 oracle step is ~4-5 s of CPU work)."""
    from oracle import models as OM
    from oracle import ops as O
    O.FAST_PATHS = True  # the torch ops the reference itself calls (oracle/ops.py)
    threads = host_threads()
    torch.set_num_threads(threads)
    import gvl.gpt2 as g2
    with torch.device("meta"):
        if workload == "lm":
            mdl = g2.GPT(g2.GPTConfig(vocab_size=50304))
        else:
            mdl = build_caption_meta(workload)
    keys = [(k, tuple(v.shape)) for k, v in mdl.state_dict().items() if not k.endswith("attn.bias")]
    g = torch.Generator().manual_seed(0)
    P = {k: torch.randn(s, generator=g) * 0.02 for k, s in keys}
    if workload == "lm":
        B = 4
        P["transformer.wte.weight"] = P["lm_head.weight"]
        ids = torch.randint(0, 50257, (B * 1024 + 1,), generator=g)
        x, y = ids[:-1].view(B, 1024), ids[1:].view(B, 1024)
        kind, units_per_step, unit = "gpt", B * 1024, "tokens/s"
        train = OM.trainable_keys("gpt", list(P))
        loss_of = lambda P_, it: OM.gpt_forward(P_, x, 12, 12, y)[1]
        sample = f"GPT-2 124M LM step, B={B} x T=1024 (configs[0]; fp32 oracle restatement)"
    else:
        from gvl.train import caption_batch, caption_labels
        from oracle import ops as O
        B = 128
        z, xx, yy, mm = caption_batch(B, device="cpu")
        zp = O.pool_clip(z)
        lab = caption_labels(yy, mm)
        kind = {"qformer": "qformer", "linear": "linear"}.get(workload, "cross")
        units_per_step, unit = B, "images/s"
        train = OM.trainable_keys(kind, list(P))
        if kind == "cross":
            P["transformer.wte.weight"] = P["lm_head.weight"]
            loss_of = lambda P_, it: OM.cross_att_forward(P_, xx, zp, 12, 12, yy, mm)[1]
        else:
            P["gpt.transformer.wte.weight"] = P["gpt.lm_head.weight"]
            loss_of = lambda P_, it: OM.caption_forward(P_, kind, zp, xx, 12, 12, 1024, lab)[1]
        sample = f"{workload} caption step, B={B} images (fp32 oracle restatement)"
    if workload == "lm":
        OM.train_steps(P, kind, train, loss_of, 1, lambda it: 1e-4)  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        OM.train_steps(P, kind, train, loss_of, 1, lambda it: 1e-4)
        n += 1
        if time.perf_counter() - t0 > seconds or n >= max_steps:
            break
    dt = time.perf_counter() - t0
    return dict(value=round(units_per_step * n / dt, 2), unit=unit, cores=threads, kind="port",
                cpu=cpu_model(), sample=f"{sample}; {n} steps in {dt:.1f}s")


def build_caption_meta(kind):
    import gvl.caption as cap
    import gvl.cross_att as xa
    import gvl.gpt2 as g2
    if kind == "cross":
        return xa.GPT(xa.GPTConfig(vocab_size=50304))
    lm = cap.GPT_previous(g2.GPTConfig(vocab_size=50304, block_size=1024))
    cls = cap.QFormerCaption if kind == "qformer" else cap.LinearCaption
    return cls(enc_dim=768, lm=lm, m_vis_tokens=32)


# ----------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="lm", choices=["lm", "qformer", "linear", "cross"])
    ap.add_argument("--micro-batch", type=int, default=16)
    ap.add_argument("--caption-batch", type=int, default=128)
    ap.add_argument("--bucket-mb", type=float, default=None,
                    help="gradient bucket size (default: 32 MB for the LM, 8 MB for the captions)")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--caption-steps", type=int, default=10)
    ap.add_argument("--captions", default="qformer,linear,cross",
                    help="secondary caption-step lines of the default (lm) run")
    ap.add_argument("--no-pixels", dest="pixels", action="store_false",
                    help="skip the pixel-input (CLIP ViT-L/14) linear caption line")
    ap.add_argument("--cpu-seconds", type=float, default=20.0,
                    help="CPU work per cpu_baseline sample (LM; captions get half)")
    ap.add_argument("--no-kernel-pass", action="store_true",
                    help="skip the eager per-GEMM timing pass (profiling runs)")
    ap.add_argument("--gemm-table", action="store_true",
                    help="list every GEMM instance of the step in roofline.all_gemms")
    ap.add_argument("--no-graph", action="store_true",
                    help="eager steps (default: the step is captured into hipGraphs; at N>1 two "
                         "graphs around the RCCL gradient all-reduce)")
    args = ap.parse_args()

    world, rank, dev = setup()
    from gvl import _lib
    from gvl import kernels as K
    _lib.load()

    if args.workload == "lm":
        step, units, cfg = run_lm(args, world, rank, dev)
        unit, flop_per_unit = "tokens/s", LM_FLOP_PER_TOKEN
    else:
        step, units, cfg = run_caption(args.workload, args, world, rank, dev)
        unit, flop_per_unit = "images/s", CAP_FLOP_PER_IMAGE[args.workload]
    use_graph = not args.no_graph
    timer = None if args.no_kernel_pass else K.KernelTimer()
    dt, res = timed(step, args.steps, args.warmup, world, timer, graph=use_graph)
    value = units * args.steps / dt
    roof = dominant_kernel(timer.summary(), args.workload, steps=1, full=args.gemm_table) if timer else None
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": unit, "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 2), "higher_is_better": True,
        "scaling": "strong" if args.workload == "lm" else "weak", "vs_baseline": None,
        "dtype": "bf16", "data": "synthetic (random tokens / N(0,1) CLIP tokens), random-init weights",
        "config": dict(cfg, model="gpt2-124m", parallelism=f"dp{world}"),
        "step_mfma_frac": round(value * flop_per_unit / 1e12 / PEAK_BF16_TFLOPS / world, 4),
        "loss": round(res[0], 5), "grad_norm": round(res[1], 5),
        "hip_graph": use_graph,
        "peak_hbm_gib": round(torch.cuda.max_memory_allocated(dev) / 2**30, 2),
        "roofline": roof,
    }
    if args.workload == "lm" and not args.no_secondary:
        del step
        torch.cuda.empty_cache()
        for kind in args.captions.split(","):
            if not kind:
                continue
            torch.cuda.reset_peak_memory_stats(dev)
            cstep, cunits, ccfg = run_caption(kind, args, world, rank, dev)
            ctimer = None if args.no_kernel_pass else K.KernelTimer()
            cdt, cres = timed(cstep, args.caption_steps, 3, world, ctimer, graph=use_graph,
                              kernel_steps=3)
            cval = cunits * args.caption_steps / cdt
            line = dict(
                value=round(cval, 1), unit="images/s",
                ms_per_step=round(cdt / args.caption_steps * 1e3, 3),
                step_mfma_frac=round(cval * CAP_FLOP_PER_IMAGE[kind] / 1e12 / PEAK_BF16_TFLOPS
                                     / world, 4),
                loss=round(cres[0], 5), config=ccfg,
                peak_hbm_gib=round(torch.cuda.max_memory_allocated(dev) / 2**30, 2),
                roofline=dominant_kernel(ctimer.summary(), kind, steps=3, full=args.gemm_table)
                if ctimer else None)
            if rank == 0 and world == 1 and not args.no_cpu_baseline:
                line["cpu_baseline"] = cpu_baseline(kind, seconds=args.cpu_seconds / 2)
            out[f"caption_{kind}"] = line
            del cstep
            torch.cuda.empty_cache()
    if args.workload == "lm" and not args.no_secondary and args.pixels and world == 1:
        out["caption_linear_pixels"] = run_pixels(args, world, rank, dev, args.caption_steps, 3)
        torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.workload, seconds=args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        # the library's teardown: every captured step is closed (bucket work joined, device
        # drained, graphs reset) before the communicator goes
        from gvl.dist import close_graphed_steps, destroy_process_group
        close_graphed_steps()
        dist.barrier()
        destroy_process_group()


if __name__ == "__main__":
    main()
