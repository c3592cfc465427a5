"""Yardstick for the bf16 gradient bounds of tests/test_gpu_parity_bench.py (runs only in the
build container, where /root/reference exists): the REFERENCE's own bf16 GPU-path arithmetic
(model.to(torch.bfloat16) + autocast bf16, train_gpt2.py:264,463 / gpt2_q_former/train.py:
116,308), executed here on the CPU, against its fp32 arithmetic on the same bf16-valued
weights and the same bench-shape inputs (tools/make_fixtures.py fixture_bench_shapes).  The
per-tensor gradient relative L2 errors go to tests/golden/bf16_yardstick.json.

    python tools/bf16_yardstick.py [lm,qformer,cross,linear]
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import make_fixtures as MF  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "bf16_yardstick.json")


def grads(model, run, bf16):
    model.zero_grad(set_to_none=True)
    if bf16:
        with torch.autocast(device_type="cpu", dtype=torch.bfloat16):
            loss = run(model)
    else:
        loss = run(model)
    loss.backward()
    return float(loss), {n: p.grad.detach().double().clone() for n, p in model.named_parameters()
                         if p.requires_grad and p.grad is not None}


def compare(kind, build, run):
    t0 = time.time()
    m32 = MF.round_bf16_(MF.set_recipe(build()))
    m32.eval()
    l32, g32 = grads(m32, run, False)
    mbf = MF.round_bf16_(MF.set_recipe(build())).to(torch.bfloat16)
    mbf.eval()
    lbf, gbf = grads(mbf, run, True)
    err = {n: float((gbf[n] - g32[n]).norm() / g32[n].norm().clamp_min(1e-30)) for n in g32}
    worst = max(err.items(), key=lambda kv: kv[1])
    # signed projection error per tensor and the global norm (round 5: a systematic gradient
    # scale error shows in these, not in the rel-L2 noise)
    scale = {n: float((gbf[n] * g32[n]).sum() / (g32[n] * g32[n]).sum().clamp_min(1e-300) - 1.0) for n in g32}
    n32 = float(torch.sqrt(sum((g * g).sum() for g in g32.values())))
    nbf = float(torch.sqrt(sum((g * g).sum() for g in gbf.values())))
    rec = dict(loss_fp32=l32, loss_bf16=lbf, loss_rel=abs(lbf - l32) / abs(l32),
               worst=worst, median=float(np.median(list(err.values()))), grad_rel_l2=err,
               grad_norm_fp32=n32, grad_norm_bf16=nbf, grad_norm_rel=(nbf - n32) / n32,
               scale_err=scale, scale_err_median=float(np.median(list(scale.values()))),
               seconds=round(time.time() - t0, 1))
    print(kind, f"grad norm rel {rec['grad_norm_rel']:+.2e}, scale err median "
          f"{rec['scale_err_median']:+.2e}", flush=True)
    print(kind, f"loss rel {rec['loss_rel']:.2e} worst {worst[1]:.3e} ({worst[0]}) median "
          f"{rec['median']:.3e} in {rec['seconds']}s", flush=True)
    return rec


def post_update_lm(g2):
    """Loss after 1 and 2 optimizer updates of the full-size LM (tests/test_gpu_parity_full.py's
    config: 2 micro-steps of B=1 x 1024, lr 6e-4, clip 1.0, AdamW(0.9, 0.95)): the reference's
    own bf16 GPU path (model.to(bf16) + autocast, bf16 AdamW state) vs its fp32 path."""
    mbs = [MF.inputs_lm(1, 1024, 50257, s) for s in (404, 405)]

    def run(bf16):
        m = MF.set_recipe(g2["GPT"](g2["GPTConfig"](vocab_size=50304)))
        if bf16:
            m = m.to(torch.bfloat16)
        opt = m.configure_optimizers(weight_decay=0.1, learning_rate=6e-4, device="cpu")
        losses = []
        for step in range(3):
            opt.zero_grad()
            la = 0.0
            for x, y in mbs:
                with torch.autocast(device_type="cpu", dtype=torch.bfloat16, enabled=bf16):
                    loss = m(x, y)[1] / len(mbs)
                la += float(loss.detach())
                if step < 2:
                    loss.backward()
            losses.append(la)
            if step < 2:
                torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)
                opt.step()
        return losses
    t0 = time.time()
    l32, lbf = run(False), run(True)
    rel = [abs(a - b) / abs(a) for a, b in zip(lbf, l32)]
    print("lm post-update: fp32", l32, "bf16", lbf, "rel", rel, f"{time.time() - t0:.0f}s", flush=True)
    return dict(losses_fp32=l32, losses_bf16=lbf, rel=rel)


def main():
    kinds = sys.argv[1].split(",") if len(sys.argv) > 1 else ["qformer", "lm"]
    torch.set_num_threads(os.cpu_count() or 8)
    g2 = MF.load_gpt2_classes()
    mods = {"linear": MF.load_module("gpt2_linear", "ref_lin"),
            "qformer": MF.load_module("gpt2_q_former", "ref_qf"),
            "cross": MF.load_module("gpt2_cross-att", "ref_xa")}
    out = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for kind in kinds:
        if kind == "lm_post":
            out[kind] = post_update_lm(g2)
            with open(OUT, "w") as f:
                json.dump(out, f, indent=1)
            continue
        if kind == "lm":
            x, y = MF.inputs_lm(MF.BENCH_LM_B, 1024, 50257, 4040)
            rec = compare(kind, lambda: g2["GPT"](g2["GPTConfig"](vocab_size=50304)),
                          lambda m: m(x, y)[1])
        elif kind == "cross":
            xa = mods["cross"]
            z_raw, x, yy, mask = MF.inputs_caption(MF.BENCH_CAP_B, 257, 768, 31, 50257, 1414)
            z = xa.pool_clip_197_to_33_avg_with_cls(z_raw)
            rec = compare(kind, lambda: xa.GPT(xa.GPTConfig(vocab_size=50304, block_size=1024)),
                          lambda m: m(x, z=z.to(next(m.parameters()).dtype), targets=yy,
                                      target_mask=mask)[1])
        else:
            mod = mods[kind]
            z_raw, x, yy, mask = MF.inputs_caption(MF.BENCH_CAP_B, 257, 768, 31, 50257, 1313)
            labels = yy.masked_fill(~mask, -100)
            z = mod.pool_clip_197_to_33_avg_with_cls(z_raw)

            def build(mod=mod):
                lm = mod.GPT_previous(mod.GPTConfig(vocab_size=50304, block_size=1024))
                return mod.GPT_Caption(enc_dim=768, lm=lm, m_vis_tokens=32)
            rec = compare(kind, build, lambda m: m(z.to(next(m.parameters()).dtype), x,
                                                   labels=labels)[1])
        out[kind] = rec
        with open(OUT, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
