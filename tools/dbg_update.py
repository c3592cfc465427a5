"""Debug: per-tensor gradient / first-update agreement of the full-size linear caption step
with the reference fixture, and the AdamW kernels vs torch.optim.AdamW (fp32, CPU)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpt2-vision-language_amd")]
import numpy as np, torch
from tests.test_gpu_parity_full import _build_full, _recipe, _loss_fn, _sampled
import json
cuda = torch.device("cuda:0")
import gvl._lib as L; L.load()

# 2) linear full-size step detail
meta = json.load(open(os.path.join(ROOT, "tests/golden/meta.json")))
fx = dict(np.load(os.path.join(ROOT, "tests/golden/full_train.npz")))
for kind in ("lm",):
    model, P = _recipe(_build_full(kind), cuda)
    model.eval()
    lr = 6e-4 if kind == "lm" else 1e-3
    opt = model.configure_optimizers(0.1, lr, "cuda")
    mbs, loss_fn = _loss_fn(kind, fx, cuda)
    from gvl.train import train_step
    r = train_step(model, opt, mbs, loss_fn, lr)
    gsave = {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}
    r2 = train_step(model, opt, mbs, loss_fn, lr)
    print(kind, "losses", r.loss.item(), r2.loss.item(), "ref mp", fx["mp_" + kind + "_losses"])
    pre = "mp_" + kind + "_"
    params = dict(model.named_parameters())
    rows = []
    for n in meta[f"full_{kind}_trainable"]:
        p = params[n]
        got, ref, idx = _sampled(fx, pre + "grad:" + n, gsave[n])
        p0 = P[n].reshape(-1).double().numpy(); p0b = P[n].to(torch.bfloat16).reshape(-1).double().numpy()
        if idx is not None: p0, p0b = p0[idx], p0b[idx]
        m1, r1, _ = _sampled(fx, pre + "step2:" + n, opt.master_of(p))
        du, dr = m1 - p0b, r1 - p0b
        clear = np.abs(ref) > 0.02 * np.abs(ref).max()
        ge = np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-30)
        ue = np.linalg.norm(du[clear] - dr[clear]) / max(np.linalg.norm(dr[clear]), 1e-30) if clear.any() else 0
        sg = float((np.sign(du[clear]) == np.sign(dr[clear])).mean()) if clear.any() else 1
        g2 = p.grad.double().reshape(-1).cpu().numpy()
        if idx is not None: g2 = g2[idx]
        scale = p.numel() / len(g2)
        contrib = float((g2 * (du - dr)).sum() * scale)
        allerr = np.linalg.norm(du - dr) / max(np.linalg.norm(dr), 1e-30)
        rows.append((abs(contrib), n, contrib, ue, allerr, float(np.abs(dr).mean()), float(np.abs(du).mean())))
    rows.sort(reverse=True)
    print("sum of first-order contributions", sum(r[2] for r in rows))
    for _, n, c, ue, ae, a, b in rows[:15]:
        print(f"{kind} {n}: dLoss~{c:+.3e} clear relL2 {ue:.2e} all relL2 {ae:.2e} |d_ref| {a:.2e} |d_got| {b:.2e}")
    del model, opt
