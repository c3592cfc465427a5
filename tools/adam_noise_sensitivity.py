"""How much the reference's own training trajectory moves when its gradients carry bf16-level
noise (justifies the post-update loss bound of tests/test_gpu_parity_full.py).

Runs the REFERENCE GPT-2 124M (AST-extracted from source/gpt2/train_gpt2.py, build container
only) through the mixed-precision loop of tools/make_fixtures.py (bf16 compute weights, fp32
masters, 2 micro-steps of B=1x1024, 2 AdamW steps at lr 6e-4) and reports the loss after the
2 updates with additive Gaussian noise of sigma x rms(grad) per tensor added to every
gradient.  Measured (2 seeds each): sigma 0.3% -> +1.5e-4 / +2.1e-4 relative, 1% -> +1.7e-3 /
+1.8e-3, 2% -> +4.6e-3 / +4.9e-3 — always an increase: Adam's per-element normalisation turns
noise on small-gradient weights into full-size +-lr moves in random directions.
"""
import sys, torch, numpy as np, contextlib, io
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]
import make_fixtures as MF
torch.set_num_threads(8)
g2 = MF.load_gpt2_classes()
mbs = [MF.inputs_lm(1, 1024, 50257, s) for s in (404, 405)]
def run(perturb, seed=0):
    torch.manual_seed(seed)
    model = MF.round_bf16_(MF.set_recipe(g2["GPT"](g2["GPTConfig"](vocab_size=50304))))
    opt = model.configure_optimizers(weight_decay=0.1, learning_rate=6e-4, device="cpu")
    for step in range(2):
        opt.zero_grad()
        with MF._Bf16Weights(model, True):
            for x, y in mbs:
                (model(x, y)[1] / 2).backward()
        with torch.no_grad():
            for p in model.parameters():
                if p.grad is not None:
                    p.grad.copy_(perturb(p.grad))
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
    with torch.no_grad(), MF._Bf16Weights(model, True):
        return float(model(*mbs[0])[1])
with contextlib.redirect_stdout(io.StringIO()):
    base = run(lambda g: g)
    res = {}
    for s in (0.003, 0.01, 0.02):
        res[s] = [run(lambda g: g + s * g.pow(2).mean().sqrt() * torch.randn_like(g), seed=k) for k in range(2)]
print("base", base)
for s, v in res.items():
    print(f"additive {s}: ", [(x, (x - base) / base) for x in v])
