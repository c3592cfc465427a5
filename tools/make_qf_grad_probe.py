"""Gradient probes inside the Q-Former caption step at the bench shape (round 5, the verdict's
"Q-Former bench-shape grad-norm 9.3e-4 off" item): the REFERENCE model (gpt2_q_former/model.py,
loaded read-only by tools/make_fixtures.py's loaders; runs only in the build container) on the
bf16-valued recipe weights in fp32 math, the same inputs as the bench_shapes fixture, with the
gradient captured at

  * bridge.layers[0] output  (q after the first Q-Former layer, [B, 32, 768])
  * bridge output            (q after the second layer = the decoder's 32 prefix rows)
  * the decoder input         (input of transformer.h[0]: the 32 prefix rows + 31 text rows)

Each is stored as 65,536 sampled elements (fixed indices) plus its full sum of squares, in
tests/golden/qf_grad_probe.npz.  tests/test_gpu_parity_bench.py::test_qformer_grad_probe
compares gvl's gradients at the same points (signed scale error and relative L2), which splits
a systematic gradient scale error between the decoder backward and the bridge backward.
Usage: python tools/make_qf_grad_probe.py
"""
import os
import sys
import zlib

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import make_fixtures as MF  # noqa: E402

N = 65536


def sample(name, t, out):
    a = t.detach().to(torch.float64).reshape(-1).numpy()
    idx = np.random.default_rng(zlib.crc32(name.encode())).choice(a.size, size=min(N, a.size), replace=False)
    idx.sort()
    out[name + "#idx"] = idx.astype(np.int64)
    out[name + "#val"] = a[idx].astype(np.float32)
    out[name + "#sq"] = np.array(float((a * a).sum()))


def main():
    torch.set_grad_enabled(True)
    qf = MF.load_module("gpt2_q_former", "ref_qf_model")
    lm = qf.GPT_previous(qf.GPTConfig(vocab_size=50304, block_size=1024))
    model = MF.set_recipe(qf.GPT_Caption(enc_dim=768, lm=lm, m_vis_tokens=32))
    model.eval()
    MF.round_bf16_(model)
    z_raw, x, yy, mask = MF.inputs_caption(MF.BENCH_CAP_B, 257, 768, 31, 50257, 1313)
    labels = yy.masked_fill(~mask, -100)
    z = qf.pool_clip_197_to_33_avg_with_cls(z_raw)
    caught = {}

    def keep(name):
        def hook(mod, inp, out):
            out.retain_grad()
            caught[name] = out
        return hook

    model.bridge.layers[0].register_forward_hook(keep("layer0_out"))
    model.bridge.register_forward_hook(keep("bridge_out"))

    def keep_in(mod, args):
        args[0].retain_grad()
        caught["dec_in"] = args[0]

    model.gpt.transformer.h[0].register_forward_pre_hook(keep_in)
    _, loss = model(z, x, labels=labels)
    loss.backward()
    out = {"loss": np.array(float(loss))}
    for name, t in caught.items():
        sample(name, t.grad, out)
        print(name, tuple(t.shape), float(t.grad.double().norm()), flush=True)
    np.savez_compressed(os.path.join(MF.OUT, "qf_grad_probe.npz"), **out)
    print("loss", float(loss))


if __name__ == "__main__":
    main()
