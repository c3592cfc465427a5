"""Known-byte kernels for calibrating rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 (run under
one `--pmc FETCH_SIZE` pass and one `--pmc WRITE_SIZE` pass; tools/pmc_calib.sh).

Each case streams buffers far larger than L2 + Infinity Cache (256 MiB), each byte once:
  ce     gvl_cross_entropy over a [rows, V] bf16 logit matrix: reads 2*rows*V B (16-B row
         loads into registers), writes 2*rows*V B of dlogits (16-B stores);
  gemm   gvl_gemm with one 256-wide column tile (N = 256): A [M, K] bf16 moves once by
         buffer_load ... lds (2*M*K B), B [256, K] stays in L2, C writes 2*M*N B;
  copy   torch copy_ of a bf16 tensor (ATen elementwise kernel): 2*n B read, 2*n B written.
Prints the expected bytes per launch; tools/pmc_calib_report.py pairs them with the counters."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "gpt2-vision-language_amd"))
from gvl import _lib  # noqa: E402
from gvl import kernels as K  # noqa: E402

BF = torch.bfloat16


def main():
    _lib.load()
    dev = torch.device("cuda")
    g = torch.Generator(device="cuda").manual_seed(0)
    rows, V = 8192, 50304  # 824 MB of logits
    lg = torch.randn(rows, V, device=dev, generator=g).to(BF)
    tg = torch.randint(0, V, (rows,), device=dev, generator=g)
    M, N, Kd = 262144, 256, 1024  # A = 512 MiB
    A = torch.randn(M, Kd, device=dev, generator=g).to(BF)
    B = torch.randn(N, Kd, device=dev, generator=g).to(BF)
    C = torch.empty(M, N, dtype=BF, device=dev)
    x = torch.randn(256 * 2**20, device=dev, generator=g).to(BF)  # 512 MiB
    y = torch.empty_like(x)
    for _ in range(3):
        K.cross_entropy(lg, tg)
        K.gemm(A, B, out=C)
        y.copy_(x)
    torch.cuda.synchronize()
    expect = {
        "ce_row_kernel": dict(read=2 * rows * V, write=2 * rows * V),
        "gemm": dict(read=2 * M * Kd + 2 * N * Kd, write=2 * M * N),
        "copy": dict(read=2 * x.numel(), write=2 * x.numel()),
    }
    print("EXPECT " + json.dumps(expect), flush=True)


if __name__ == "__main__":
    main()
