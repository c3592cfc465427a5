"""ISA checks of the hand-scheduled kernels (CPU: hipcc cross-compiles gfx950 device assembly).

tools/isa_lds_hazards.py flags instructions that read a VGPR an in-flight LDS read is still
filling — the hazard behind round 3's intermittent wrong dQ (frag_tr_asm outputs without
early-clobber: the second transposed read took its address from the register the first read
was filling).
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_lds_hazards as H  # noqa: E402

HIPCC = "/opt/rocm/bin/hipcc"


def test_checker_flags_address_clobber_and_stale_read():
    asm = """_Zk:
\tds_read_b64_tr_b16 v[38:39], v38
\tds_read_b64_tr_b16 v[40:41], v39
\tv_mov_b64_e32 v[56:57], v[40:41]
\ts_waitcnt lgkmcnt(0)
\tv_mfma_f32_16x16x32_bf16 v[0:3], v[38:41], v[4:7], v[0:3]
"""
    hits = H.scan(asm.split("\n"))["_Zk"]
    assert [h[1] for h in hits] == ["address clobber", "stale read"]


def test_checker_models_counted_lgkmcnt():
    asm = """_Zk:
\tds_read_b128 v[10:13], v1
\tds_read_b128 v[14:17], v2
\ts_waitcnt lgkmcnt(1)
\tv_mfma_f32_16x16x32_bf16 v[0:3], v[10:13], v[4:7], v[0:3]
\tv_mfma_f32_16x16x32_bf16 v[0:3], v[14:17], v[4:7], v[0:3]
"""
    hits = H.scan(asm.split("\n"))
    assert len(hits["_Zk"]) == 1 and "v[14:17]" in hits["_Zk"][0][2]


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("unit", ["attention", "gemm_w4x"])
def test_asm_lds_kernels_have_no_pending_lds_reads(tmp_path, unit):
    """attention.hip and gemm_w4x.hip issue transposed LDS reads by inline asm (hipcc's own
    builtin drains the LDS-DMA queue in front of each one): none of their kernels may read a
    register such a read is still filling."""
    src = os.path.join(ROOT, "gpt2-vision-language_amd", "csrc", unit + ".hip")
    out = tmp_path / (unit + ".s")
    subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                    "-Wno-unused-function", "-mllvm", "-pragma-unroll-threshold=1000000", src, "-o",
                    str(out)], check=True, capture_output=True, timeout=600)
    hits = H.scan(out.read_text().split("\n"))
    assert not hits, {k[:60]: v[:2] for k, v in hits.items()}
