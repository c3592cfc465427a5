"""The drop-in boundary: libgvl.so loads on a CPU-only host and exports exactly the
symbols include/gvl.h declares, and the ctypes binding covers all of them."""
import ctypes
import os
import re

from tests.conftest import ROOT

HDR = os.path.join(ROOT, "include", "gvl.h")
LIB = os.path.join(ROOT, "gpt2-vision-language_amd", "gvl", "libgvl.so")


def declared():
    txt = open(HDR).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w]+\s*\*?\s*(gvl_\w+)\s*\(", txt, re.M)))


def test_header_declares_api():
    names = declared()
    assert "gvl_gemm" in names and "gvl_attn_bwd" in names and len(names) >= 20


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "libgvl.so not built (run __graft_entry__.build())"
    lib = ctypes.CDLL(LIB)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing
    lib.gvl_abi_version.restype = ctypes.c_int
    assert lib.gvl_abi_version() == 14


def test_library_links_no_vendor_blas():
    """Since ABI v10 every GEMM runs on libgvl's own kernels: the library has no hipBLASLt /
    rocBLAS dependency (round 4's gvl_gemm_lib_route is gone)."""
    import subprocess
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-d", LIB], capture_output=True,
                         text=True, check=True).stdout
    needed = [ln for ln in out.splitlines() if "NEEDED" in ln]
    assert needed and not any("blas" in ln.lower() for ln in needed), needed


def test_binding_covers_header():
    from gvl import _lib
    assert sorted(_lib.SIGNATURES) == declared()
    lib = _lib.load()  # binds every symbol with its argtypes
    assert lib.gvl_abi_version() == 14


def test_rejects_bad_arguments_without_gpu():
    """Argument validation runs on the host before any launch (no device needed)."""
    from gvl import _lib
    lib = _lib.load()
    d = _lib.GemmDesc()
    d.a = d.b = d.c = 16
    d.m, d.n, d.k = 8, 8, 7  # K not a multiple of 8
    d.lda = d.ldb = d.ldc = 8
    rc = lib.gvl_gemm(ctypes.byref(d), None)
    assert rc == -1 and b"multiple of 8" in lib.gvl_last_error()
    rc = lib.gvl_layernorm_fwd(None, 4, None, None, None, 4, None, None, 1, 2048, 1e-5, None)
    assert rc == -1 and b"cols" in lib.gvl_last_error()
