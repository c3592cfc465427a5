"""ctypes binding of libgvl.so — the C-ABI declared in include/gvl.h.

This is the reference-side "FFI stub" for the hot path: the reference is Python, so the
binding is ctypes.  Loading fails loudly (ImportError at first use) when the library was
not built; there is no CPU or eager-PyTorch fallback behind it.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GVL_LIB", os.path.join(_HERE, "libgvl.so"))
ABI_VERSION = 14  # include/gvl.h GVL_ABI_VERSION

c_i64 = C.c_int64
c_i32 = C.c_int32
c_f32 = C.c_float
c_u64 = C.c_uint64
c_vp = C.c_void_p


class GemmDesc(C.Structure):
    _fields_ = [
        ("a", c_vp), ("b", c_vp), ("c", c_vp),
        ("m", c_i64), ("n", c_i64), ("k", c_i64),
        ("lda", c_i64), ("ldb", c_i64), ("ldc", c_i64),
        ("a_mn", c_i32), ("b_mn", c_i32),
        ("alpha", c_f32), ("alpha_ptr", c_vp),
        ("bias", c_vp),
        ("act", c_i32), ("dact", c_i32),
        ("pre_out", c_vp), ("pre_in", c_vp), ("ldp", c_i64),
        ("residual", c_vp), ("ldr", c_i64),
        ("gate", c_vp),
        ("drop_p", c_f32), ("seed", c_u64),
        ("c_fp32", c_i32),
        ("workspace", c_vp), ("workspace_bytes", c_i64),
        ("seed_ptr", c_vp),
        ("tickets", c_vp), ("ticket_count", c_i64),
    ]


class AttnDesc(C.Structure):
    _fields_ = [
        ("q", c_vp), ("k", c_vp), ("v", c_vp), ("o", c_vp), ("lse", c_vp),
        ("B", c_i64), ("H", c_i64), ("Tq", c_i64), ("Tk", c_i64),
        ("q_sb", c_i64), ("q_st", c_i64), ("q_sh", c_i64),
        ("k_sb", c_i64), ("k_st", c_i64), ("k_sh", c_i64),
        ("v_sb", c_i64), ("v_st", c_i64), ("v_sh", c_i64),
        ("o_sb", c_i64), ("o_st", c_i64), ("o_sh", c_i64),
        ("causal", c_i32), ("scale", c_f32), ("drop_p", c_f32), ("seed", c_u64),
        ("seed_ptr", c_vp),
    ]


class AttnBwdDesc(C.Structure):
    _fields_ = [
        ("dout", c_vp), ("do_sb", c_i64), ("do_st", c_i64), ("do_sh", c_i64),
        ("dq", c_vp), ("dq_sb", c_i64), ("dq_st", c_i64), ("dq_sh", c_i64),
        ("dk", c_vp), ("dk_sb", c_i64), ("dk_st", c_i64), ("dk_sh", c_i64),
        ("dv", c_vp), ("dv_sb", c_i64), ("dv_st", c_i64), ("dv_sh", c_i64),
        ("workspace", c_vp),
    ]


# name -> (restype, argtypes); every symbol include/gvl.h declares.
SIGNATURES = {
    "gvl_last_error": (C.c_char_p, []),
    "gvl_abi_version": (C.c_int, []),
    "gvl_set_launch_events": (C.c_int, [c_vp, c_vp]),
    "gvl_gemm": (C.c_int, [C.POINTER(GemmDesc), c_vp]),
    "gvl_gemm_batched": (C.c_int, [C.POINTER(GemmDesc), c_i32, c_vp]),
    "gvl_gemm_batched_dbias": (C.c_int, [C.POINTER(GemmDesc), C.POINTER(c_vp), c_i32, c_vp]),
    "gvl_gemm_grouped": (C.c_int, [C.POINTER(GemmDesc), C.POINTER(c_vp), c_i32, c_vp]),
    "gvl_gemm_tune": (C.c_int, [c_i32, c_i32]),
    "gvl_gemm_kernel_name": (C.c_int, [C.POINTER(GemmDesc), C.c_char_p, c_i32]),
    "gvl_gemm_batched_kernel_name": (C.c_int, [C.c_char_p, c_i32]),
    "gvl_layernorm_fwd": (C.c_int, [c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp,
                                    c_i64, c_i64, c_f32, c_vp]),
    "gvl_layernorm_bwd_workspace_size": (c_i64, [c_i64, c_i64]),
    "gvl_layernorm_bwd_blocks": (c_i32, [c_i64]),
    "gvl_layernorm_bwd_finalize_batched": (C.c_int, [C.POINTER(c_vp), C.POINTER(c_i32), c_i32, c_i64,
                                                     C.POINTER(c_vp), C.POINTER(c_vp), c_i32, c_vp]),
    "gvl_layernorm_bwd": (C.c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64,
                                    c_i32, c_vp, c_vp, c_i32, c_vp, c_i64, c_i64, c_vp]),
    "gvl_layernorm_bwd_res": (C.c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64,
                                        c_vp, c_i64, c_vp, c_vp, c_i32, c_vp, c_i64, c_i64, c_vp]),
    "gvl_attn_fwd": (C.c_int, [C.POINTER(AttnDesc), c_vp]),
    "gvl_attn_bwd_workspace_size": (c_i64, [C.POINTER(AttnDesc)]),
    "gvl_attn_bwd": (C.c_int, [C.POINTER(AttnDesc), C.POINTER(AttnBwdDesc), c_vp]),
    "gvl_cross_entropy": (C.c_int, [c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp,
                                    c_i32, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "gvl_embedding_fwd": (C.c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64,
                                    c_i64, c_vp]),
    "gvl_embedding_bwd": (C.c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64,
                                    c_i64, c_vp]),
    "gvl_copy_rows": (C.c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_i64, c_i64,
                                c_i64, c_i64, c_i32, c_vp]),
    "gvl_embedding_bwd_workspace": (c_i64, [c_i64]),
    "gvl_embedding_bwd_det": (C.c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64,
                                        c_i64, c_i64, c_vp, c_i64, c_vp]),
    "gvl_pool_clip": (C.c_int, [c_vp, c_i32, c_vp, c_i32, c_i64, c_i64, c_i64, c_vp]),
    "gvl_pool_clip_ex": (C.c_int, [c_vp, c_i32, c_vp, c_i32, c_i64, c_i64, c_i64, c_i32, c_vp]),
    "gvl_l2_normalize_rows": (C.c_int, [c_vp, c_vp, c_i32, c_i64, c_i64, c_vp]),
    "gvl_grad_norm_workspace_size": (c_i64, [c_i64]),
    "gvl_grad_norm": (C.c_int, [c_vp, c_i64, c_f32, c_vp, c_vp, c_vp]),
    "gvl_adamw": (C.c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_f32, c_f32, c_f32, c_f32,
                            c_f32, c_i64, c_vp, c_vp]),
    "gvl_adamw_dev": (C.c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_f32, c_f32, c_f32,
                                c_f32, c_vp, c_vp]),
    "gvl_adamw_master_dev": (C.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_f32,
                                       c_f32, c_f32, c_f32, c_vp, c_vp]),
    "gvl_attn_decode": (C.c_int, [c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64,
                                  c_i64, c_i64, c_i64, c_f32, c_vp]),
    "gvl_sample": (C.c_int, [c_vp, c_i64, c_i32, c_i64, c_i64, c_f32, c_i32, c_f32, c_vp, c_vp,
                             c_vp]),
    "gvl_colsum_workspace_size": (c_i64, [c_i64, c_i64]),
    "gvl_colsum": (C.c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, c_i32, c_vp, c_vp]),
    "gvl_colsum_batched_workspace_size": (c_i64, [c_i32, c_i64, c_i64]),
    "gvl_colsum_batched": (C.c_int, [C.POINTER(c_vp), C.POINTER(c_vp), c_i32, c_i64, c_i64, c_i64,
                                     c_i32, c_vp, c_vp]),
    "gvl_dropout_mask_apply": (C.c_int, [c_vp, c_i64, c_vp, c_i64, c_i64, c_i64, c_f32, c_u64, c_vp,
                                         c_vp]),
    "gvl_gate_bwd": (C.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "gvl_gate_bwd_acc_bf16": (C.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "gvl_gate_bwd_workspace_size": (c_i64, [c_i64]),
    "gvl_f32_to_bf16": (C.c_int, [c_vp, c_vp, c_i64, c_i32, c_vp]),
}

_lib = None
_lock = threading.Lock()


class GvlError(RuntimeError):
    pass


def load(path: str | None = None):
    """Load libgvl.so and bind every symbol; raises ImportError if absent."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        # GVL_LIB: an alternative build of the same library (A/B of compile-time variants)
        p = path or os.environ.get("GVL_LIB") or LIB_PATH
        if not os.path.exists(p):
            raise ImportError(
                f"libgvl.so not found at {p}: build it with `python -c 'import __graft_entry__ as g; "
                f"g.build()'` (or `make -C gpt2-vision-language_amd/csrc`). The gvl hot path has no "
                f"fallback.")
        lib = C.CDLL(p)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)  # AttributeError -> missing export: fail loudly
            fn.restype = res
            fn.argtypes = args
        if lib.gvl_abi_version() != ABI_VERSION:
            raise ImportError(f"{p} has C-ABI v{lib.gvl_abi_version()}, the bindings expect "
                              f"v{ABI_VERSION}: rebuild it (make -C gpt2-vision-language_amd/csrc)")
        if path is None:
            _lib = lib
        return lib


def check(rc: int, what: str):
    if rc != 0:
        msg = _lib.gvl_last_error().decode() if _lib is not None else "?"
        raise GvlError(f"{what} failed (rc={rc}): {msg}")


def lib():
    return _lib if _lib is not None else load()
