"""Loader for the in-tree gfx950 kernel library ``_native/libedge_kernels.so``.

The library is plain HIP C ABI (no torch headers), built by ``build.py`` with
``hipcc --offload-arch=gfx950``.  Kernels are launched on the current torch
stream, so they compose with torch ops, CUDA-graph capture and RCCL streams.

On a GPU process the library is mandatory: ``lib()`` raises instead of silently
falling back to the PyTorch reference path.
"""
from __future__ import annotations

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# EDGE_KERNEL_LIB: load another build of the library (A/B of two kernel builds in one GPU session)
LIB_PATH = os.environ.get("EDGE_KERNEL_LIB") or os.path.join(os.path.dirname(_HERE), "_native", "libedge_kernels.so")

_lib = None

c_p = ctypes.c_void_p
c_i = ctypes.c_int
c_f = ctypes.c_float
c_ll = ctypes.c_longlong

_SIGS = {
    "edge_rmsnorm": [c_p, c_p, c_p, c_p, c_i, c_i, c_f, c_p],
    "edge_layernorm": [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_f, c_p],
    "edge_embedding": [c_p, c_p, c_p, c_i, c_i, c_i, c_p],
    "edge_gemm": [c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_p, c_p, c_i, c_i, c_p, c_p, c_p],
    "edge_row_ssq": [c_p, c_p, c_i, c_i, c_p],
    "edge_row_rscale": [c_p, c_p, c_i, c_i, c_i, c_f, c_p],
    "edge_gemm_set_tile": [c_i],
    "edge_gemm_set_variant": [c_i],
    "edge_gemm_set_walk": [c_i],
    "edge_gemm_set_w7": [c_i],
    "edge_gemm_set_qkv256": [c_i],
    "edge_gemm_set_qkv192": [c_i],
    "edge_gemm_set_qkv192_bf16": [c_i],
    "edge_gemm_set_skip_epi": [c_i],
    "edge_gemm_set_rs_lds": [c_i],
    "edge_gemm_set_lse256": [c_i],
    "edge_gemm_set_w7_mode": [c_i],
    "edge_gemm_set_stagger": [c_i],
    "edge_gemm_set_split": [c_i],
    "edge_gemm_get_split": [],
    "edge_gemm_set_ws": [c_p, c_ll, c_p],
    "edge_gemm_ws_floats": [],
    "edge_gemm_checked_build": [],
    "edge_gemm_ssq_parts": [c_i, c_i, c_i, c_i, c_i, c_i],
    "edge_gemm_qkv_rope": [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_f, c_p, c_p,
                           c_i, c_f, c_p],
    "edge_gemm_lse": [c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_f, c_p],
    "edge_lse_reduce": [c_p, c_p, c_p, c_p, c_i, c_i, c_p],
    "edge_flash_attn_fwd": [c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_i, c_p],
    "edge_attn_set_variant": [c_i],
    "edge_attn_f32_set_variant": [c_i],
    "edge_attn_lastrow": [c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_p],
    "edge_attn_colsum": [c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_p],
    "edge_head_combine": [c_p, c_p, c_p, c_i, c_i, c_i, c_f, c_f, c_p],
    "edge_select": [c_p, c_i, c_i, c_i, c_p, c_ll, c_i, c_f, c_ll, c_p],
    "edge_set_mask": [c_p, c_ll, c_i, c_i, c_i, c_p],
    "edge_channel_stats": [c_p, c_p, c_ll, c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_p],
    "edge_rowmax": [c_p, c_p, c_i, c_i, c_p],
    "edge_pack": [c_p, c_p, c_ll, c_ll, c_ll, c_ll, c_ll, c_ll, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i,
                  c_i, c_p],
    "edge_lrp_attn_bwd": [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_p],
    "edge_lrp_rope_pack": [c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_i, c_f, c_p],
    "edge_swiglu_il": [c_p, c_p, c_ll, c_i, c_p],
    "edge_lrp_swiglu_bwd": [c_p, c_p, c_p, c_ll, c_i, c_p],
    "edge_lrp_gelu_bwd": [c_p, c_p, c_ll, c_p],
    "edge_lrp_ln_bwd": [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_p],
    "edge_ln_rstd": [c_p, c_p, c_i, c_i, c_f, c_p],
    "edge_unpack": [c_p, c_p, c_ll, c_ll, c_ll, c_ll, c_ll, c_ll, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i,
                    c_i, c_i, c_p],
    # fp32 execution mode (h3 split-fp16 GEMM operands, fp32 attention / norms / codec)
    "edge_rmsnorm_f32_rstd": [c_p, c_p, c_p, c_p, c_i, c_i, c_f, c_f, c_p, c_p],
    "edge_gemm_swiglu_raw": [c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_p, c_p],
    "edge_gemm_f32_swiglu_raw": [c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_p, c_f, c_f, c_p],
    "edge_gemm_f32_cs": [c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_p, c_p, c_i, c_p, c_f, c_p],
    "edge_gemm_f32": [c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_p, c_p, c_i, c_i, c_p, c_f, c_f, c_p],
    "edge_gemm_qkv_rope_f32": [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_f,
                               c_f, c_p, c_p, c_f, c_f, c_p],
    "edge_flash_attn_fwd_h3p": [c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_i, c_f, c_f, c_f, c_f, c_p],
    "edge_flash_attn_fwd_f32": [c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_i, c_f, c_f, c_f, c_f, c_p],
    "edge_attn_lastrow_f32": [c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_f, c_f, c_p],
    "edge_attn_colsum_f32": [c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_f, c_f, c_p],
    "edge_rmsnorm_f32": [c_p, c_p, c_p, c_p, c_i, c_i, c_f, c_f, c_p],
    "edge_layernorm_f32": [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_f, c_f, c_f, c_p],
    "edge_split_h3": [c_p, c_p, c_p, c_i, c_i, c_f, c_p],
    "edge_embedding_f32": [c_p, c_p, c_p, c_i, c_i, c_i, c_p],
    # fp32 AttnLRP backward (csrc/lrp_f32.hip)
    "edge_lrp_attn_set_x6": [c_i],
    "edge_lrp_attn_bwd_f32": [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_p],
    "edge_lrp_rope_pack_h3": [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_i, c_f, c_p],
    "edge_lrp_attn_bwd_f32_gs": [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_p],
    "edge_lrp_attn_gqa_sum_ok": [],
    "edge_lrp_rope_pack_h3_gs": [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_i, c_f, c_p],
    "edge_split_h3_dyn": [c_p, c_p, c_p, c_p, c_i, c_i, c_p],
    "edge_lrp_swiglu_bwd_h3": [c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_p],
    "edge_lrp_gelu_bwd_h3": [c_p, c_p, c_p, c_p, c_i, c_i, c_p],
    "edge_act_h3": [c_p, c_p, c_ll, c_i, c_i, c_f, c_p],
    "edge_row_rstd_f32": [c_p, c_p, c_i, c_i, c_f, c_i, c_p],
    "edge_lrp_ln_bwd_f32": [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_p],
    "edge_group_absprod": [c_p, c_p, c_p, c_i, c_i, c_i, c_i, c_p],
}


_LL_RESULT = {"edge_gemm_ws_floats"}


class NativeLibraryMissing(RuntimeError):
    pass


def tuning() -> bool:
    """Kernel A/B switches (EDGE_GEMM_VARIANT, EDGE_ATTN_VARIANT, ...) are honoured only with EDGE_TUNING=1, so a
    stray environment variable can never change the production kernel selection."""
    return os.environ.get("EDGE_TUNING", "0") not in ("", "0")


def _apply_tuning_env(L) -> None:
    v = os.environ.get("EDGE_GEMM_VARIANT")  # A/B of the 256x256 main loop (see ops.set_gemm_variant)
    if v:
        L.edge_gemm_set_variant(int(v))
    av = os.environ.get("EDGE_ATTN_VARIANT")  # A/B of the flash-attention forward (see ops.set_attn_variant)
    if av:
        L.edge_attn_set_variant(int(av))
    if os.environ.get("EDGE_GEMM_LSE256", "1") == "0":  # LM-head LSE GEMM on 128x128 tiles
        L.edge_gemm_set_lse256(0)
    if os.environ.get("EDGE_GEMM_RS_LDS", "1") == "0":  # row scales by global loads in the epilogue
        L.edge_gemm_set_rs_lds(0)
    if os.environ.get("EDGE_GEMM_W7", "1") == "0":  # N = 896 GEMMs back on the 256x256 tiles
        L.edge_gemm_set_w7(0)
    st = os.environ.get("EDGE_GEMM_STAGGER")  # four-wave GEMMs: odd workgroups start st x 1024 cycles late
    if st and hasattr(L, "edge_gemm_set_stagger"):
        L.edge_gemm_set_stagger(int(st))
    lx = os.environ.get("EDGE_LRP_ATTN_X6")  # fp32 AttnLRP attention backward: 1 bf16-plane sweeps, 0 f32 MFMA
    if lx and hasattr(L, "edge_lrp_attn_set_x6"):
        L.edge_lrp_attn_set_x6(int(lx))
    qb = os.environ.get("EDGE_GEMM_QKV192_BF16")  # bf16 QKV on the four-wave 256x192 tiles (1) or 128x128 (0)
    if qb and hasattr(L, "edge_gemm_set_qkv192_bf16"):
        L.edge_gemm_set_qkv192_bf16(int(qb))
    sp = os.environ.get("EDGE_GEMM_SPLIT")  # four-wave GEMM epilogue desync: -1 auto, 0 off, k K-tiles
    if sp and hasattr(L, "edge_gemm_set_split"):
        L.edge_gemm_set_split(int(sp))


def available() -> bool:
    return os.path.exists(LIB_PATH)


def lib():
    """Return the loaded ctypes library, loading it on first use (raises if absent)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryMissing(
                f"{LIB_PATH} not found: build the gfx950 kernels first "
                "(python -c 'import __graft_entry__ as g; g.build()')")
        L = ctypes.CDLL(LIB_PATH)
        for name, argt in _SIGS.items():
            if os.environ.get("EDGE_KERNEL_LIB") and not hasattr(L, name):
                continue  # an older build under A/B: entry points it predates stay unbound
            fn = getattr(L, name)
            fn.argtypes = argt
            fn.restype = c_ll if name in _LL_RESULT else c_i
        _lib = L
        if tuning():
            _apply_tuning_env(L)
    return _lib


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def call(name: str, *args) -> None:
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed with HIP error {rc}")
