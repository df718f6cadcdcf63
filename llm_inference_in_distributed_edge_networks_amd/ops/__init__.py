"""Compute ops of the framework.

Every op has exactly two implementations with identical layouts and semantics:

* CUDA/HIP tensors -> the hand-written gfx950 kernel from ``csrc/`` (``_native``);
  a missing library is an error, never a silent fallback.  Two GPU precisions:
  bf16 activations (bf16 MFMA), and fp32 activations - the reference's precision - where
  GEMM operands travel in the h3 split-fp16 layout (``reference.h3_act`` / ``h3_weight``,
  csrc/common.h: two fp16 planes, three fp16 MFMA products per fp32 product, power-of-two
  operand scales) and attention runs on split-bf16 matrix-core products (csrc/attention_f32.hip);
* CPU tensors -> the fp32 PyTorch oracle in ``reference.py`` (used for the
  CPU WikiText-2 configuration and as the test oracle).
"""
from __future__ import annotations


import math

import torch

from . import reference as ref
from ._native import call, lib, ptr, stream

IL_BLOCK = ref.IL_BLOCK
s_pad = ref.s_pad
rope_tables = ref.rope_tables
interleave_gate_up = ref.interleave_gate_up
deinterleave_gate_up = ref.deinterleave_gate_up

_ACT = {None: 0, "gelu": 1, "swiglu_il": 2}




def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


def _check_f32(*ts):
    for t in ts:
        if t is not None and t.dtype != torch.float32:
            raise TypeError(f"fp32-mode HIP kernels take fp32 tensors, got {t.dtype}")
        if t is not None and not t.is_contiguous():
            raise ValueError("HIP kernels take contiguous tensors")


def _check_h3(a3, w3, alpha) -> int:
    """a3: 2-plane activation [rows, 2K] (reference.h3_act), w3: h3 weight [N, 3K] or the single plane [N, K]
    (reference.h3_weight).  Returns (plane width K, the GEMM's K' = 3K or 2K)."""
    for t, what in ((a3, "activations [rows, 2K] (reference.h3_act)"), (w3, "weights (reference.h3_weight)")):
        if t.dtype != torch.float16 or not t.is_contiguous():
            raise TypeError(f"h3 {what} must be contiguous fp16")
    terms = ref.h3_terms(a3, w3)
    if not alpha > 0.0:
        raise ValueError(f"h3 product scale alpha must be > 0, got {alpha}")
    return a3.shape[-1] // 2, terms * (a3.shape[-1] // 2)


def _check_bf16(*ts):
    for t in ts:
        if t is not None and t.dtype != torch.bfloat16:
            raise TypeError(f"HIP kernels take bf16 tensors, got {t.dtype}")
        if t is not None and not t.is_contiguous():
            raise ValueError("HIP kernels take contiguous tensors")


# --------------------------------------------------------------------------------------------
def embedding(ids: torch.Tensor, table: torch.Tensor) -> torch.Tensor:
    if not _gpu(table):
        return ref.embedding(ids, table)
    ids = ids.reshape(-1).to(torch.int64).contiguous()
    T, (V, H) = ids.numel(), table.shape
    out = torch.empty(T, H, dtype=table.dtype, device=table.device)
    if table.dtype == torch.float32:
        _check_f32(table)
        call("edge_embedding_f32", ptr(ids), ptr(table), ptr(out), T, H, V, stream())
        return out
    _check_bf16(table)
    call("edge_embedding", ptr(ids), ptr(table), ptr(out), T, H, V, stream())
    return out


def _out_f32_or_h3(R: int, H: int, h3: float, device) -> torch.Tensor:
    return torch.empty(R, 2 * H, dtype=torch.float16, device=device) if h3 else \
        torch.empty(R, H, dtype=torch.float32, device=device)


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, rows: torch.Tensor | None = None,
            h3: float = 0.0, rstd_out: torch.Tensor | None = None) -> torch.Tensor:
    """RMSNorm of ``x[rows]`` (all rows if ``rows`` is None).  fp32 ``x`` with ``h3`` = s > 0: output as the
    2-plane h3 activation of s * y (the next GEMM's input).  ``rstd_out`` (fp32 [R]): also the row normalisers
    rsqrt(mean(x^2) + eps) the norm applied (fp32 ``x``; what ``row_rstd`` computes, without a second pass)."""
    if not _gpu(x):
        xs = x if rows is None else x.index_select(0, rows.long())
        if rstd_out is not None:
            rstd_out.copy_(ref.row_rstd(xs, eps))
        y = ref.rmsnorm(xs, w, eps)
        return ref.h3_act(y, h3) if h3 else y
    R = x.shape[0] if rows is None else rows.numel()
    H = x.shape[1]
    rows32 = None if rows is None else rows.to(torch.int32).contiguous()
    if x.dtype == torch.float32:
        _check_f32(x, w, rstd_out)
        y = _out_f32_or_h3(R, H, h3, x.device)
        if rstd_out is not None:
            assert rstd_out.shape == (R,)
            call("edge_rmsnorm_f32_rstd", ptr(x), ptr(w), ptr(y), ptr(rows32), R, H, float(eps), float(h3),
                 ptr(rstd_out), stream())
            return y
        call("edge_rmsnorm_f32", ptr(x), ptr(w), ptr(y), ptr(rows32), R, H, float(eps), float(h3), stream())
        return y
    if rstd_out is not None:
        raise TypeError("rstd_out: fp32 activations only")
    _check_bf16(x, w)
    y = torch.empty(R, H, dtype=x.dtype, device=x.device)
    call("edge_rmsnorm", ptr(x), ptr(w), ptr(y), ptr(rows32), R, H, float(eps), stream())
    return y


def layernorm(x, w, b, eps, rows=None, h3: float = 0.0):
    if not _gpu(x):
        y = ref.layernorm(x if rows is None else x.index_select(0, rows.long()), w, b, eps)
        return ref.h3_act(y, h3) if h3 else y
    R = x.shape[0] if rows is None else rows.numel()
    H = x.shape[1]
    rows32 = None if rows is None else rows.to(torch.int32).contiguous()
    if x.dtype == torch.float32:
        _check_f32(x, w, b)
        y = _out_f32_or_h3(R, H, h3, x.device)
        call("edge_layernorm_f32", ptr(x), ptr(w), ptr(b), None, None, ptr(y), None, ptr(rows32), R, H, float(eps),
             float(h3), 0.0, stream())
        return y
    _check_bf16(x, w, b)
    y = torch.empty(R, H, dtype=x.dtype, device=x.device)
    call("edge_layernorm", ptr(x), ptr(w), ptr(b), None, None, ptr(y), None, ptr(rows32), R, H, float(eps), stream())
    return y


def layernorm_dual(x, w1, b1, w2, b2, eps, h3: tuple[float, float] = (0.0, 0.0)):
    """Two LayerNorms of the same input (GPT-NeoX parallel residual reads ln1(x) and ln2(x)).  fp32 ``x`` with
    ``h3`` = (s1, s2) > 0: both outputs as h3 activations at their scales."""
    s1, s2 = h3
    if not _gpu(x):
        y1, y2 = ref.layernorm_dual(x, w1, b1, w2, b2, eps)
        return (ref.h3_act(y1, s1), ref.h3_act(y2, s2)) if s1 else (y1, y2)
    if x.dtype == torch.float32:
        _check_f32(x, w1, b1, w2, b2)
        R, H = x.shape
        y1, y2 = _out_f32_or_h3(R, H, s1, x.device), _out_f32_or_h3(R, H, s2, x.device)
        call("edge_layernorm_f32", ptr(x), ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(y1), ptr(y2), None, R, H,
             float(eps), float(s1), float(s2), stream())
        return y1, y2
    _check_bf16(x, w1, b1, w2, b2)
    R, H = x.shape
    y1 = torch.empty_like(x)
    y2 = torch.empty_like(x)
    call("edge_layernorm", ptr(x), ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(y1), ptr(y2), None, R, H, float(eps),
         stream())
    return y1, y2


def set_gemm_tile(tile: int) -> None:
    """Force the GEMM block tile at any M (tests only): 128 (the 128x128 kernel), 256 / 224 / 192 (the persistent
    four-wave kernel's 256x256, 256x224 - N % 224 == 0 shapes that 256 does not divide, the Qwen2 hidden size 896 -
    and 256x192 - the QKV GEMMs with N % 192 == 0 - tiles); 0 = automatic by shape."""
    call("edge_gemm_set_tile", int(tile))


def set_gemm_ring(code: int) -> None:
    """DMA schedule of the paired-B h3 (fp32-mode) four-wave GEMMs per tile width: code = 100 x (192-wide QKV tiles)
    + 10 x (224-wide O-projection / down tiles) + (256-wide gate/up / LM-head tiles), each digit 0 two LDS buffers,
    1 the three-slot A ring (a K-tile's A and B pieces in different K-halves), 2 two buffers with the B pieces staged
    a K-half early; -1 from EDGE_GEMM_RING (three digits, default 022)."""
    call("edge_gemm_set_ring", int(code))


def set_gemm_store_wait(on: int) -> None:
    """The four-wave GEMMs leave a full tile's last epilogue stores in flight across the next tile's first K-tile wait
    (vmcnt counts stores; without this that wait drains them): 1 on, 0 off, -1 from EDGE_GEMM_STORE_WAIT."""
    call("edge_gemm_set_store_wait", int(on))


def gemm_ssq_parts(M: int, N: int, K: int, act=None, bias=False, residual=False) -> int:
    """Row sum-of-squares partials ``linear(..., want_ssq=True)`` produces for this shape: N/64 (64-column
    slabs), or N/112 (wave slabs) when the 256x224 kernel runs it."""
    return int(lib().edge_gemm_ssq_parts(M, N, K, _ACT[act], int(bool(bias)), int(bool(residual))))


def row_ssq(x: torch.Tensor) -> torch.Tensor:
    """Per-row sum of squares in 64-column slabs [T, H/64] (input of the fused-RMSNorm GEMMs)."""
    if not _gpu(x):
        return ref.row_ssq(x)
    _check_bf16(x)
    T, H = x.shape
    out = torch.empty(T, H // 64, dtype=torch.float32, device=x.device)
    call("edge_row_ssq", ptr(x), ptr(out), T, H, stream())
    return out


def row_rscale(ssq: torch.Tensor, K: int, eps: float) -> torch.Tensor:
    """rsqrt(sum(ssq_parts)/K + eps) per row: the fused RMSNorm's row scale [T] fp32."""
    if not ssq.is_cuda:
        return ref.rownorm_scale(ssq, K, eps)
    T, P = ssq.shape
    out = torch.empty(T, dtype=torch.float32, device=ssq.device)
    call("edge_row_rscale", ptr(ssq), ptr(out), T, P, K, float(eps), stream())
    return out


def _norm_scale(norm, K):
    """norm = (ssq_parts, eps) -> per-row scale tensor (device side)."""
    ssq, eps = norm
    return row_rscale(ssq, K, eps)


def linear(x: torch.Tensor, w: torch.Tensor, bias=None, residual=None, act=None, out=None, norm=None,
           want_ssq: bool = False) -> torch.Tensor:
    """``act(rowscale * (x @ w.T) + bias) + residual`` on MFMA (``residual`` may alias ``out``).

    ``norm=(ssq, eps)``: fused RMSNorm of ``x`` - rows are scaled by rsqrt(sum(ssq)/K + eps) (``w`` must
    carry the folded norm weight).  ``want_ssq``: the output's per-row sum-of-squares partials (64- or 112-column slabs)
    are produced in the epilogue and attached as ``out._edge_ssq`` (for the next fused norm)."""
    if not _gpu(x):
        y = ref.linear(x, w, None, None, None, out_dtype=torch.float32) if norm is not None else None
        if norm is not None:
            ssq, eps = norm
            y = y * ref.rownorm_scale(ssq, x.shape[1], eps).view(-1, 1)
            if bias is not None:
                y = y + bias.float()
            if act == "swiglu_il":
                g, u = ref.deinterleave_gate_up(y)
                y = torch.nn.functional.silu(g) * u
            elif act == "gelu":
                y = ref.gelu(y)
            if residual is not None:
                y = y + residual.float()
            y = y.to(x.dtype)
        else:
            y = ref.linear(x, w, bias, residual, act)
        if out is not None:
            out.copy_(y)
            y = out
        if want_ssq:
            y._edge_ssq = ref.row_ssq(y)
        return y
    _check_bf16(x, w, bias, residual)
    M, K = x.shape
    N = w.shape[0]
    No = N // 2 if act == "swiglu_il" else N
    if out is None:
        out = torch.empty(M, No, dtype=x.dtype, device=x.device)
    rs = None if norm is None else _norm_scale(norm, K)
    ssq_out = torch.empty(M, gemm_ssq_parts(M, N, K, act, bias is not None, residual is not None),
                          dtype=torch.float32, device=x.device) if want_ssq else None
    call("edge_gemm", ptr(x), ptr(w), ptr(out), M, N, K, x.stride(0), w.stride(0), out.stride(0), ptr(bias),
         ptr(residual), 0 if residual is None else residual.stride(0), _ACT[act], ptr(rs), ptr(ssq_out), stream())
    if want_ssq:
        out._edge_ssq = ssq_out
    return out


def qkv_rope(x, wqkv, bqkv, cos, sin, B, S, Hq, Hkv, D, rot_dim, q_scale, norm=None):
    """Fused QKV GEMM + bias + RoPE + head-major scatter (+ fused RMSNorm row scale).  Returns (q, k, vt)."""
    if not _gpu(x):
        if norm is not None:
            xs = (x.float() * ref.rownorm_scale(norm[0], x.shape[1], norm[1]).view(-1, 1))
            return ref.qkv_rope(xs, wqkv.float(), bqkv.float(), cos, sin, B, S, Hq, Hkv, D, rot_dim, q_scale)
        return ref.qkv_rope(x, wqkv, bqkv, cos, sin, B, S, Hq, Hkv, D, rot_dim, q_scale)
    _check_bf16(x, wqkv, bqkv)
    assert D == 64, "HIP attention path is specialised for head_dim 64"
    M, K = x.shape
    sp = s_pad(S)
    q = torch.empty(B, Hq, S, D, dtype=x.dtype, device=x.device)
    k = torch.empty(B, Hkv, S, D, dtype=x.dtype, device=x.device)
    vt = torch.zeros(B, Hkv, D, sp, dtype=x.dtype, device=x.device) if sp != S else \
        torch.empty(B, Hkv, D, sp, dtype=x.dtype, device=x.device)
    # fused RMSNorm: with 8 or 14 sum-of-squares partials per row the kernel forms the row scale itself at tile
    # start (no row_rscale launch)
    ssq, eps = norm if norm is not None else (None, 0.0)
    rs = None
    if ssq is not None:
        if ssq.shape[1] not in (8, 14) or not ssq.is_contiguous() or ssq.data_ptr() % 16:
            rs, ssq = _norm_scale(norm, K), None
    call("edge_gemm_qkv_rope", ptr(x), ptr(wqkv), ptr(bqkv), ptr(q), ptr(k), ptr(vt), ptr(cos), ptr(sin), M, K, S,
         Hq, Hkv, rot_dim, sp, float(q_scale), ptr(rs), ptr(ssq), 0 if ssq is None else ssq.shape[1], float(eps),
         stream())
    return q, k, vt


def attention(q, k, vt, S, need_lse=False, n_rows=None, h3: float = 0.0, in_scales=None, kv_planes=None,
              f32_out=False):
    """Causal GQA flash attention -> (o [B*S, Hq*64], lse [B,Hq,S] or None).

    ``n_rows`` ([B] fp32, scored rows per window as in ``WindowBatch.n_rows``): only query rows
    >= S-1-n_rows[b] are needed (last layer of the model); other 64-row blocks may be skipped and their
    output rows are then undefined.  fp32 q/k/vt run the fp32 kernels; ``h3`` = s > 0 then writes s * o as the
    2-plane h3 activation [B*S, 2*Hq*64] the O-projection consumes.  ``in_scales`` = (s_q, s_k, s_v), powers of two
    with s |x| <= 2^15 for every element of q, k and v: the matrix work runs on scaled fp16 planes (three products;
    the model derives them from weight bounds), else on three bf16 planes (six products).  ``kv_planes`` = (kp, vp)
    from ``qkv_rope_h3(kv_scales=(s_k, s_v))`` (with ``in_scales``): the kernel stages those planes by LDS DMA
    instead of splitting the fp32 K / V^T itself (the same result bit for bit).  ``f32_out`` (with ``h3`` and
    ``kv_planes``): O as fp32 rows too -> (o planes, lse, o fp32)."""
    if not _gpu(q):
        o, lse = ref.attention(q, k, vt, S, need_lse)
        if f32_out:
            return ref.h3_act(o, h3), lse, o
        return (ref.h3_act(o, h3) if h3 else o), lse
    B, Hq, _, D = q.shape
    Hkv = k.shape[1] if k is not None else kv_planes[0].shape[1]   # (k may be None when its planes are given)
    lse = torch.empty(B, Hq, S, dtype=torch.float32, device=q.device) if need_lse else None
    nr = None
    if n_rows is not None:
        nr = n_rows.to(device=q.device, dtype=torch.float32).contiguous()
        assert nr.numel() == B
    if q.dtype == torch.float32 and kv_planes is not None:
        kp, vp = kv_planes
        sp = vp.shape[-1]
        _check_f32(q)
        assert in_scales is not None and kp.dtype == torch.float16 and vp.dtype == torch.float16
        assert kp.shape == (B, Hkv, 2, S, D) and vp.shape == (B, Hkv, 2, D, sp) and sp % 64 == 0 and sp >= S
        assert kp.is_contiguous() and vp.is_contiguous() and kp.is_cuda and vp.is_cuda
        o = _out_f32_or_h3(B * S, Hq * D, h3, q.device)
        o32 = torch.empty(B * S, Hq * D, dtype=torch.float32, device=q.device) if f32_out else None
        assert not f32_out or h3, "f32_out: the fp32 rows next to the h3 planes"
        sq, sk, sv = in_scales
        call("edge_flash_attn_fwd_h3p", ptr(q), ptr(kp), ptr(vp), ptr(o), ptr(lse), ptr(nr), B, Hq, Hkv, S, sp,
             float(h3), float(sq), float(sk), float(sv), ptr(o32), stream())
        return (o, lse, o32) if f32_out else (o, lse)
    if q.dtype == torch.float32:
        _check_f32(q, k, vt)
        assert D == 64 and vt.shape[-1] % 64 == 0 and vt.shape[-1] >= S
        o = _out_f32_or_h3(B * S, Hq * D, h3, q.device)
        sq, sk, sv = in_scales if in_scales is not None else (0.0, 0.0, 0.0)
        call("edge_flash_attn_fwd_f32", ptr(q), ptr(k), ptr(vt), ptr(o), ptr(lse), ptr(nr), B, Hq, Hkv, S,
             vt.shape[-1], float(h3), float(sq), float(sk), float(sv), stream())
        return o, lse
    _check_bf16(q, k, vt)
    o = torch.empty(B * S, Hq * D, dtype=q.dtype, device=q.device)
    call("edge_flash_attn_fwd", ptr(q), ptr(k), ptr(vt), ptr(o), ptr(lse), ptr(nr), B, Hq, Hkv, S, vt.shape[-1],
         stream())
    return o, lse


def attn_lastrow(q, k, S, in_scales=None):
    """P[S-1, :] per head [B, Hq, S] fp32.  fp32 q/k with ``in_scales`` = (s_q, s_k) (the attention's plane scales):
    scores on the scaled fp16 planes of the forward (matrix cores); without: exact fp32 products."""
    if not _gpu(q):
        return ref.attn_lastrow(q, k, S)
    B, Hq = q.shape[:2]
    out = torch.empty(B, Hq, S, dtype=torch.float32, device=q.device)
    if q.dtype == torch.float32:
        sq, sk = in_scales if in_scales is not None else (0.0, 0.0)
        call("edge_attn_lastrow_f32", ptr(q), ptr(k), ptr(out), B, Hq, k.shape[1], S, float(sq), float(sk), stream())
        return out
    call("edge_attn_lastrow", ptr(q), ptr(k), ptr(out), B, Hq, k.shape[1], S, stream())
    return out


def attn_colsum(q, k, lse, S, in_scales=None):
    """Column sums sum_i P[i, j] per head [B, Hq, S] fp32 from q, k and the forward's row LSE.  fp32 q/k with
    ``in_scales`` = (s_q, s_k): the split-plane matrix-core kernel (the forward's scores); without: exact fp32."""
    if not _gpu(q):
        return ref.attn_colsum(q, k, lse, S)
    B, Hq = q.shape[:2]
    out = torch.empty(B, Hq, S, dtype=torch.float32, device=q.device)
    if q.dtype == torch.float32:
        sq, sk = in_scales if in_scales is not None else (0.0, 0.0)
        call("edge_attn_colsum_f32", ptr(q), ptr(k), ptr(lse.contiguous()), ptr(out), B, Hq, k.shape[1], S, float(sq),
             float(sk), stream())
        return out
    call("edge_attn_colsum", ptr(q), ptr(k), ptr(lse.contiguous()), ptr(out), B, Hq, k.shape[1], S, stream())
    return out


def head_combine(x, w=None, scale=1.0, out=None, beta=0.0):
    """out = beta*out + scale * sum_h w[h] * x[:, h, :]   (x: [B, Hq, S] fp32)."""
    if not _gpu(x):
        wv = torch.ones(x.shape[1], dtype=torch.float32) if w is None else w.float().to(x.device)
        r = scale * (x * wv.view(1, -1, 1)).sum(1)
        if out is None:
            return r
        out.mul_(beta).add_(r) if beta != 0.0 else out.copy_(r)
        return out
    B, Hq, S = x.shape
    if out is None:
        out = torch.empty(B, S, dtype=torch.float32, device=x.device)
        beta = 0.0
    wv = None if w is None else w.to(device=x.device, dtype=torch.float32).contiguous()
    call("edge_head_combine", ptr(x), ptr(wv), ptr(out), B, Hq, S, float(scale), float(beta), stream())
    return out


def head_nll(h, w, targets):
    """Fused LM head + cross entropy on the scored rows only: per-row NLL (fp32)."""
    if not _gpu(h):
        return ref.head_nll(h, w, targets)
    _check_bf16(h, w)
    R, K = h.shape
    V = w.shape[0]
    nparts = V // 64
    pmax = torch.empty(R, nparts, dtype=torch.float32, device=h.device)
    psum = torch.empty_like(pmax)
    tgt = torch.empty(R, dtype=torch.float32, device=h.device)
    nll = torch.empty(R, dtype=torch.float32, device=h.device)
    t64 = targets.to(torch.int64).contiguous()
    call("edge_gemm_lse", ptr(h), ptr(w), ptr(t64), ptr(pmax), ptr(psum), ptr(tgt), R, V, K, 0, 0.0, stream())
    call("edge_lse_reduce", ptr(pmax), ptr(psum), ptr(tgt), ptr(nll), R, nparts, stream())
    return nll


# ---- fp32 execution mode: h3 GEMMs (csrc/gemm.hip EPI_F32*, EPI_H3_*) ---------------------------------------
def split_h3(x: torch.Tensor, s: float, rows: torch.Tensor | None = None) -> torch.Tensor:
    """fp32 [R, K] (optionally rows gathered) -> 2-plane h3 activation of s * x, [R, 2K] fp16."""
    if not _gpu(x):
        return ref.h3_act(x if rows is None else x.index_select(0, rows.long()), s)
    _check_f32(x)
    R = x.shape[0] if rows is None else rows.numel()
    rows32 = None if rows is None else rows.to(torch.int32).contiguous()
    y = torch.empty(R, 2 * x.shape[1], dtype=torch.float16, device=x.device)
    call("edge_split_h3", ptr(x), ptr(y), ptr(rows32), R, x.shape[1], float(s), stream())
    return y


def linear_h3(a3: torch.Tensor, w3: torch.Tensor, alpha: float, bias=None, residual=None, act=None, out=None,
              rscale=None, out_scale: float = 1.0, colscale=None, planes_bound=None):
    """fp32-accurate ``act(rscale * (x @ w.T) + bias) + residual`` from h3 operands (a3 [M, 2K] the 2-plane
    activation of s_a x, w3 [N, 3K] the h3 weight of w at scale s_w, alpha = 1 / (s_a s_w)).

    act None -> fp32 [M, N] (``residual`` fp32, may alias ``out``); act "gelu" / "swiglu_il" -> the activation as
    the 2-plane h3 activation of ``out_scale`` * act(...) ([M, 2N] / [M, N]) for the next GEMM.
    ``colscale`` [N] (with a residual, no bias / act): ``colscale * rscale * (x @ w.T) + residual`` - a norm weight on
    the output columns instead of folded into w, which then keeps a weight exact in fp16 on two products.
    ``planes_bound`` = (bnd_a [M], bnd_b [M], c) with ``colscale``: the result also as the h3 activation of the next
    backward GEMM, at per-row powers of two from the caller's bound 2^15 (bnd_a + bnd_b c) on |row| (no row-max pass)
    -> (out, planes [M, 2N], rinv [M])."""
    M = a3.shape[0]
    N = w3.shape[0]
    if not _gpu(a3):
        y = ref.h3_matmul(a3, w3, alpha)
        if rscale is not None:
            y = y * rscale.float().view(-1, 1)
        if colscale is not None:
            y = y * colscale.float().view(1, -1)
        if bias is not None:
            y = y + bias.float()
        if act == "gelu":
            return ref.h3_act(ref.gelu(y), out_scale)
        if act == "swiglu_il":
            g, u = ref.deinterleave_gate_up(y)
            return ref.h3_act(torch.nn.functional.silu(g) * u, out_scale)
        if residual is not None:
            y = y + residual.float()
        if out is not None:
            out.copy_(y)
            y = out
        if planes_bound is not None:
            return (y,) + ref.bound_planes(y, *planes_bound)
        return y
    kp, Kx = _check_h3(a3, w3, alpha)
    _check_f32(bias, residual, rscale, colscale)
    if colscale is not None:
        if residual is None or bias is not None or act is not None:
            raise ValueError("colscale: a residual GEMM without bias / activation")
        if out is None:
            out = torch.empty(M, N, dtype=torch.float32, device=a3.device)
        pl = pr = ba = bb = None
        bc = 0.0
        if planes_bound is not None:
            ba, bb, bc = planes_bound
            _check_f32(ba, bb)
            assert ba.numel() == M and bb.numel() == M
            pl = torch.empty(M, 2 * N, dtype=torch.float16, device=a3.device)
            pr = torch.empty(M, dtype=torch.float32, device=a3.device)
        call("edge_gemm_f32_cs", ptr(a3), ptr(w3), ptr(out), M, N, Kx, kp, a3.stride(0), w3.stride(0), out.stride(0),
             ptr(colscale), ptr(residual), residual.stride(0), ptr(rscale), float(alpha), ptr(pl), ptr(pr), ptr(ba),
             ptr(bb), float(bc), stream())
        return out if planes_bound is None else (out, pl, pr)
    if act is None:
        if out is None:
            out = torch.empty(M, N, dtype=torch.float32, device=a3.device)
        ldc = out.stride(0)
        code = 0
    else:
        No = N // 2 if act == "swiglu_il" else N
        out = torch.empty(M, 2 * No, dtype=torch.float16, device=a3.device)
        ldc = 2 * No
        code = _ACT[act]
    call("edge_gemm_f32", ptr(a3), ptr(w3), ptr(out), M, N, Kx, kp, a3.stride(0), w3.stride(0), ldc, ptr(bias),
         ptr(residual), 0 if residual is None else residual.stride(0), code, ptr(rscale), float(alpha),
         float(out_scale), stream())
    return out


def gemm_np_supported(M: int, N: int, Kx: int) -> bool:
    """Whether ``linear_h3_np`` runs this GPU shape (the 256x224 persistent tiles: N % 224 == 0, N % 256 != 0 and at
    least one tile per CU)."""
    return bool(lib().edge_gemm_f32_np_ok(int(M), int(N), int(Kx)))


def linear_h3_np(a3: torch.Tensor, w3: torch.Tensor, alpha: float, residual: torch.Tensor, g: torch.Tensor,
                 rstd_in: torch.Tensor, g_max: float, prod_bound: float, out: torch.Tensor | None = None):
    """The O-projection / down GEMM with the NEXT RMSNorm's producer side fused into its epilogue (no separate norm
    pass): y = alpha (x @ w.T) + residual (fp32, ``out`` may alias ``residual``) and, for the GEMM that consumes
    rmsnorm(y) * g, the h3 planes of p_m (y_m * g) at a power-of-two row scale p_m from the bound
    g_max (sqrt(N) / rstd_in[m] + prod_bound) on |y_m * g| (``rstd_in``: the residual's own RMSNorm normalisers,
    ``prod_bound``: a bound on |alpha (x @ w.T)|, ``g_max`` = max |g|), 1 / p_m and y's row sum-of-squares partials
    -> (y, planes [M, 2N], prinv [M], ssq [M, N / 112]).  The consumer takes ``rscale = row_rscale_mul(ssq, prinv)`` and
    its weight's own product scale (no activation scale)."""
    M, N = a3.shape[0], w3.shape[0]
    if not _gpu(a3):
        y = ref.h3_matmul(a3, w3, alpha) + residual.float()
        if out is not None:
            out.copy_(y)
            y = out
        return (y,) + ref.np_planes(y, g, rstd_in, g_max, prod_bound)
    kp, Kx = _check_h3(a3, w3, alpha)
    _check_f32(residual, g, rstd_in, out)
    if N % 112:
        raise ValueError(f"linear_h3_np: N = {N} is not a multiple of the 112-column slabs")
    if out is None:
        out = torch.empty(M, N, dtype=torch.float32, device=a3.device)
    planes = torch.empty(M, 2 * N, dtype=torch.float16, device=a3.device)
    prinv = torch.empty(M, dtype=torch.float32, device=a3.device)
    ssq = torch.empty(M, N // 112, dtype=torch.float32, device=a3.device)
    call("edge_gemm_f32_np", ptr(a3), ptr(w3), ptr(out), M, N, Kx, kp, a3.stride(0), w3.stride(0), out.stride(0),
         ptr(residual), residual.stride(0), float(alpha), ptr(g), ptr(rstd_in), float(g_max), float(prod_bound),
         ptr(planes), ptr(prinv), ptr(ssq), stream())
    return out, planes, prinv, ssq


def row_rscale_mul(ssq: torch.Tensor, mul: torch.Tensor, K: int, eps: float) -> torch.Tensor:
    """rsqrt(sum(ssq_parts) / K + eps) * mul per row: the consumer row scale of ``linear_h3_np``'s fused RMSNorm."""
    if not ssq.is_cuda:
        return ref.row_rscale_mul(ssq, mul, K, eps)
    _check_f32(ssq, mul)
    T, P = ssq.shape
    out = torch.empty(T, dtype=torch.float32, device=ssq.device)
    call("edge_row_rscale_mul", ptr(ssq), ptr(mul), ptr(out), T, P, K, float(eps), stream())
    return out


def linear_swiglu_raw(x: torch.Tensor, w: torch.Tensor, norm=None):
    """``linear(x, w, act="swiglu_il", norm=norm)`` that also returns the pre-activations ``linear(x, w, norm=norm)``
    (interleaved gate|up [M, N], bit-identical) from the same GEMM -> (activation [M, N/2], pre-activations)."""
    if not _gpu(x):
        y = ref.linear(x, w, None, None, None, out_dtype=torch.float32)
        if norm is not None:
            y = y * ref.rownorm_scale(norm[0], x.shape[1], norm[1]).view(-1, 1)
        g, u = ref.deinterleave_gate_up(y)
        return (torch.nn.functional.silu(g) * u).to(x.dtype), y.to(x.dtype)
    _check_bf16(x, w)
    M, K = x.shape
    N = w.shape[0]
    act = torch.empty(M, N // 2, dtype=x.dtype, device=x.device)
    raw = torch.empty(M, N, dtype=x.dtype, device=x.device)
    rs = None if norm is None else _norm_scale(norm, K)
    call("edge_gemm_swiglu_raw", ptr(x), ptr(w), ptr(act), ptr(raw), M, N, K, x.stride(0), w.stride(0), act.stride(0),
         ptr(rs), stream())
    return act, raw


def linear_h3_swiglu_raw(a3: torch.Tensor, w3: torch.Tensor, alpha: float, out_scale: float, rscale=None):
    """``linear_h3(..., act="swiglu_il", out_scale)`` that also returns the fp32 pre-activations
    ``rscale * (x @ w.T)`` (interleaved gate|up [M, N], bit-identical to ``linear_h3`` without ``act``) from the same
    GEMM: the SwiGLU planes and the saved pre-activations of the AttnLRP forward in one pass, instead of an fp32 GEMM
    plus an ``act_h3`` pass re-reading its output -> (planes [M, N], pre-activations [M, N])."""
    M, N = a3.shape[0], w3.shape[0]
    if not _gpu(a3):
        y = ref.h3_matmul(a3, w3, alpha)
        if rscale is not None:
            y = y * rscale.float().view(-1, 1)
        g, u = ref.deinterleave_gate_up(y)
        return ref.h3_act(torch.nn.functional.silu(g) * u, out_scale), y
    kp, Kx = _check_h3(a3, w3, alpha)
    _check_f32(rscale)
    planes = torch.empty(M, N, dtype=torch.float16, device=a3.device)
    raw = torch.empty(M, N, dtype=torch.float32, device=a3.device)
    call("edge_gemm_f32_swiglu_raw", ptr(a3), ptr(w3), ptr(planes), ptr(raw), M, N, Kx, kp, a3.stride(0),
         w3.stride(0), N, ptr(rscale), float(alpha), float(out_scale), stream())
    return planes, raw


def qkv_rope_h3(a3, w3, alpha, bias, cos, sin, B, S, Hq, Hkv, D, rot_dim, q_scale, kv_scales=None, need_k=True,
                v_rows=False):
    """fp32 fused QKV projection + bias + RoPE + head-major scatter from h3 operands -> fp32 (q, k, vt).

    ``kv_scales`` = (s_k, s_v): also the K / V^T h3 planes at those scales for ``attention(kv_planes=...)`` ->
    (q, k, vt, kp, vp); on the GPU ``vt`` is then None (the planes replace it), and with ``need_k=False`` so is the
    fp32 ``k`` (the attention stages the planes; only the importance scorers read fp32 K).  ``v_rows``: V row-major
    fp32 [B, Hkv, S, 64] appended to the outputs (the AttnLRP backward's V, from the same epilogue)."""
    if not _gpu(a3):
        y = ref.h3_matmul(a3, w3, alpha)            # x @ w.T, then the rest of the fused op on fp32
        eye = torch.eye(y.shape[1], dtype=torch.float32)
        q, k, vt = ref.qkv_rope(y, eye, bias.float(), cos, sin, B, S, Hq, Hkv, D, rot_dim, q_scale)
        out = (q, k, vt) if kv_scales is None else (q, k, vt) + ref.kv_planes(k, vt, *kv_scales)
        return out + ((vt[..., :S].transpose(-1, -2).contiguous(),) if v_rows else ())
    kp, Kx = _check_h3(a3, w3, alpha)
    _check_f32(bias)
    assert D == 64, "HIP attention path is specialised for head_dim 64"
    M = a3.shape[0]
    sp = s_pad(S)
    f32 = dict(dtype=torch.float32, device=a3.device)
    q = torch.empty(B, Hq, S, D, **f32)
    k = torch.empty(B, Hkv, S, D, **f32) if (need_k or kv_scales is None) else None
    kpl = vpl = vt = None
    if kv_scales is None:
        vt = torch.zeros(B, Hkv, D, sp, **f32) if sp != S else torch.empty(B, Hkv, D, sp, **f32)
    else:   # the planes replace the fp32 V^T (only the attention reads it)
        f16 = dict(dtype=torch.float16, device=a3.device)
        kpl = torch.empty(B, Hkv, 2, S, D, **f16)
        vpl = torch.zeros(B, Hkv, 2, D, sp, **f16) if sp != S else torch.empty(B, Hkv, 2, D, sp, **f16)
    v = torch.empty(B, Hkv, S, D, **f32) if v_rows else None
    sk_, sv_ = kv_scales if kv_scales is not None else (0.0, 0.0)
    call("edge_gemm_qkv_rope_f32", ptr(a3), ptr(w3), ptr(bias), ptr(q), ptr(k), ptr(vt), ptr(cos), ptr(sin), M, Kx, kp, S,
         Hq, Hkv, rot_dim, sp, float(q_scale), float(alpha), ptr(kpl), ptr(vpl), float(sk_), float(sv_), ptr(v),
         stream())
    out = (q, k, vt) if kv_scales is None else (q, k, vt, kpl, vpl)
    return out + ((v,) if v_rows else ())


def head_nll_h3(a3: torch.Tensor, w3: torch.Tensor, alpha: float, targets: torch.Tensor) -> torch.Tensor:
    """fp32 fused LM head + cross entropy on the scored rows from h3 operands: per-row NLL."""
    if not _gpu(a3):
        logits = ref.h3_matmul(a3, w3, alpha)
        return torch.logsumexp(logits, -1) - logits.gather(1, targets.long().view(-1, 1)).squeeze(1)
    kp, Kx = _check_h3(a3, w3, alpha)
    R = a3.shape[0]
    V = w3.shape[0]
    nparts = V // 64
    f32 = dict(dtype=torch.float32, device=a3.device)
    pmax, psum = torch.empty(R, nparts, **f32), torch.empty(R, nparts, **f32)
    tgt, nll = torch.empty(R, **f32), torch.empty(R, **f32)
    t64 = targets.to(torch.int64).contiguous()
    call("edge_gemm_lse", ptr(a3), ptr(w3), ptr(t64), ptr(pmax), ptr(psum), ptr(tgt), R, V, Kx, kp, float(alpha),
         stream())
    call("edge_lse_reduce", ptr(pmax), ptr(psum), ptr(tgt), ptr(nll), R, nparts, stream())
    return nll


# ---- AttnLRP relevance backward (csrc/lrp.hip) ---------------------------------------------------------
def linear_rowscale(x: torch.Tensor, w: torch.Tensor, rscale: torch.Tensor, residual=None) -> torch.Tensor:
    """``rscale[:, None] * (x @ w.T) + residual`` (rscale fp32 [M]): the input-gradient GEMM of a norm-folded
    projection under the detached-normaliser rule."""
    if not _gpu(x):
        y = ref._f(x) @ ref._f(w).t() * rscale.float().view(-1, 1)
        if residual is not None:
            y = y + ref._f(residual)
        return y.to(x.dtype)
    _check_bf16(x, w, residual)
    M, K = x.shape
    N = w.shape[0]
    out = torch.empty(M, N, dtype=x.dtype, device=x.device)
    rs = rscale.to(torch.float32).contiguous()
    call("edge_gemm", ptr(x), ptr(w), ptr(out), M, N, K, x.stride(0), w.stride(0), out.stride(0), None,
         ptr(residual), 0 if residual is None else residual.stride(0), 0, ptr(rs), None, stream())
    return out


def lrp_gqa_sum_native(t: torch.Tensor) -> bool:
    """True when ``lrp_attn_bwd(..., gqa_sum=True)`` computes the GQA group sums in the kernel for tensors like ``t``
    (fp32 on the GPU)."""
    return _gpu(t) and t.dtype == torch.float32


def lrp_attn_bwd(q, k, v, o, dO, lse, gqa_sum: bool = False, in_scales=None):
    """-> (D [B,Hq,S], rel [B,Hq], dq, dk, dv [B,Hq,S,64]) fp32 (dk/dv per-q-head partials); see
    ``reference.lrp_attn_bwd``.  ``gqa_sum``: dk, dv as the sums over each GQA group, [B,Hkv,S,64] (the fp32 sweeps
    compute them directly; elsewhere the partials are summed).  fp32: the sweeps run on scaled fp16 planes (three
    products, csrc/lrp_f32.hip lrp_attn_*_h3; dO's scale from its per-head maxima) at ``in_scales`` = (s_q, s_k,
    s_v), the forward attention's plane scales (powers of two, s |x| <= 2^15); without them the scales are taken
    from the tensors' maxima."""
    B, Hq, S, D = q.shape
    Hkv = k.shape[1]
    if not _gpu(q):
        Dl, rel, dq, dk, dv = ref.lrp_attn_bwd(q, k, v, o, dO, lse)
        if gqa_sum:
            dk, dv = (t.view(B, Hkv, Hq // Hkv, S, D).sum(2) for t in (dk, dv))
        return Dl, rel, dq, dk, dv
    fp32 = q.dtype == torch.float32
    (_check_f32 if fp32 else _check_bf16)(q, k, v, o, dO)
    assert D == 64 and k.shape == v.shape == (B, Hkv, S, D) and o.shape == dO.shape == (B * S, Hq * D)
    assert lse.shape == (B, Hq, S) and lse.dtype == torch.float32 and lse.is_contiguous()
    f32 = dict(dtype=torch.float32, device=q.device)
    Dl, rel = torch.empty(B, Hq, S, **f32), torch.empty(B, Hq, **f32)
    dq = torch.empty(B, Hq, S, D, **f32)
    args = (ptr(q), ptr(k), ptr(v), ptr(o), ptr(dO), ptr(lse), ptr(Dl), ptr(rel), ptr(dq))
    if fp32:
        if in_scales is None:
            in_scales = tuple(ref.h3_scale(t.abs().max().item()) for t in (q, k, v))
        gs = bool(gqa_sum)
        Hk = Hkv if gs else Hq
        dk, dv = torch.empty(B, Hk, S, D, **f32), torch.empty(B, Hk, S, D, **f32)
        dmax = torch.empty(B * Hq, **f32)
        sq, sk, sv = (float(x) for x in in_scales)
        call("edge_lrp_attn_bwd_h3", *args, ptr(dk), ptr(dv), ptr(dmax), B, Hq, Hkv, S, int(gs), sq, sk, sv, stream())
        return Dl, rel, dq, dk, dv
    dk, dv = torch.empty(B, Hq, S, D, **f32), torch.empty(B, Hq, S, D, **f32)
    call("edge_lrp_attn_bwd", *args, ptr(dk), ptr(dv), B, Hq, Hkv, S, stream())
    if gqa_sum:
        dk, dv = (t.view(B, Hkv, Hq // Hkv, S, D).sum(2) for t in (dk, dv))
    return Dl, rel, dq, dk, dv


def lrp_rope_pack(dq, dk, dv, cos, sin, B, S, Hq, Hkv, rot_dim, q_scale, dtype=torch.bfloat16):
    if not _gpu(dq):
        return ref.lrp_rope_pack(dq, dk, dv, cos, sin, B, S, Hq, Hkv, rot_dim, q_scale, dtype)
    for t in (dq, dk, dv):
        assert t.dtype == torch.float32 and t.is_contiguous()
    out = torch.empty(B * S, (Hq + 2 * Hkv) * 64, dtype=torch.bfloat16, device=dq.device)
    call("edge_lrp_rope_pack", ptr(dq), ptr(dk), ptr(dv), ptr(cos), ptr(sin), ptr(out), B, S, Hq, Hkv, rot_dim,
         float(q_scale), stream())
    return out


def swiglu_il(gu: torch.Tensor) -> torch.Tensor:
    if not _gpu(gu):
        return ref.swiglu_il(gu)
    _check_bf16(gu)
    T, N2 = gu.shape
    a = torch.empty(T, N2 // 2, dtype=gu.dtype, device=gu.device)
    call("edge_swiglu_il", ptr(gu), ptr(a), T, N2 // 2, stream())
    return a


def lrp_swiglu_bwd(dm: torch.Tensor, gu: torch.Tensor) -> torch.Tensor:
    if not _gpu(gu):
        return ref.lrp_swiglu_bwd(dm, gu)
    _check_bf16(dm, gu)
    T, N2 = gu.shape
    assert dm.shape == (T, N2 // 2)
    dgu = torch.empty_like(gu)
    call("edge_lrp_swiglu_bwd", ptr(dm), ptr(gu), ptr(dgu), T, N2 // 2, stream())
    return dgu


def lrp_gelu_bwd(dy: torch.Tensor, a: torch.Tensor) -> torch.Tensor:
    if not _gpu(dy):
        return ref.lrp_gelu_bwd(dy, a)
    _check_bf16(dy, a)
    out = dy.clone()
    call("edge_lrp_gelu_bwd", ptr(out), ptr(a), out.numel(), stream())
    return out


def ln_rstd(x: torch.Tensor, eps: float) -> torch.Tensor:
    if not _gpu(x):
        return ref.ln_rstd(x, eps)
    _check_bf16(x)
    R, H = x.shape
    out = torch.empty(R, dtype=torch.float32, device=x.device)
    call("edge_ln_rstd", ptr(x), ptr(out), R, H, float(eps), stream())
    return out


def lrp_ln_bwd(dy1, rs1, w1, dy2, rs2, w2, resid):
    if not _gpu(resid):
        return ref.lrp_ln_bwd(dy1, rs1, w1, dy2, rs2, w2, resid)
    _check_bf16(dy1, w1, dy2, w2, resid)
    R, H = resid.shape
    out = torch.empty_like(resid)
    call("edge_lrp_ln_bwd", ptr(dy1), ptr(rs1), ptr(w1), ptr(dy2), ptr(rs2), ptr(w2), ptr(resid), ptr(out), R, H,
         stream())
    return out


# ---- fp32 AttnLRP (csrc/lrp_f32.hip): rule outputs as per-row-scaled h3 GEMM inputs ---------------------------
def _rows_out(R: int, K: int, device):
    return (torch.empty(R, 2 * K, dtype=torch.float16, device=device),
            torch.empty(R, dtype=torch.float32, device=device))


def _post(post, R):
    if post is None:
        return None
    _check_f32(post)
    assert post.numel() == R
    return post


def split_h3_dyn(x: torch.Tensor, post: torch.Tensor | None = None):
    """fp32 [R, K] -> (h3 activation [R, 2K] with a per-row power-of-two scale s_r, rinv [R] = post / s_r): the
    input of a backward GEMM (``linear_h3(..., rscale=rinv)`` undoes the scale exactly)."""
    if not _gpu(x):
        return ref.split_h3_dyn(x, post)
    _check_f32(x)
    R, K = x.shape
    out, rinv = _rows_out(R, K, x.device)
    call("edge_split_h3_dyn", ptr(x), ptr(out), ptr(rinv), ptr(_post(post, R)), R, K, stream())
    return out, rinv


def lrp_swiglu_bwd_h3(dm: torch.Tensor, gu: torch.Tensor, post: torch.Tensor | None = None):
    """SwiGLU LRP rule (fp32 dm [T, I], saved gate|up pre-activations gu [T, 2I]) -> (h3 d[gate|up] [T, 4I], rinv)."""
    if not _gpu(gu):
        return ref.lrp_swiglu_bwd_h3(dm, gu, post)
    _check_f32(dm, gu)
    T, N2 = gu.shape
    assert dm.shape == (T, N2 // 2)
    out, rinv = _rows_out(T, N2, gu.device)
    call("edge_lrp_swiglu_bwd_h3", ptr(dm), ptr(gu), ptr(out), ptr(rinv), ptr(_post(post, T)), T, N2 // 2, stream())
    return out, rinv


def linear_h3_lrp_swiglu(a3: torch.Tensor, w3: torch.Tensor, alpha: float, gu: torch.Tensor, c0: float,
                         rinv: torch.Tensor, post: torch.Tensor | None = None):
    """The MLP backward's dm GEMM with the SwiGLU LRP rule in its epilogue: a3 the per-row-scaled h3 gradient
    (``split_h3_dyn`` -> rinv), w3 the transposed down-projection weight, gu the saved interleaved pre-activations
    [T, 2I] -> (h3 d[gate|up] [T, 4I], its row scale [T]) - what ``lrp_swiglu_bwd_h3(linear_h3(a3, w3, alpha,
    rscale=rinv), gu, post)`` returns, without the fp32 dm round trip or the rule's row-max pass.

    The planes are at a fixed scale: the rule runs on c0 x (the product still at a3's row scale, max |row| < 2^15);
    c0 (a power of two) must keep 2^15 x 0.5 max|dm / dx| x max|gu| under 2^15 (``lrp_swiglu_scale``) - an a-priori
    bound from the weights replaces the row max that needs every column tile.  The row scale rinv post / c0 is exact
    (powers of two times the detached norm's rstd)."""
    rs = rinv / c0 if post is None else rinv * _post(post, rinv.numel()) / c0
    if not _gpu(a3):
        return ref.linear_h3_lrp_swiglu(a3, w3, alpha, gu, c0, rinv, post)
    kp, Kx = _check_h3(a3, w3, alpha)
    _check_f32(gu)
    M, N = a3.shape[0], w3.shape[0]
    assert gu.shape == (M, 2 * N) and gu.stride(1) == 1
    out = torch.empty(M, 4 * N, dtype=torch.float16, device=a3.device)
    call("edge_gemm_f32_lrp_swiglu", ptr(a3), ptr(w3), ptr(out), ptr(gu), M, N, Kx, kp, a3.stride(0), w3.stride(0),
         gu.stride(0), float(alpha * c0), stream())
    return out, rs


def lrp_swiglu_scale(wd: torch.Tensor, wgu: torch.Tensor, norm_w: torch.Tensor) -> float:
    """c0 of ``linear_h3_lrp_swiglu`` for a Qwen2 MLP (wd [H, I] down, wgu [2I, H] interleaved gate|up, norm_w [H]
    the post-attention RMSNorm weight): |dm_c| <= max|dx| max_c sum_k |wd[k, c]| and |g|, |u| <= sqrt(H)
    max_j ||wgu_j * norm_w||_2 (the normalised row has ||x_hat||_2 <= sqrt(H)); |dg|, |du| <= 0.5 |dm| max(|g|, |u|).
    The largest power of two with 2^15 x that bound x c0 <= 2^15."""
    H = wd.shape[0]
    cd = float(wd.float().abs().sum(0).max())
    bgu = float((wgu.float() * norm_w.float().view(1, -1)).norm(dim=1).max()) * H ** 0.5
    bound = 0.5 * cd * bgu * (1 + 2 ** -10)   # margin for the product's own rounding
    return 2.0 ** -math.ceil(math.log2(bound)) if bound > 0 else 1.0


def lrp_gelu_bwd_h3(dy: torch.Tensor, a: torch.Tensor):
    """GELU identity rule (fp32) -> (h3 [T, 2I], rinv)."""
    if not _gpu(a):
        return ref.lrp_gelu_bwd_h3(dy, a)
    _check_f32(dy, a)
    T, I = a.shape
    out, rinv = _rows_out(T, I, a.device)
    call("edge_lrp_gelu_bwd_h3", ptr(dy), ptr(a), ptr(out), ptr(rinv), T, I, stream())
    return out, rinv


def lrp_rope_pack_h3(dq, dk, dv, cos, sin, B, S, Hq, Hkv, rot_dim, q_scale, post=None):
    """Inverse RoPE + q scale + GQA sum + token-major scatter (fp32) -> (h3 d[q|k|v] [B*S, 2(Hq+2Hkv)64], rinv).
    dk, dv: per-q-head partials [B,Hq,S,64] or already the GQA group sums [B,Hkv,S,64]."""
    if not _gpu(dq):
        return ref.lrp_rope_pack_h3(dq, dk, dv, cos, sin, B, S, Hq, Hkv, rot_dim, q_scale, post)
    _check_f32(dq, dk, dv, cos, sin)
    assert dq.shape == (B, Hq, S, 64) and dk.shape == dv.shape and dk.shape in ((B, Hq, S, 64), (B, Hkv, S, 64))
    summed = dk.shape[1] == Hkv and Hq != Hkv
    out, rinv = _rows_out(B * S, (Hq + 2 * Hkv) * 64, dq.device)
    call("edge_lrp_rope_pack_h3_gs" if summed else "edge_lrp_rope_pack_h3", ptr(dq), ptr(dk), ptr(dv), ptr(cos),
         ptr(sin), ptr(out), ptr(rinv), ptr(_post(post, B * S)), B, S, Hq, Hkv, rot_dim, float(q_scale), stream())
    return out, rinv


def act_h3(x: torch.Tensor, act: str, s: float) -> torch.Tensor:
    """Forward activation of saved fp32 pre-activations ("swiglu_il": interleaved gate|up [T, 2I] -> [T, I];
    "gelu": [T, I]) as the next GEMM's h3 input at the model scale ``s``."""
    if not _gpu(x):
        return ref.act_h3(x, act, s)
    _check_f32(x)
    T, N = x.shape
    I = N // 2 if act == "swiglu_il" else N
    out = torch.empty(T, 2 * I, dtype=torch.float16, device=x.device)
    call("edge_act_h3", ptr(x), ptr(out), T, I, 0 if act == "swiglu_il" else 1, float(s), stream())
    return out


def row_rstd(x: torch.Tensor, eps: float, center: bool = False) -> torch.Tensor:
    """fp32 rows -> rsqrt(mean(x^2) + eps) (RMSNorm), of the centred row with ``center`` (LayerNorm)."""
    if not _gpu(x):
        return ref.row_rstd(x, eps, center)
    _check_f32(x)
    R, H = x.shape
    out = torch.empty(R, dtype=torch.float32, device=x.device)
    call("edge_row_rstd_f32", ptr(x), ptr(out), R, H, float(eps), int(center), stream())
    return out


def lrp_ln_bwd_f32(dy1, rs, w1, dy2, w2, resid):
    """fp32 LayerNorm rule of a dual norm sharing one input (and so one rstd ``rs``)."""
    if not _gpu(resid):
        return ref.lrp_ln_bwd(dy1, rs, w1, dy2, rs, w2, resid)
    _check_f32(dy1, rs, w1, dy2, w2, resid)
    R, H = resid.shape
    out = torch.empty_like(resid)
    call("edge_lrp_ln_bwd_f32", ptr(dy1), ptr(rs), ptr(w1), ptr(dy2), ptr(w2), ptr(resid), ptr(out), R, H, stream())
    return out


def group_absprod(x: torch.Tensor, dx: torch.Tensor, B: int, S: int, out: torch.Tensor | None = None,
                  sens_out: torch.Tensor | None = None):
    """[B, H/64] sums of |x dx| per window and 64-channel group (into ``out`` [B, >= H/64] rows if given).
    ``sens_out`` (same layout as ``out``): also the groups' quantization sensitivity (``reference.group_sens``)."""
    if not _gpu(x):
        r = ref.group_absprod(x, dx, B, S)
        if sens_out is not None:
            sens_out.copy_(ref.group_sens(x, dx, B, S))
        if out is not None:
            out.copy_(r)
            return out
        return r
    _check_f32(x, dx)
    H = x.shape[1]
    if out is None:
        out = torch.empty(B, H // 64, dtype=torch.float32, device=x.device)
    assert out.dtype == torch.float32 and out.stride(1) == 1
    if sens_out is not None:
        assert sens_out.dtype == torch.float32 and sens_out.stride() == out.stride() and sens_out.shape == out.shape
    call("edge_group_absprod", ptr(x), ptr(dx), ptr(out), ptr(sens_out), B, S, H, out.stride(0), stream())
    return out
