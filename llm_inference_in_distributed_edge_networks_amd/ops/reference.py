"""Plain-PyTorch fp32 implementations of every op.

These are the numerics oracle for the HIP kernels (tests compare each kernel
against the function of the same name here) and the execution path on CPU
(BASELINE config 1 "CPU WikiText-2 PPL").  They use exactly the tensor layouts
of the HIP kernels so that the two are interchangeable op by op:

* activations are token-major ``[T, H]`` with ``T = B * S``;
* ``q`` is ``[B, Hq, S, D]`` with RoPE applied and pre-multiplied by ``q_scale``;
* ``k`` is ``[B, Hkv, S, D]`` with RoPE applied;
* ``vt`` is V transposed, ``[B, Hkv, D, S_pad]`` with ``S_pad = ceil(S/64)*64``
  and zero padding (the attention kernel streams 64-key tiles of it);
* gate/up weights of SwiGLU MLPs are interleaved in blocks of 16 rows
  (``[g0..g15, u0..u15, g16..]``) so one GEMM tile holds matching gate and up
  columns and the SiLU*up product is an epilogue.

Reference sites of the ops (SURVEY §2.4 K-ids; paths relative to the reference repo):
embedding K1 (``Experiments/Qwen2-0.5B/qwen_layer_wise.py:46``), RoPE K2 (``qwen_layer_wise.py:47-48``,
partial rotary ``Experiments/Pythia-70M/pythia_model.py:158-161``), RMSNorm / LayerNorm K3
(``qwen_layer_wise.py:75``, ``pythia_model.py:193``), causal SDPA attention K5 (``qwen_layer_wise.py:17``),
eager attention probabilities K6 (``Experiments/Qwen2-0.5B/main.py:159``; here ``attention_probs``, test-only),
LM head + shifted CE K9/K10 (``qwen_layer_wise.py:28-40``), importance reductions K11
(``Experiments/Qwen2-0.5B/main.py:46-92``), AttnLRP backward K17 (``Experiments/Relevance/main.py:84-103``).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

IL_BLOCK = 16  # gate/up interleave granularity (rows)


def _f(x):
    """fp32 view of an operand (fp64 stays fp64: the oracles also run in double precision for the tests)."""
    return x if x.dtype == torch.float64 else x.float()


def embedding(ids: torch.Tensor, table: torch.Tensor) -> torch.Tensor:
    return table.index_select(0, ids.reshape(-1).long())


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    # HF Qwen2RMSNorm: fp32 variance, cast back to input dtype, then * weight.
    xf = _f(x)
    var = xf.pow(2).mean(-1, keepdim=True)
    y = (xf * torch.rsqrt(var + eps)).to(x.dtype)
    return (w * y).to(x.dtype)


def layernorm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float) -> torch.Tensor:
    return F.layer_norm(_f(x), (x.shape[-1],), _f(w), _f(b), eps).to(x.dtype)


def layernorm_dual(x, w1, b1, w2, b2, eps):
    return layernorm(x, w1, b1, eps), layernorm(x, w2, b2, eps)


def gelu(x: torch.Tensor) -> torch.Tensor:
    return F.gelu(x)  # exact (erf) GELU, HF "gelu"


def deinterleave_gate_up(y: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """Split the output of an interleaved gate/up GEMM into (gate, up)."""
    T, N2 = y.shape
    y4 = y.reshape(T, N2 // (2 * IL_BLOCK), 2, IL_BLOCK)
    return y4[:, :, 0, :].reshape(T, N2 // 2), y4[:, :, 1, :].reshape(T, N2 // 2)


def interleave_gate_up(wg: torch.Tensor, wu: torch.Tensor) -> torch.Tensor:
    """[I,H] gate and up weights -> [2I,H] interleaved in blocks of IL_BLOCK rows."""
    I, H = wg.shape
    assert I % IL_BLOCK == 0
    w = torch.stack([wg.reshape(I // IL_BLOCK, IL_BLOCK, H), wu.reshape(I // IL_BLOCK, IL_BLOCK, H)], 1)
    return w.reshape(2 * I, H).contiguous()


def linear(x: torch.Tensor, w: torch.Tensor, bias=None, residual=None, act=None, out_dtype=None) -> torch.Tensor:
    """y = act(x @ w.T + bias) (+ residual).  Accumulates in fp32."""
    y = _f(x) @ _f(w).t()
    if bias is not None:
        y = y + _f(bias)
    if act == "gelu":
        y = gelu(y)
    elif act == "swiglu_il":
        g, u = deinterleave_gate_up(y)
        y = F.silu(g) * u
    elif act is not None:
        raise ValueError(act)
    if residual is not None:
        y = y + _f(residual)
    return y.to(out_dtype or x.dtype)


def rope_tables(max_pos: int, rot_dim: int, theta: float, device=None):
    """fp32 cos/sin tables ``[max_pos, rot_dim/2]`` (HF default rope recipe)."""
    inv_freq = 1.0 / (theta ** (torch.arange(0, rot_dim, 2, dtype=torch.int64).float() / rot_dim))
    pos = torch.arange(max_pos, dtype=torch.int64).float()
    freqs = torch.outer(pos, inv_freq)
    return freqs.cos().to(device), freqs.sin().to(device)


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, rot_dim: int) -> torch.Tensor:
    """x: [..., S, D] fp32; cos/sin: [S, rot_dim/2]; rotate_half on the first rot_dim dims."""
    half = rot_dim // 2
    x1 = x[..., :half]
    x2 = x[..., half:rot_dim]
    c, s = cos, sin
    r1 = x1 * c - x2 * s
    r2 = x2 * c + x1 * s
    return torch.cat([r1, r2, x[..., rot_dim:]], -1)


def s_pad(S: int) -> int:
    return ((S + 63) // 64) * 64


def qkv_rope(x, wqkv, bqkv, cos, sin, B, S, Hq, Hkv, D, rot_dim, q_scale):
    """Fused QKV projection + bias + RoPE + head-major scatter (+ q scaling)."""
    y = linear(x, wqkv, bqkv, out_dtype=torch.float32)       # [T, (Hq+2Hkv)*D]
    y = y.reshape(B, S, Hq + 2 * Hkv, D).permute(0, 2, 1, 3)  # [B, Htot, S, D]
    q, k, v = y[:, :Hq], y[:, Hq:Hq + Hkv], y[:, Hq + Hkv:]
    c, s_ = cos[:S], sin[:S]
    q = apply_rope(q, c, s_, rot_dim) * q_scale
    k = apply_rope(k, c, s_, rot_dim)
    dt = x.dtype
    vt = torch.zeros(B, Hkv, D, s_pad(S), dtype=dt, device=x.device)
    vt[..., :S] = v.transpose(-1, -2).to(dt)
    return q.to(dt).contiguous(), k.to(dt).contiguous(), vt


def attention_probs(q, k, S):
    """Full causal softmax probabilities [B, Hq, S, S] in fp32 (GQA expanded)."""
    B, Hq = q.shape[:2]
    Hkv = k.shape[1]
    kk = _f(k).repeat_interleave(Hq // Hkv, dim=1)
    sc = _f(q) @ kk.transpose(-1, -2)
    mask = torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1)
    sc = sc.masked_fill(mask, float("-inf"))
    return torch.softmax(sc, -1)


def attention(q, k, vt, S, need_lse=False):
    """Causal GQA attention.  q is pre-scaled.  Returns (o [B*S, Hq*D], lse [B,Hq,S] or None)."""
    B, Hq, _, D = q.shape
    Hkv = k.shape[1]
    kk = _f(k).repeat_interleave(Hq // Hkv, dim=1)
    vv = _f(vt[..., :S]).transpose(-1, -2).repeat_interleave(Hq // Hkv, dim=1)
    sc = _f(q) @ kk.transpose(-1, -2)
    mask = torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1)
    sc = sc.masked_fill(mask, float("-inf"))
    lse = torch.logsumexp(sc, -1)
    p = torch.exp(sc - lse[..., None])
    o = p @ vv                                           # [B, Hq, S, D]
    o = o.permute(0, 2, 1, 3).reshape(B * S, Hq * D).to(q.dtype)
    return o, (lse if need_lse else None)


def attn_lastrow(q, k, S):
    """Per-head attention probabilities of the last query row: [B, Hq, S] fp32."""
    B, Hq, _, D = q.shape
    Hkv = k.shape[1]
    kk = _f(k).repeat_interleave(Hq // Hkv, dim=1)
    sc = (_f(q[:, :, S - 1:S]) @ kk.transpose(-1, -2))[:, :, 0]
    return torch.softmax(sc, -1)


def attn_colsum(q, k, lse, S):
    """Per-head column sums of the causal attention probabilities: [B, Hq, S] fp32."""
    B, Hq, _, D = q.shape
    Hkv = k.shape[1]
    kk = _f(k).repeat_interleave(Hq // Hkv, dim=1)
    sc = _f(q) @ kk.transpose(-1, -2)
    mask = torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1)
    p = torch.exp(sc - lse[..., None]).masked_fill(mask, 0.0)
    return p.sum(-2)


def head_nll(h, w, targets):
    """Fused final projection + cross entropy: per-row NLL (fp32) = lse(h @ w.T) - logit[target]."""
    logits = _f(h) @ _f(w).t()
    return torch.logsumexp(logits, -1) - logits.gather(1, targets.long().view(-1, 1)).squeeze(1)


# ---- fp32 GEMMs by split-fp16 MFMA ("h3", csrc/common.h) ---------------------------------------------------
# s x = hi + lo with hi = fp16(s x), lo = fp16(s x - hi) (s a power of two that keeps both planes in the fp16
# range); a GEMM over the K-concatenations
#   A' = [a_lo | a_hi | a_hi],  B' = [b_hi | b_lo | b_hi]
# sums hi_a hi_b + hi_a lo_b + lo_a hi_b = s_a s_b (a b) up to the dropped lo_a lo_b (2^-22 relative) and the
# residual rounding (2^-23): below the CPU fp32 GEMM's own error (tools/h3_error.py).  Weights are stored as B'
# [N, 3K] fp16; activations once per plane, [hi | lo] [R, 2K] fp16 (the GEMM's A loader reads block j of A' from
# plane H3_APLANES[j]); the epilogue multiplies by alpha = 1 / (s_a s_b).  A weight exact in fp16 after scaling
# (b_lo == 0, e.g. bf16 / fp16 checkpoint values) is stored as its single plane b_hi [N, K]: the GEMM over K' = 2K
# sums a_lo b_hi + a_hi b_hi (the kernel interleaves the two A planes against each B tile), the same result, its
# third product being exactly zero.
H3_APLANES = (1, 0, 0)
H3_BPLANES = (0, 1, 0)
H3_TOP = 15   # the scaled bound is at most 2^15: hi and lo stay below the fp16 maximum 65504 (< 2^16)


def h3_scale(bound: float) -> float:
    """Power-of-two s with s * bound <= 2^15 (largest such; 1 for a zero or non-finite bound)."""
    bound = float(bound)
    if not (bound > 0.0 and math.isfinite(bound)):
        return 1.0
    e = H3_TOP - math.ceil(math.log2(bound))
    return float(2.0 ** max(-100, min(100, e)))


def split2h(x: torch.Tensor, s: float) -> tuple[torch.Tensor, torch.Tensor]:
    xs = _f(x) * s
    hi = xs.to(torch.float16)
    lo = (xs - hi.float()).to(torch.float16)
    return hi, lo


def kv_plane_perm(S_pad: int) -> torch.Tensor:
    """Key order of the V^T h3 planes (gemm.hip kv_plane_pos): element index of key p within its row."""
    p = torch.arange(S_pad)
    k = p % 64
    return (p - k) + ((4 * (k >> 5) + ((k >> 2) & 3)) << 3) + (((k >> 4) & 1) << 2) + (k & 3)


def kv_planes(k: torch.Tensor, vt: torch.Tensor, sk: float, sv: float):
    """fp32 K [B, Hkv, S, D] / V^T [B, Hkv, D, S_pad] -> the scaled fp16 h3 planes the fp32 QKV GEMM writes for the
    plane-staged attention: kp [B, Hkv, 2, S, D], vp [B, Hkv, 2, D, S_pad] (keys in kv_plane_perm order)."""
    kh, kl = split2h(k, sk)
    vh, vl = split2h(vt, sv)
    vp = torch.stack([vh, vl], 2)
    out = torch.empty_like(vp)
    out[..., kv_plane_perm(vt.shape[-1])] = vp
    return torch.stack([kh, kl], 2).contiguous(), out.contiguous()


def h3_act(x: torch.Tensor, s: float) -> torch.Tensor:
    """fp32 [R, K] -> 2-plane h3 activation [R, 2K] fp16 = [hi | lo] of s x (what the fp32-mode kernels emit for
    GEMM inputs)."""
    return torch.cat(split2h(x, s), -1).contiguous()


def h3_expand(a3: torch.Tensor, terms: int = 3) -> torch.Tensor:
    """2-plane activation [R, 2K] -> the A' K-concatenation [R, terms K] the GEMM reads (H3_APLANES)."""
    K = a3.shape[-1] // 2
    return torch.cat([a3[..., i * K:(i + 1) * K] for i in H3_APLANES[:terms]], -1)


def h3_weight(w: torch.Tensor, two_term: bool = True) -> tuple[torch.Tensor, float]:
    """fp32 [N, K] nn.Linear weight -> (h3 weight B' [N, 3K] fp16, its scale s_w); the single plane hi [N, K] when
    the weight is exact in fp16 after scaling and ``two_term`` (the lo plane would be all zero)."""
    s = h3_scale(_f(w).abs().max().item())
    p = split2h(w, s)
    if two_term and not p[1].any():
        return p[0].contiguous(), s
    return torch.cat([p[i] for i in H3_BPLANES], -1).contiguous(), s


def h3_terms(a3: torch.Tensor, w3: torch.Tensor) -> int:
    """Products of the h3 GEMM of a3 [R, 2K] and w3: 3 for [N, 3K], 2 for a single-plane weight [N, K]."""
    K = a3.shape[-1] // 2
    if w3.shape[-1] not in (K, 3 * K):
        raise ValueError(f"h3 activation width {a3.shape[-1]} does not match the weight width {w3.shape[-1]}")
    return 3 if w3.shape[-1] == 3 * K else 2


def h3_to_f32(a3: torch.Tensor, s: float = 1.0) -> torch.Tensor:
    """Inverse of ``h3_act``: (hi + lo) / s (exact in fp32)."""
    K = a3.shape[-1] // 2
    return (a3[..., :K].float() + a3[..., K:].float()) / s


def h3w_to_f32(w3: torch.Tensor, s: float, K: int) -> torch.Tensor:
    """Inverse of ``h3_weight`` (K = the weight's input width): (hi + lo) / s, or hi / s for a two-term weight."""
    if w3.shape[-1] == K:
        return w3.float() / s
    return (w3[..., :K].float() + w3[..., K:2 * K].float()) / s


def h3_matmul(a3: torch.Tensor, w3: torch.Tensor, alpha: float) -> torch.Tensor:
    """What the h3 GEMM computes: alpha * (A' @ B'^T), fp16 x fp16 products (exact) accumulated in fp32."""
    if h3_terms(a3, w3) == 2:
        w3 = torch.cat([w3, w3], -1)
        return (h3_expand(a3, 2).float() @ w3.float().t()) * alpha
    return (h3_expand(a3, 3).float() @ w3.float().t()) * alpha


# ---- fused RMSNorm (GPU fast path) semantics -------------------------------------------------------
def row_ssq(x: torch.Tensor) -> torch.Tensor:
    """Per-row sum of squares in 64-column slabs: [T, H/64] fp32."""
    T, H = x.shape
    return _f(x).pow(2).reshape(T, H // 64, 64).sum(-1)


def rownorm_scale(ssq: torch.Tensor, K: int, eps: float) -> torch.Tensor:
    return torch.rsqrt(ssq.sum(-1) / K + eps)


def fold_norm_weight(w: torch.Tensor, norm_w: torch.Tensor) -> torch.Tensor:
    """W' = W diag(norm_w): rmsnorm(x) @ W^T == (x @ W'^T) * rsqrt(mean(x^2) + eps) (up to rounding)."""
    return (_f(w) * _f(norm_w).view(1, -1)).to(w.dtype)


# ---- AttnLRP relevance backward (csrc/lrp.hip) --------------------------------------------------------
def lrp_attn_bwd(q, k, v, o, dO, lse):
    """Uniform rule on Q K^T and A V, plain softmax gradient.  q [B,Hq,S,D] pre-scaled, k/v [B,Hkv,S,D],
    o/dO token-major [B*S, Hq*D], lse [B,Hq,S].  Returns (D [B,Hq,S], rel [B,Hq], dq [B,Hq,S,D],
    dk, dv [B,Hq,S,D]) in fp32: dq w.r.t. the pre-scaled q; dk/dv are per-q-head partials (the GQA group
    sum is part of ``lrp_rope_pack``)."""
    B, Hq, S, D = q.shape
    Hkv = k.shape[1]
    G = Hq // Hkv
    kk, vv = _f(k).repeat_interleave(G, 1), _f(v).repeat_interleave(G, 1)
    oh = _f(o).view(B, S, Hq, D).permute(0, 2, 1, 3)
    dOh = _f(dO).view(B, S, Hq, D).permute(0, 2, 1, 3)
    Dl = 0.5 * (oh * dOh).sum(-1)
    mask = torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1)
    p = torch.exp(_f(q) @ kk.transpose(-1, -2) - lse[..., None]).masked_fill(mask, 0.0)
    dA = 0.5 * dOh @ vv.transpose(-1, -2)
    dS = p * (dA - Dl[..., None])
    dq = 0.5 * dS @ kk
    dk = 0.5 * dS.transpose(-1, -2) @ _f(q)
    dv = 0.5 * p.transpose(-1, -2) @ dOh
    return Dl, Dl.sum(-1), dq, dk, dv


def rope_bwd(dx: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, rot_dim: int) -> torch.Tensor:
    """Transpose of ``apply_rope``: x1 = r1 c + r2 s, x2 = r2 c - r1 s."""
    half = rot_dim // 2
    r1, r2 = dx[..., :half], dx[..., half:rot_dim]
    return torch.cat([r1 * cos + r2 * sin, r2 * cos - r1 * sin, dx[..., rot_dim:]], -1)


def lrp_rope_pack(dq, dk, dv, cos, sin, B, S, Hq, Hkv, rot_dim, q_scale, dtype=torch.float32):
    """Inverse RoPE + q scale + GQA group sum of the dk/dv partials [B,Hq,S,D] (or dk/dv already summed,
    [B,Hkv,S,D]), scattered to token-major d[q|k|v] [B*S, (Hq+2Hkv)*D]."""
    c, s_ = cos[:S], sin[:S]
    G = Hq // Hkv
    if dk.shape[1] == Hq:   # per-q-head partials (else already the group sums [B, Hkv, S, D])
        dk = _f(dk).view(B, Hkv, G, S, -1).sum(2)
        dv = _f(dv).view(B, Hkv, G, S, -1).sum(2)
    dqp = rope_bwd(_f(dq) * q_scale, c, s_, rot_dim)
    dkp = rope_bwd(_f(dk), c, s_, rot_dim)
    y = torch.cat([dqp, dkp, _f(dv)], 1)                     # [B, Ht, S, D]
    return y.permute(0, 2, 1, 3).reshape(B * S, -1).to(dtype)


def swiglu_il(gu: torch.Tensor) -> torch.Tensor:
    g, u = deinterleave_gate_up(_f(gu))
    return (F.silu(g) * u).to(gu.dtype)


def lrp_swiglu_bwd(dm: torch.Tensor, gu: torch.Tensor) -> torch.Tensor:
    """dg = 0.5 dm u sigmoid(g), du = 0.5 dm silu(g), re-interleaved like ``gu``."""
    g, u = deinterleave_gate_up(_f(gu))
    sg = torch.sigmoid(g)
    dg, du = 0.5 * _f(dm) * u * sg, 0.5 * _f(dm) * g * sg
    T, I = dg.shape
    out = torch.stack([dg.reshape(T, I // IL_BLOCK, IL_BLOCK), du.reshape(T, I // IL_BLOCK, IL_BLOCK)], 2)
    return out.reshape(T, 2 * I).to(gu.dtype)


def lrp_gelu_bwd(dy: torch.Tensor, a: torch.Tensor) -> torch.Tensor:
    af = _f(a)
    ratio = torch.where(af.abs() > 1e-6, gelu(af) / torch.where(af.abs() > 1e-6, af, torch.ones_like(af)),
                        torch.full_like(af, 0.5))
    return (_f(dy) * ratio).to(dy.dtype)


def ln_rstd(x: torch.Tensor, eps: float) -> torch.Tensor:
    xf = _f(x)
    return torch.rsqrt((xf - xf.mean(-1, keepdim=True)).pow(2).mean(-1) + eps)


def lrp_ln_bwd(dy1, rs1, w1, dy2, rs2, w2, resid):
    """resid + sum over the (one or two) LayerNorms of (gc - mean(gc)), gc = dy * rstd * w."""
    def one(dy, rs, w):
        gc = _f(dy) * rs.view(-1, 1) * _f(w).view(1, -1)
        return gc - gc.mean(-1, keepdim=True)
    out = _f(resid) + one(dy1, rs1, w1)
    if dy2 is not None:
        out = out + one(dy2, rs2, w2)
    return out.to(resid.dtype)


# ---- fp32 AttnLRP backward on h3 GEMMs (csrc/lrp_f32.hip) ---------------------------------------------------
def h3_row_scales(x: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """Per-row power-of-two scale s = 2^(15 - E) for max |row| = m 2^E, m in [0.5, 1) (s * max < 2^15; 1 for a zero
    or non-finite row) and its inverse.  [R] each."""
    mx = _f(x).abs().amax(-1)
    ok = (mx > 0) & torch.isfinite(mx)
    _, e = torch.frexp(torch.where(ok, mx, torch.ones_like(mx)))
    sh = torch.where(ok, 15 - e, torch.zeros_like(e)).to(torch.float32)
    return torch.exp2(sh), torch.exp2(-sh)


def split_h3_dyn(x: torch.Tensor, post: torch.Tensor | None = None) -> tuple[torch.Tensor, torch.Tensor]:
    """fp32 rows [R, K] -> (h3 activation [R, 2K] of s_r x_r, rinv [R] = post / s_r): the GEMM input of a gradient,
    whose per-row epilogue scale ``rinv`` undoes s exactly."""
    s, inv = h3_row_scales(x)
    xs = _f(x) * s.view(-1, 1)
    hi = xs.to(torch.float16)
    lo = (xs - hi.float()).to(torch.float16)
    rinv = inv if post is None else inv * _f(post)
    return torch.cat([hi, lo], -1).contiguous(), rinv


def lrp_swiglu_bwd_h3(dm, gu, post=None):
    """``lrp_swiglu_bwd`` in fp32, as a per-row-scaled h3 activation (csrc/lrp_f32.hip)."""
    return split_h3_dyn(lrp_swiglu_bwd(_f(dm), _f(gu)), post)


def bound_planes(y: torch.Tensor, bnd_a, bnd_b, bnd_c: float):
    """(h3 activation [M, 2N] of s_m y_m, 1 / s_m) with s_m = 2^(15 - E) for the bound 2^15 (bnd_a[m] + bnd_b[m]
    bnd_c) = f 2^E, f in [0.5, 1) (gemm.hip GemmArgs::planes)."""
    bound = 32768.0 * (_f(bnd_a) + _f(bnd_b) * float(bnd_c))
    _, e = torch.frexp(bound)
    s = torch.exp2((15 - e).to(torch.float32))
    ys = _f(y) * s.view(-1, 1)
    hi = ys.to(torch.float16)
    lo = (ys - hi.float()).to(torch.float16)
    return torch.cat([hi, lo], -1).contiguous(), 1.0 / s


def np_planes(y: torch.Tensor, g: torch.Tensor, rstd_in: torch.Tensor, g_max: float, prod_bound: float):
    """The fused-RMSNorm producer outputs of gemm.hip EPI_F32_RESID_NP besides C = y: (planes [M, 2N] = h3 of
    p_m (y_m * g), prinv [M] = 1 / p_m, ssq [M, N / 112] row sum-of-squares partials of y), with p_m = 2^(14 - E) for
    the bound u_m = g_max (sqrt(N) / rstd_in[m] + prod_bound) = f 2^E on |y_m * g| (fp32 arithmetic as the kernel's).
    The consumer GEMM then takes rscale[m] = rsqrt(sum ssq[m] / N + eps) * prinv[m] (``row_rscale_mul``)."""
    M, N = y.shape
    yf = _f(y)
    u = torch.tensor(float(g_max), dtype=torch.float32) * (
        torch.tensor(math.sqrt(N), dtype=torch.float32) / _f(rstd_in) + torch.tensor(float(prod_bound), dtype=torch.float32))
    _, e = torch.frexp(u)
    p = torch.exp2((14 - e).to(torch.float32))
    ys = (yf * _f(g).view(1, -1)) * p.view(-1, 1)
    hi = ys.to(torch.float16)
    lo = (ys - hi.float()).to(torch.float16)
    ssq = yf.pow(2).reshape(M, N // 112, 112).sum(-1) if N % 112 == 0 else yf.pow(2).sum(-1, keepdim=True)
    return torch.cat([hi, lo], -1).contiguous(), 1.0 / p, ssq


def row_rscale_mul(ssq: torch.Tensor, mul: torch.Tensor, K: int, eps: float) -> torch.Tensor:
    return torch.rsqrt(_f(ssq).sum(-1) / K + eps) * _f(mul)


def h3_unit(x: torch.Tensor) -> torch.Tensor:
    """fp32 [R, K] -> the 2-plane h3 activation [R, 2K] at scale 1 (the caller bounds |x| below 2^15)."""
    hi = _f(x).to(torch.float16)
    lo = (_f(x) - hi.float()).to(torch.float16)
    return torch.cat([hi, lo], -1).contiguous()


def linear_h3_lrp_swiglu(a3, w3, alpha, gu, c0, rinv, post=None):
    """``lrp_swiglu_bwd_h3`` of the dm GEMM's product with a bound-derived scale instead of the row max: the rule on
    d = c0 alpha (a3 . w3^T) (the GEMM input's own row scale not undone) as unit-scale h3 planes, and the row scale
    rinv post / c0 that undoes both (gemm.hip EPI_H3_LRP_SWIGLU)."""
    d = h3_matmul(a3, w3, alpha * c0)
    rs = rinv / c0 if post is None else rinv * _f(post) / c0
    return h3_unit(lrp_swiglu_bwd(d, _f(gu))), rs


def lrp_gelu_bwd_h3(dy, a):
    return split_h3_dyn(lrp_gelu_bwd(_f(dy), _f(a)))


def lrp_rope_pack_h3(dq, dk, dv, cos, sin, B, S, Hq, Hkv, rot_dim, q_scale, post=None):
    return split_h3_dyn(lrp_rope_pack(dq, dk, dv, cos, sin, B, S, Hq, Hkv, rot_dim, q_scale), post)


def act_h3(x: torch.Tensor, act: str, s: float) -> torch.Tensor:
    """SwiGLU (interleaved gate|up [T, 2I] -> [T, I]) or GELU of fp32 pre-activations, as the h3 activation at s."""
    y = swiglu_il(_f(x)) if act == "swiglu_il" else gelu(_f(x))
    return h3_act(y, s)


def row_rstd(x: torch.Tensor, eps: float, center: bool = False) -> torch.Tensor:
    xf = _f(x)
    if center:
        xf = xf - xf.mean(-1, keepdim=True)
    return torch.rsqrt(xf.pow(2).mean(-1) + eps)


def group_absprod(x: torch.Tensor, dx: torch.Tensor, B: int, S: int, group: int = 64) -> torch.Tensor:
    """[B, H / group]: sum over each window's tokens and the group's channels of |x dx|."""
    H = x.shape[-1]
    return (_f(x) * _f(dx)).abs().view(B, S, H // group, group).sum((1, 3))


def group_sens(x: torch.Tensor, dx: torch.Tensor, B: int, S: int, group: int = 64) -> torch.Tensor:
    """[B, H / group]: the quantization sensitivity of each channel group, sum over the window's tokens t of
    max_c |x_tc|^2 * sum_c dx_tc^2 (c over the group): a max-abs quantizer of step max_c |x_tc| / qmax moves the
    first-order output by a zero-mean error of variance step^2 / 12 * sum_c dx_tc^2 (codec.wire.allocate_group_bits)."""
    H = x.shape[-1]
    xg, dg = _f(x).view(B, S, H // group, group), _f(dx).view(B, S, H // group, group)
    return (xg.abs().amax(-1).pow(2) * dg.pow(2).sum(-1)).sum(1)
