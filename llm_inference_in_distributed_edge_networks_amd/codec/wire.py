"""Wire format of a boundary message and the encode/decode entry points.

Message for a micro-batch of ``B`` windows of ``S`` tokens, hidden size ``H``,
``k`` lo-class tokens per window (all sections 16-byte aligned)::

    header   32 B   int32[8] = magic 'EDGB', version, codec id, B, S, H, k (-1: variable), hi-row format
    mask     B * MW uint32        bit j of window b set <=> token j is in the lo class (MW = 2*ceil(S/64))
    scales   fp32                 per token [B*S] | per window [B] | per channel [B*H]
    hi rows  B*(S-k) rows         token order within each window
    lo rows  B*k rows             token order within each window

The size depends only on (codec, B, S, H, k, native dtype), so sender and
receiver agree on it without a handshake and the receiver can post its
``irecv`` before the sender has produced anything.

Selection.  ``"ratio"`` (the reference): the ``k = int(ratio*S)`` least important tokens of
every window.  ``"top_rho"`` (Pythia ``'upto ratio'``, ``pythia_model.py:92-112``): each
window keeps the shortest prefix of its tokens by descending importance whose mass reaches
``1 - ratio`` and quantizes the rest, so k varies per window.  That message carries
``k`` per window after the mask and stores the lo rows first and the hi rows right after
the ``sum k`` lo rows (compact); its buffer (``Layout.total``) has capacity for any k and
``payload_bytes(sum_k)`` is what a link would carry.

``encode``/``decode`` run the gfx950 kernels of ``csrc/codec.hip`` for CUDA
tensors and a bit-identical PyTorch implementation for CPU tensors.
"""
from __future__ import annotations

from dataclasses import dataclass
from functools import lru_cache

import torch

from ..ops._native import call, ptr, stream

MAGIC = 0x45444742
VERSION = 1
FMT_BF16, FMT_INT8, FMT_INT4, FMT_INT2, FMT_F32, FMT_MXFP4, FMT_MXFP8, FMT_GRP = 0, 1, 2, 3, 4, 5, 6, 7
MX_FORMATS = (FMT_MXFP4, FMT_MXFP8)
SC_TOKEN, SC_WINDOW, SC_CHANNEL, SC_NONE = 0, 1, 2, 3
CH_MAXABS, CH_MEAN = 0, 1
NATIVE = -1  # "keep in the activation dtype" (bf16 on GPU, fp32 in the CPU reference mode)


@dataclass(frozen=True)
class CodecSpec:
    name: str
    cid: int
    hi_fmt: int
    lo_fmt: int
    scale_mode: int
    qmax_hi: int = 0
    qmax_lo: int = 0
    ch_kind: int = CH_MAXABS
    uses_ratio: bool = True      # lo class = int(ratio*S) least important tokens
    needs_importance: bool = True
    plan: tuple | None = None    # FMT_GRP rows: bits (GROUP_BITS) of every 64-channel group (with_plan)


CODECS = {c.name: c for c in [
    CodecSpec("passthrough", 0, NATIVE, NATIVE, SC_NONE, uses_ratio=False, needs_importance=False),
    CodecSpec("ref_int4_global", 1, NATIVE, FMT_INT4, SC_WINDOW, 0, 7),
    CodecSpec("int4_token", 2, NATIVE, FMT_INT4, SC_TOKEN, 0, 7),
    CodecSpec("int8_token", 3, FMT_INT8, FMT_INT8, SC_TOKEN, 127, 127, uses_ratio=False, needs_importance=False),
    CodecSpec("mixed_int4_int8", 4, FMT_INT8, FMT_INT4, SC_TOKEN, 127, 7),
    CodecSpec("mixed_int2_int8", 5, FMT_INT8, FMT_INT2, SC_TOKEN, 127, 1),
    CodecSpec("channel_8", 6, FMT_INT8, FMT_INT8, SC_CHANNEL, 127, 127, CH_MAXABS, False, False),
    CodecSpec("channel_4", 7, FMT_INT4, FMT_INT4, SC_CHANNEL, 7, 7, CH_MAXABS, False, False),
    CodecSpec("channel_1_mean", 8, FMT_INT2, FMT_INT2, SC_CHANNEL, 1, 1, CH_MEAN, False, False),
    CodecSpec("channel_1_max", 9, FMT_INT2, FMT_INT2, SC_CHANNEL, 1, 1, CH_MAXABS, False, False),
    CodecSpec("int8_token_keep", 10, NATIVE, FMT_INT8, SC_TOKEN, 0, 127),
    # OCP microscaling (32-channel blocks, E8M0 scales inline in the row; gfx950 scaled converts)
    CodecSpec("mxfp4", 11, FMT_MXFP4, FMT_MXFP4, SC_NONE, uses_ratio=False, needs_importance=False),
    CodecSpec("mxfp8", 12, FMT_MXFP8, FMT_MXFP8, SC_NONE, uses_ratio=False, needs_importance=False),
    CodecSpec("mixed_mxfp4_mxfp8", 13, FMT_MXFP8, FMT_MXFP4, SC_NONE),
    CodecSpec("mxfp4_keep", 14, NATIVE, FMT_MXFP4, SC_NONE),
    # head-group rows (FMT_GRP): every 64-channel group (one head's width) has its own bit width and max-abs scale;
    # the widths come from the relevance of the boundary's channel groups (group_bits / allocate_group_bits)
    CodecSpec("rgroup", 15, FMT_GRP, FMT_GRP, SC_NONE, uses_ratio=False, needs_importance=False),
    CodecSpec("mixed_rgroup_int8", 16, FMT_INT8, FMT_GRP, SC_TOKEN, 127, 0),
]}
GROUP = 64                  # channels per group of FMT_GRP rows
GROUP_BITS = (2, 3, 4, 5, 6, 8)


def needs_plan(spec: CodecSpec) -> bool:
    return FMT_GRP in (spec.hi_fmt, spec.lo_fmt)


def with_plan(spec: CodecSpec, plan) -> CodecSpec:
    """The codec with a group bit plan (one entry per 64-channel group, each in GROUP_BITS)."""
    from dataclasses import replace
    plan = tuple(int(b) for b in plan)
    if any(b not in GROUP_BITS for b in plan):
        raise ValueError(f"group bits must be in {GROUP_BITS}, got {plan}")
    return replace(spec, plan=plan)


def boundary_group_relevance(table, boundary: int, groups: int) -> list:
    """The channel-group relevance of the tensor crossing the boundary after layer ``boundary`` from a
    [layers][groups] table of the relevance ENTERING each layer (``channel_group_relevance.json``): row
    ``boundary + 1``.  After the last layer the tensor is the final norm's input, which the table does not hold;
    its last row (the stream entering the last layer) stands in.  No table: every group equal.  A dict table
    ``{"relevance": ..., "sensitivity": ...}`` (``load_group_tables``) gives its relevance."""
    if isinstance(table, dict):
        table = table.get("relevance")
    if table is None:
        return [1.0] * groups
    t = torch.as_tensor(table, dtype=torch.float32)
    return [float(v) for v in t[min(boundary + 1, t.shape[0] - 1)]]


def boundary_group_plan(table, boundary: int, groups: int, avg_bits: float = 4.0) -> tuple:
    """The bit plan of the head-group codec at the boundary after layer ``boundary``.

    ``table`` = ``{"relevance": [layers][G], "sensitivity": [layers][G]}`` (``load_group_tables``): the MSE
    allocation over the groups' quantization sensitivity when it is there (``allocate_group_bits(model="mse")``),
    else the first-order allocation over the LRP relevance (``model="linear"``, the round-3 allocator); a plain
    [layers][G] list is a relevance table; None: the uniform plan (every group at ``avg_bits`` when that is a
    width, else the MSE allocation of equal weights: the nearest widths, as evenly as the budget allows)."""
    if table is None:
        return allocate_group_bits([1.0] * groups, avg_bits, model="mse")
    if isinstance(table, dict) and table.get("sensitivity") is not None:
        w = boundary_group_relevance({"relevance": table["sensitivity"]}, boundary, groups)
        return allocate_group_bits(w, avg_bits, model="mse")
    return allocate_group_bits(boundary_group_relevance(table, boundary, groups), avg_bits, model="linear")


def _qmax(bits: int) -> int:
    return (1 << (bits - 1)) - 1


def allocate_group_bits(weights, avg_bits: float = 4.0, model: str = "mse", widths=GROUP_BITS) -> tuple:
    """Bit allocation over the 64-channel groups of a boundary: every group starts at the narrowest width and the
    budget ``avg_bits * G`` bits goes, one step up the width ladder at a time, to the step with the largest error
    reduction per bit.  Error models of a group g quantized at b bits (max-abs scale, step amax / qmax_b):

    * ``"mse"``: the expected squared first-order output change, W_g / (12 qmax_b^2) with W_g the group's
      quantization sensitivity sum_t max_c |x_tc|^2 sum_c dx_tc^2 (``ops.reference.group_sens``: a rounding error
      uniform in +-step/2 per channel, independent across channels, propagated through the gradient dx).  The
      error falls 4-9x per added bit, so a group gets a wider code only where its sensitivity is that much larger
      than the others' - the outlier-heavy groups;
    * ``"linear"``: R_g / qmax_b with R_g the LRP relevance sum |x dx| (the round-3 allocator: error ~ sum |dx|
      step / 2), only on the widths 2 / 4 / 8.

    The error reductions per bit fall along the ladder (convex), so the greedy allocation is optimal for the
    model.  Equal weights give the uniform plan."""
    w = [max(float(r), 0.0) for r in weights]
    G = len(w)
    if not any(w):
        w = [1.0] * G
    if model == "linear":
        ladder = (2, 4, 8)
        err = {b: 1.0 / _qmax(b) for b in ladder}
    elif model == "mse":
        ladder = tuple(sorted(widths))
        err = {b: 1.0 / _qmax(b) ** 2 for b in ladder}
    else:
        raise ValueError(f"unknown allocation model {model!r} (mse | linear)")
    nxt = {ladder[i]: ladder[i + 1] for i in range(len(ladder) - 1)}
    bits = [ladder[0]] * G
    budget = int(round(avg_bits * G)) - ladder[0] * G
    while budget > 0:
        best, best_gain = -1, 0.0
        for g in range(G):
            b = bits[g]
            if b not in nxt:
                continue
            nb = nxt[b]
            cost = nb - b
            if cost > budget:
                continue
            gain = w[g] * (err[b] - err[nb]) / cost
            if gain > best_gain or (gain == best_gain and best >= 0 and w[g] > w[best]):
                best, best_gain = g, gain
        if best < 0:
            break
        budget -= nxt[bits[best]] - bits[best]
        bits[best] = nxt[bits[best]]
    return tuple(bits)


def load_group_tables(relevance_path: str):
    """``channel_group_relevance.json`` and, when the relevance pass wrote it beside, the sensitivity table
    ``channel_group_sensitivity.json`` -> {"relevance": tensor, "sensitivity": tensor or None}."""
    import json
    import os
    with open(relevance_path) as f:
        rel = torch.tensor(json.load(f), dtype=torch.float32)
    sp = os.path.join(os.path.dirname(os.path.abspath(relevance_path)), "channel_group_sensitivity.json")
    sens = None
    if os.path.exists(sp):
        with open(sp) as f:
            sens = torch.tensor(json.load(f), dtype=torch.float32)
    return {"relevance": rel, "sensitivity": sens}


def get_codec(name: str) -> CodecSpec:
    if name not in CODECS:
        raise KeyError(f"unknown codec {name!r}; known: {sorted(CODECS)}")
    return CODECS[name]


def _a16(n: int) -> int:
    return (n + 15) // 16 * 16


def _row_bytes(fmt: int, H: int, plan=None) -> int:
    if fmt == FMT_GRP:   # codes of every group (8 * bits bytes), then one fp32 scale per group
        return sum(8 * b for b in plan) + 4 * len(plan)
    return {FMT_BF16: 2 * H, FMT_INT8: H, FMT_INT4: H // 2, FMT_INT2: H // 4, FMT_F32: 4 * H,
            FMT_MXFP4: H // 2 + H // 32, FMT_MXFP8: H + H // 32}[fmt]


@dataclass(frozen=True)
class Layout:
    B: int
    S: int
    H: int
    k: int            # lo tokens per window (-1: variable, see kvar)
    mw: int
    hi_fmt: int
    lo_fmt: int
    off_mask: int
    off_scale: int
    off_hi: int       # -1 when kvar (the hi section follows the sum-k lo rows)
    off_lo: int
    total: int        # bytes of the message buffer (the capacity when kvar)
    kvar: bool = False
    off_kvec: int = -1
    plan: tuple | None = None   # FMT_GRP group bits (also stored in the message at off_plan, one byte each)
    off_plan: int = -1

    def row_bytes(self, fmt: int) -> int:
        return _row_bytes(fmt, self.H, self.plan)

    @property
    def payload_bytes_per_token(self) -> float:
        return self.total / (self.B * self.S)

    def payload_bytes(self, k_total: int | None = None) -> int:
        """Bytes of the message proper: ``total`` for fixed k; for variable k with ``k_total`` lo rows in all."""
        if not self.kvar:
            return self.total
        return self.off_lo + _a16(k_total * self.row_bytes(self.lo_fmt)) + \
            (self.B * self.S - k_total) * self.row_bytes(self.hi_fmt)

    def hi_offset(self, k_total: int) -> int:
        return self.off_hi if not self.kvar else self.off_lo + _a16(k_total * self.row_bytes(self.lo_fmt))


def native_fmt(dtype: torch.dtype) -> int:
    if dtype == torch.bfloat16:
        return FMT_BF16
    if dtype == torch.float32:
        return FMT_F32
    raise TypeError(f"unsupported activation dtype {dtype}")


def num_lo(spec: CodecSpec, ratio: float, S: int) -> int:
    """Reference truncation: ``int(ratio * S)`` (qwen_layer_wise.py:57)."""
    if not spec.uses_ratio:
        return 0
    return max(0, min(S, int(ratio * S)))


@lru_cache(maxsize=256)
def layout(spec: CodecSpec, B: int, S: int, H: int, k: int, dtype: torch.dtype = torch.bfloat16,
           kvar: bool = False) -> Layout:
    if H % 32:
        raise ValueError("hidden size must be a multiple of 32 for the packed formats")
    nf = native_fmt(dtype)
    hi = nf if spec.hi_fmt == NATIVE else spec.hi_fmt
    lo = nf if spec.lo_fmt == NATIVE else spec.lo_fmt
    plan = None
    if FMT_GRP in (hi, lo):
        if H % GROUP:
            raise ValueError(f"head-group rows need a hidden size multiple of {GROUP}")
        plan = spec.plan if spec.plan is not None else (4,) * (H // GROUP)
        if len(plan) != H // GROUP:
            raise ValueError(f"group plan has {len(plan)} entries, hidden size {H} has {H // GROUP} groups")
    rb = lambda f: _row_bytes(f, H, plan)  # noqa: E731
    mw = 2 * ((S + 63) // 64)
    off_mask = 32
    n_scale = {SC_TOKEN: B * S, SC_WINDOW: B, SC_CHANNEL: B * H, SC_NONE: 0}[spec.scale_mode]
    # the group plan section (one byte per group) follows the mask (and the k vector)
    plan_bytes = _a16(len(plan)) if plan is not None else 0
    if kvar:
        off_kvec = off_mask + _a16(B * mw * 4)
        off_plan = off_kvec + _a16(B * 4) if plan is not None else -1
        off_scale = off_kvec + _a16(B * 4) + plan_bytes
        off_lo = off_scale + _a16(n_scale * 4)
        total = off_lo + _a16(B * S * max(rb(hi), rb(lo))) + 16
        return Layout(B, S, H, -1, mw, hi, lo, off_mask, off_scale, -1, off_lo, total, True, off_kvec, plan, off_plan)
    off_plan = off_mask + _a16(B * mw * 4) if plan is not None else -1
    off_scale = off_mask + _a16(B * mw * 4) + plan_bytes
    off_hi = off_scale + _a16(n_scale * 4)
    off_lo = off_hi + _a16(B * (S - k) * rb(hi))
    total = off_lo + _a16(B * k * rb(lo))
    return Layout(B, S, H, k, mw, hi, lo, off_mask, off_scale, off_hi, off_lo, total, False, -1, plan, off_plan)


def message_bytes(spec: CodecSpec, B: int, S: int, H: int, ratio: float, dtype=torch.bfloat16) -> int:
    return layout(spec, B, S, H, num_lo(spec, ratio, S), dtype).total


# --------------------------------------------------------------------------------------------
# CPU (reference) implementation
def _mask_words(lo: torch.Tensor, mw: int) -> torch.Tensor:
    """bool [B, S] -> int32 [B, mw] little-endian bit words."""
    B, S = lo.shape
    bits = torch.zeros(B, mw * 32, dtype=torch.int64)
    bits[:, :S] = lo.to(torch.int64)
    w = (bits.view(B, mw, 32) << torch.arange(32, dtype=torch.int64)).sum(-1)
    w = torch.where(w >= 2 ** 31, w - 2 ** 32, w)
    return w.to(torch.int32)


def _words_to_mask(words: torch.Tensor, S: int) -> torch.Tensor:
    w = words.to(torch.int64) & 0xFFFFFFFF
    bits = (w.unsqueeze(-1) >> torch.arange(32, dtype=torch.int64)) & 1
    return bits.reshape(words.shape[0], -1)[:, :S].bool()


def _canon(imp: torch.Tensor) -> torch.Tensor:
    v = imp.float()
    return torch.where(v == 0, torch.zeros_like(v), v)   # -0 == +0 (the kernel's key canonicalisation)


def select_mask(imp: torch.Tensor, k) -> torch.Tensor:
    """bool [B, S]: the k least important tokens (ascending, ties by position, NaN last) of each window; ``k`` an
    int or a per-window sequence."""
    B, S = imp.shape
    ks = torch.as_tensor(k, dtype=torch.int64).reshape(-1).expand(B) if not isinstance(k, int) else \
        torch.full((B,), k, dtype=torch.int64)
    order = torch.sort(_canon(imp).cpu(), dim=1, stable=True).indices
    pos = torch.arange(S).view(1, S).expand(B, S)
    lo = torch.zeros(B, S, dtype=torch.bool)
    lo.scatter_(1, order, pos < ks.view(B, 1).clamp(0, S))
    return lo.to(imp.device)


def top_rho_k(imp: torch.Tensor, mass: float) -> torch.Tensor:
    """Per-window lo count of top-rho selection: keep the shortest descending-importance prefix whose mass reaches
    ``mass`` (keep = first i with sum_{j<i} desc_j >= mass; mass <= 0 keeps nothing), quantize the rest.  [B] int64.
    Descending order = the ascending stable order reversed (as csrc/codec.hip)."""
    B, S = imp.shape
    asc = torch.sort(_canon(imp).cpu(), dim=1, stable=True).values
    desc = asc.flip(1).double()
    excl = torch.cumsum(desc, 1) - desc
    ge = excl >= mass
    keep = torch.where(ge.any(1), ge.to(torch.int64).argmax(1), torch.full((B,), S, dtype=torch.int64))
    return S - keep


def _qcodes(x: torch.Tensor, spec: CodecSpec, is_lo: bool, scale_row, ch_scale) -> torch.Tensor:
    """Quantize fp32 rows [n, H] -> int codes, exactly as csrc/codec.hip does."""
    qmax = spec.qmax_lo if is_lo else spec.qmax_hi
    if spec.scale_mode == SC_TOKEN:
        inv = torch.where(scale_row > 0, 1.0 / torch.where(scale_row > 0, scale_row, torch.ones_like(scale_row)),
                          torch.zeros_like(scale_row))
        return torch.round(x * inv[:, None]).clamp(-qmax, qmax)
    if spec.scale_mode == SC_WINDOW:
        m = scale_row  # [n] (window max broadcast per row)
        safe = torch.where(m > 0, m, torch.ones_like(m))
        t = torch.round((x / safe[:, None] * float(qmax)).clamp(-(qmax + 1), qmax))
        return torch.where(m[:, None] > 0, t, torch.zeros_like(t))
    sc = ch_scale  # [n, H]
    if spec.ch_kind == CH_MEAN or qmax == 1:
        safe = torch.where(sc != 0, sc, torch.ones_like(sc))
        t = torch.round(x / safe).clamp(-1, 1)
        return torch.where(sc != 0, t, torch.zeros_like(t))
    safe = torch.where(sc > 0, sc, torch.ones_like(sc))
    t = torch.round(x / safe * float(qmax))
    return torch.where(sc > 0, t, torch.zeros_like(t))


def _pack_rows(q: torch.Tensor, fmt: int) -> torch.Tensor:
    n, H = q.shape
    qi = q.to(torch.int64)
    if fmt == FMT_INT8:
        return (qi & 255).to(torch.uint8).reshape(-1)
    if fmt == FMT_INT4:
        p = qi.reshape(n, H // 2, 2) & 15
        return (p[..., 0] | (p[..., 1] << 4)).to(torch.uint8).reshape(-1)
    if fmt == FMT_INT2:
        p = qi.reshape(n, H // 4, 4) & 3
        return (p[..., 0] | (p[..., 1] << 2) | (p[..., 2] << 4) | (p[..., 3] << 6)).to(torch.uint8).reshape(-1)
    raise ValueError(fmt)


def _unpack_rows(b: torch.Tensor, fmt: int, n: int, H: int) -> torch.Tensor:
    u = b.to(torch.int64)
    if fmt == FMT_INT8:
        v = u.reshape(n, H)
        return torch.where(v >= 128, v - 256, v).float()
    if fmt == FMT_INT4:
        u = u.reshape(n, H // 2)
        p = torch.stack([u & 15, (u >> 4) & 15], -1).reshape(n, H)
        return torch.where(p >= 8, p - 16, p).float()
    if fmt == FMT_INT2:
        u = u.reshape(n, H // 4)
        p = torch.stack([(u >> (2 * e)) & 3 for e in range(4)], -1).reshape(n, H)
        return torch.where(p >= 2, p - 4, p).float()
    raise ValueError(fmt)


def _dequant(q: torch.Tensor, spec: CodecSpec, is_lo: bool, scale_row, ch_scale) -> torch.Tensor:
    qmax = spec.qmax_lo if is_lo else spec.qmax_hi
    if spec.scale_mode == SC_TOKEN:
        return q * scale_row[:, None]
    if spec.scale_mode == SC_WINDOW:
        return q / float(qmax) * scale_row[:, None]
    if spec.ch_kind == CH_MEAN or qmax == 1:
        return q * ch_scale
    return q * ch_scale / float(qmax)


# ---- OCP microscaling rows (csrc/codec.hip mx_pack8 / mx_unpack8) ----------------------------------------------
_FP4_GRID = torch.tensor([0.0, 0.5, 1.0, 1.5, 2.0, 3.0, 4.0, 6.0])


def _fp4_codes(v: torch.Tensor) -> torch.Tensor:
    """E2M1 codes of v (round to nearest, ties to even code, saturating at 6), sign in bit 3 - kept on values that
    round to zero (-0, code 8), as the gfx950 scaled convert does."""
    a = v.abs()
    # thresholds between grid points; a tie goes to the even code (0, 2, 4, 6)
    c = torch.zeros_like(a, dtype=torch.int64)
    for lo, hi_excl, code in ((0.25, True, 1), (0.75, False, 2), (1.25, True, 3), (1.75, False, 4), (2.5, True, 5),
                              (3.5, False, 6), (5.0, True, 7)):
        c = torch.where(a > lo if hi_excl else a >= lo, torch.full_like(c, code), c)
    return c | torch.signbit(v).to(torch.int64) << 3


def _mx_exp(am: torch.Tensor, emax: int) -> torch.Tensor:
    """E8M0 scale byte: clamp(floor(log2 amax) - emax + 127, 0, 254); amax 0 / denormal -> exponent -127."""
    bits = am.float().contiguous().view(torch.int32).to(torch.int64)
    e = ((bits >> 23) & 0xFF) - 127
    e = torch.where(am > 0, e, torch.full_like(e, -127))
    return (e - emax + 127).clamp(0, 254)


def _e8m0(sb: torch.Tensor) -> torch.Tensor:
    v = (sb.to(torch.int64) << 23).to(torch.int32).view(torch.float32)
    return torch.where(sb == 0, torch.full_like(v, 2.0 ** -127), v)


def _mx_pack(rows: torch.Tensor, fmt: int) -> torch.Tensor:
    n, H = rows.shape
    blk = rows.float().reshape(n, H // 32, 32)
    sb = _mx_exp(blk.abs().amax(-1), 2 if fmt == FMT_MXFP4 else 8)           # [n, H/32]
    y = blk / _e8m0(sb)[..., None]
    if fmt == FMT_MXFP4:
        c = _fp4_codes(y).reshape(n, H // 2, 2)
        codes = (c[..., 0] | (c[..., 1] << 4)).to(torch.uint8)
    else:
        codes = y.clamp(-448.0, 448.0).to(torch.float8_e4m3fn).view(torch.uint8).reshape(n, H)
    return torch.cat([codes.reshape(n, -1), sb.to(torch.uint8)], 1).reshape(-1)


def _mx_unpack(b: torch.Tensor, fmt: int, n: int, H: int) -> torch.Tensor:
    r = b.reshape(n, _row_bytes(fmt, H))
    nc = H // 2 if fmt == FMT_MXFP4 else H
    codes, sb = r[:, :nc], r[:, nc:].to(torch.int64)
    if fmt == FMT_MXFP4:
        c = torch.stack([codes & 15, codes >> 4], -1).reshape(n, H).to(torch.int64)
        v = _FP4_GRID[c & 7] * torch.where(c >= 8, -1.0, 1.0)
    else:
        v = codes.contiguous().view(torch.float8_e4m3fn).float()
    return (v.reshape(n, H // 32, 32) * _e8m0(sb)[..., None]).reshape(n, H)


def _grp_bits_pack(q: torch.Tensor, bits: int) -> torch.Tensor:
    """Codes [n, 64] (two's complement, |q| < 2^(bits-1)) -> the group's little-endian bit stream [n, 8 bits] bytes:
    code c at bits [bits c, bits c + bits); 8 consecutive codes are ``bits`` whole bytes (csrc/codec.hip grp_pack8)."""
    n = q.shape[0]
    c = (q.to(torch.int64) & ((1 << bits) - 1)).view(n, 8, 8)
    w = (c << (bits * torch.arange(8, dtype=torch.int64))).sum(-1)                      # [n, 8] words < 2^(8 bits)
    return ((w[..., None] >> (8 * torch.arange(bits, dtype=torch.int64))) & 255).to(torch.uint8).reshape(n, 8 * bits)


def _grp_bits_unpack(b: torch.Tensor, bits: int) -> torch.Tensor:
    n = b.shape[0]
    w = (b.to(torch.int64).view(n, 8, bits) << (8 * torch.arange(bits, dtype=torch.int64))).sum(-1)   # [n, 8]
    c = (w[..., None] >> (bits * torch.arange(8, dtype=torch.int64))) & ((1 << bits) - 1)
    c = torch.where(c >= (1 << (bits - 1)), c - (1 << bits), c)
    return c.reshape(n, 64).float()


def _grp_pack(rows: torch.Tensor, plan) -> torch.Tensor:
    """FMT_GRP rows: per 64-channel group g of b_g bits, s = max|x| / qmax_b (qmax = 2^(b-1) - 1), codes
    clamp(round(x * (1 / s)), -qmax, qmax) packed as a b-bit stream (csrc/codec.hip grp_pack8); then the G fp32
    scales."""
    n, H = rows.shape
    parts, scales = [], []
    for g, b in enumerate(plan):
        blk = rows[:, g * GROUP:(g + 1) * GROUP].float()
        qmax = (1 << (b - 1)) - 1
        am = blk.abs().amax(-1)
        s = am / float(qmax)
        inv = torch.where(am > 0, 1.0 / torch.where(am > 0, s, torch.ones_like(s)), torch.zeros_like(s))
        q = torch.round(blk * inv[:, None]).clamp(-qmax, qmax)
        parts.append(_grp_bits_pack(q, b))
        scales.append(s)
    sc = torch.stack(scales, 1).contiguous().view(torch.uint8).reshape(n, -1)
    return torch.cat(parts + [sc], 1).reshape(-1)


def _grp_unpack(b: torch.Tensor, plan, n: int, H: int) -> torch.Tensor:
    r = b.reshape(n, _row_bytes(FMT_GRP, H, plan))
    cb = sum(8 * x for x in plan)
    sc = r[:, cb:].contiguous().view(torch.float32).reshape(n, len(plan))
    out, off = [], 0
    for g, bits in enumerate(plan):
        nb = 8 * bits
        q = _grp_bits_unpack(r[:, off:off + nb].contiguous(), bits)
        out.append(q * sc[:, g:g + 1])
        off += nb
    return torch.cat(out, 1)


def _header(spec: CodecSpec, L: Layout) -> torch.Tensor:
    return torch.tensor([MAGIC, VERSION, spec.cid, L.B, L.S, L.H, -1 if L.kvar else L.k, L.hi_fmt], dtype=torch.int32)


def _encode_cpu(x, spec, L, lo_mask):
    B, S, H, k = L.B, L.S, L.H, L.k
    msg = torch.zeros(L.total, dtype=torch.uint8)
    msg[:32] = _header(spec, L).view(torch.uint8)
    mw_bytes = _mask_words(lo_mask, L.mw).view(torch.uint8).reshape(-1)
    msg[L.off_mask:L.off_mask + mw_bytes.numel()] = mw_bytes
    kt = int(lo_mask.sum())
    if L.kvar:
        kv = lo_mask.sum(1).to(torch.int32).contiguous().view(torch.uint8)
        msg[L.off_kvec:L.off_kvec + kv.numel()] = kv
    if L.plan is not None:
        msg[L.off_plan:L.off_plan + len(L.plan)] = torch.tensor(L.plan, dtype=torch.uint8)
    xf = x.float().reshape(B, S, H)
    # statistics
    scales = None
    ch = None
    if spec.scale_mode == SC_TOKEN:
        scales = torch.zeros(B, S)
        for is_lo, fmt, qmax in ((False, L.hi_fmt, spec.qmax_hi), (True, L.lo_fmt, spec.qmax_lo)):
            if fmt in (FMT_BF16, FMT_F32, FMT_GRP) or fmt in MX_FORMATS:
                continue
            sel = lo_mask if is_lo else ~lo_mask
            am = xf.abs().amax(-1)
            scales = torch.where(sel, am / float(qmax), scales)
        msg[L.off_scale:L.off_scale + B * S * 4] = scales.reshape(-1).view(torch.uint8)
    elif spec.scale_mode == SC_WINDOW:
        am = torch.where(lo_mask[..., None], xf.abs(), torch.zeros_like(xf)).amax(dim=(1, 2))
        scales = am
        msg[L.off_scale:L.off_scale + B * 4] = am.view(torch.uint8)
    elif spec.scale_mode == SC_CHANNEL:
        ch = xf.abs().amax(1) if spec.ch_kind == CH_MAXABS else xf.mean(1) + 1e-8   # [B, H]
        msg[L.off_scale:L.off_scale + B * H * 4] = ch.reshape(-1).contiguous().view(torch.uint8)
    # rows
    for is_lo in (False, True):
        fmt = L.lo_fmt if is_lo else L.hi_fmt
        sel = lo_mask if is_lo else ~lo_mask
        if not bool(sel.any()):
            continue
        rows = xf[sel]                                      # [n, H] in window/token order
        off = L.off_lo if is_lo else L.hi_offset(kt)
        if fmt == FMT_F32:
            data = rows.contiguous().view(torch.uint8).reshape(-1)
        elif fmt == FMT_BF16:
            data = rows.to(torch.bfloat16).contiguous().view(torch.uint8).reshape(-1)
        elif fmt in MX_FORMATS:
            data = _mx_pack(rows, fmt)
        elif fmt == FMT_GRP:
            data = _grp_pack(rows, L.plan)
        else:
            if spec.scale_mode == SC_TOKEN:
                srow = scales[sel]
                q = _qcodes(rows, spec, is_lo, srow, None)
            elif spec.scale_mode == SC_WINDOW:
                srow = scales.view(B, 1).expand(B, S)[sel]
                q = _qcodes(rows, spec, is_lo, srow, None)
            else:
                chr_ = ch.view(B, 1, H).expand(B, S, H)[sel]
                q = _qcodes(rows, spec, is_lo, None, chr_)
            data = _pack_rows(q, fmt)
        msg[off:off + data.numel()] = data
    return msg


def _decode_cpu(msg, spec, L, dtype):
    B, S, H, k = L.B, L.S, L.H, L.k
    words = msg[L.off_mask:L.off_mask + B * L.mw * 4].view(torch.int32).reshape(B, L.mw)
    lo_mask = _words_to_mask(words, S)
    out = torch.empty(B, S, H, dtype=torch.float32)
    scales = None
    ch = None
    if spec.scale_mode == SC_TOKEN:
        scales = msg[L.off_scale:L.off_scale + B * S * 4].view(torch.float32).reshape(B, S)
    elif spec.scale_mode == SC_WINDOW:
        scales = msg[L.off_scale:L.off_scale + B * 4].view(torch.float32)
    elif spec.scale_mode == SC_CHANNEL:
        ch = msg[L.off_scale:L.off_scale + B * H * 4].view(torch.float32).reshape(B, H)
    kt = int(lo_mask.sum())
    for is_lo in (False, True):
        fmt = L.lo_fmt if is_lo else L.hi_fmt
        sel = lo_mask if is_lo else ~lo_mask
        n = int(sel.sum())
        if n == 0:
            continue
        off = L.off_lo if is_lo else L.hi_offset(kt)
        nb = n * L.row_bytes(fmt)
        raw = msg[off:off + nb]
        if fmt == FMT_F32:
            rows = raw.view(torch.float32).reshape(n, H)
        elif fmt == FMT_BF16:
            rows = raw.view(torch.bfloat16).reshape(n, H).float()
        elif fmt in MX_FORMATS:
            rows = _mx_unpack(raw, fmt, n, H)
        elif fmt == FMT_GRP:
            rows = _grp_unpack(raw, L.plan, n, H)
        else:
            q = _unpack_rows(raw, fmt, n, H)
            if spec.scale_mode == SC_TOKEN:
                rows = _dequant(q, spec, is_lo, scales[sel], None)
            elif spec.scale_mode == SC_WINDOW:
                rows = _dequant(q, spec, is_lo, scales.view(B, 1).expand(B, S)[sel], None)
            else:
                rows = _dequant(q, spec, is_lo, None, ch.view(B, 1, H).expand(B, S, H)[sel])
        out[sel] = rows
    return out.reshape(B * S, H).to(dtype)


# --------------------------------------------------------------------------------------------
# GPU implementation
_HDR_CACHE: dict = {}


def _gpu_header(spec, L, device):
    key = (spec.cid, L, device)
    h = _HDR_CACHE.get(key)
    if h is None:
        h = _header(spec, L).view(torch.uint8).to(device)
        _HDR_CACHE[key] = h
    return h


def _args(spec, L):
    gcb = sum(8 * b for b in L.plan) if L.plan is not None else 0
    return (L.off_mask, L.off_scale, L.off_hi, L.off_lo, L.off_kvec, L.off_plan, L.B, L.S, L.H, max(L.k, 0),
            L.hi_fmt, L.lo_fmt, spec.scale_mode, spec.qmax_hi, spec.qmax_lo, spec.ch_kind, gcb)


_PLAN_CACHE: dict = {}


def _gpu_plan(L, device):
    key = (L.plan, device)
    t = _PLAN_CACHE.get(key)
    if t is None:
        t = torch.tensor(L.plan, dtype=torch.uint8).to(device)
        _PLAN_CACHE[key] = t
    return t


def _encode_gpu(x, spec, L, imp, msg, mass=0.0):
    if x.dtype not in (torch.bfloat16, torch.float32):
        raise TypeError("GPU boundary codec expects bf16 or fp32 activations")
    xf32 = int(x.dtype == torch.float32)
    st = stream()
    msg[:32].copy_(_gpu_header(spec, L, x.device))
    if L.plan is not None:
        msg[L.off_plan:L.off_plan + len(L.plan)].copy_(_gpu_plan(L, x.device))
    if L.kvar:
        if imp is None:
            raise ValueError("top-rho selection needs token importance")
        call("edge_select", ptr(imp.float().contiguous()), L.B, L.S, 0, ptr(msg), L.off_mask, 1, float(mass),
             L.off_kvec, st)
    elif 0 < L.k < L.S:
        if imp is None:
            raise ValueError(f"codec {spec.name} with 0 < k < S needs token importance")
        call("edge_select", ptr(imp.float().contiguous()), L.B, L.S, L.k, ptr(msg), L.off_mask, 0, 0.0, -1, st)
    else:
        call("edge_set_mask", ptr(msg), L.off_mask, L.B, L.S, 1 if L.k >= L.S else 0, st)
    if spec.scale_mode == SC_WINDOW:
        tmp = torch.empty(L.B, L.H, dtype=torch.float32, device=x.device)
        call("edge_channel_stats", ptr(x), ptr(msg), L.off_mask, ptr(tmp), L.B, L.S, L.H, CH_MAXABS, 1, xf32, st)
        call("edge_rowmax", ptr(tmp), msg.data_ptr() + L.off_scale, L.B, L.H, st)
    elif spec.scale_mode == SC_CHANNEL:
        call("edge_channel_stats", ptr(x), ptr(msg), L.off_mask, msg.data_ptr() + L.off_scale, L.B, L.S, L.H,
             spec.ch_kind, 0, xf32, st)
    call("edge_pack", ptr(x), ptr(msg), *_args(spec, L), xf32, st)
    return msg


def _decode_gpu(msg, spec, L, out):
    if out.dtype not in (torch.bfloat16, torch.float32) or not out.is_contiguous():
        raise TypeError("GPU boundary codec decodes into contiguous bf16 or fp32 activations")
    call("edge_unpack", ptr(out), ptr(msg), *_args(spec, L), int(out.dtype == torch.float32), stream())
    return out


# --------------------------------------------------------------------------------------------
SELECTIONS = ("ratio", "top_rho")


def uses_kvar(spec: CodecSpec, selection: str) -> bool:
    if selection not in SELECTIONS:
        raise ValueError(f"unknown selection {selection!r}; known: {SELECTIONS}")
    return selection == "top_rho" and spec.uses_ratio


def encode(x: torch.Tensor, spec: CodecSpec, B: int, S: int, ratio: float = 0.0, importance=None,
           out: torch.Tensor | None = None, k: int | None = None,
           selection: str = "ratio") -> tuple[torch.Tensor, Layout]:
    """Quantize and pack ``x`` ([B*S, H]) into one boundary message (uint8 tensor).

    ``selection="ratio"``: the lo class is the ``k = int(ratio*S)`` least important tokens (``k`` may be given
    directly).  ``"top_rho"``: every window keeps its shortest descending-importance prefix reaching mass
    ``1 - ratio`` and quantizes the rest (per-window k, variable-k message)."""
    H = x.shape[-1]
    if uses_kvar(spec, selection):
        mass = 1.0 - float(ratio)
        if importance is None:
            if mass > 0:
                raise ValueError("top-rho selection needs token importance")
            # ratio >= 1: keep mass <= 0 keeps nothing for any importance (every window all lo, k = S)
            importance = torch.zeros(B, S, dtype=torch.float32, device=x.device)
        L = layout(spec, B, S, H, -1, x.dtype, kvar=True)
        if x.is_cuda:
            if out is None:
                out = torch.zeros(L.total, dtype=torch.uint8, device=x.device)
            return _encode_gpu(x.contiguous(), spec, L, importance, out, mass), L
        lo = select_mask(importance, top_rho_k(importance, mass))
        msg = _encode_cpu(x, spec, L, lo)
        if out is not None:
            out.copy_(msg)
            return out, L
        return msg, L
    k = num_lo(spec, ratio, S) if k is None else (k if spec.uses_ratio else 0)
    L = layout(spec, B, S, H, k, x.dtype)
    if x.is_cuda:
        if out is None:  # zero-filled so the 16-byte section padding is deterministic on the wire
            out = torch.zeros(L.total, dtype=torch.uint8, device=x.device)
        return _encode_gpu(x.contiguous(), spec, L, importance, out), L
    lo = select_mask(importance.float(), k) if (0 < k < S) else \
        torch.full((B, S), k >= S and k > 0, dtype=torch.bool)
    msg = _encode_cpu(x, spec, L, lo)
    if out is not None:
        out.copy_(msg)
        return out, L
    return msg, L


def decode(msg: torch.Tensor, spec: CodecSpec, L: Layout, dtype=torch.bfloat16, out=None) -> torch.Tensor:
    """Unpack and dequantize a boundary message into ``[B*S, H]`` activations."""
    if msg.is_cuda:
        if out is None:
            out = torch.empty(L.B * L.S, L.H, dtype=dtype, device=msg.device)
        return _decode_gpu(msg, spec, L, out)
    y = _decode_cpu(msg, spec, L, dtype)
    if out is not None:
        out.copy_(y)
        return out
    return y


def fake_quant(x: torch.Tensor, spec: CodecSpec, B: int, S: int, ratio: float = 0.0, importance=None,
               k: int | None = None, selection: str = "ratio"):
    """decode(encode(x)): what the receiving stage sees.  Returns (x_hat, message bytes)."""
    msg, L = encode(x, spec, B, S, ratio, importance, k=k, selection=selection)
    return decode(msg, spec, L, x.dtype), message_payload(msg, L)


def message_k(msg: torch.Tensor, L: Layout) -> torch.Tensor:
    """Per-window lo counts of a message [B] (reads the k vector of a variable-k message)."""
    if not L.kvar:
        return torch.full((L.B,), L.k, dtype=torch.int64)
    return msg[L.off_kvec:L.off_kvec + 4 * L.B].view(torch.int32).to(torch.int64)


def message_payload(msg: torch.Tensor, L: Layout) -> int:
    """Bytes a link carries for this message (host sync for a variable-k message)."""
    return L.total if not L.kvar else L.payload_bytes(int(message_k(msg, L).sum()))
