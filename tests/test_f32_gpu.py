"""fp32 execution mode (the reference's precision) on gfx950: h3 split-fp16 GEMMs, split-bf16 attention, fp32 norms,
fp32 boundary codec - each kernel against the plain-PyTorch fp32 oracle (ops/reference.py), and whole models
against the CPU fp32 model."""
import math

import pytest
import torch

from llm_inference_in_distributed_edge_networks_amd import codec as C
from llm_inference_in_distributed_edge_networks_amd import ops
from llm_inference_in_distributed_edge_networks_amd.ops import reference as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rnd(*shape, s=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g) * s


def rel_err(a, ref):
    a, ref = a.double().cpu(), ref.double().cpu()
    assert torch.isfinite(a).all(), "non-finite output"
    return float((a - ref).abs().max() / ref.abs().max().clamp_min(1e-30))


def test_embedding_f32_exact():
    tab = rnd(1000, 896, seed=1)
    ids = torch.randint(0, 1000, (3, 77))
    assert torch.equal(ops.embedding(ids.to(DEV), tab.to(DEV)).cpu(), R.embedding(ids, tab))


def test_split_h3_bitwise():
    x = rnd(300, 896, seed=2) * 10
    x[0, :5] = torch.tensor([0.0, -0.0, 1e-30, 1.0e3, -7.5])
    s = R.h3_scale(x.abs().max().item())
    assert torch.equal(ops.split_h3(x.to(DEV), s).cpu(), R.h3_act(x, s))
    rows = torch.tensor([7, 0, 299])
    assert torch.equal(ops.split_h3(x.to(DEV), s, rows.to(DEV)).cpu(), R.h3_act(x[rows], s))
    # the planes hold s x to ~2^-22 relative; tiny entries keep their absolute accuracy
    assert (R.h3_to_f32(R.h3_act(x, s), s) - x).abs().max() <= 2 ** -21 * x.abs().max()


@pytest.mark.parametrize("H", [512, 896, 2048])
def test_rmsnorm_f32(H):
    x = rnd(300, H, seed=3) * 4
    w = rnd(H, s=0.2, seed=4) + 1
    ref = R.rmsnorm(x, w, 1e-6)
    assert rel_err(ops.rmsnorm(x.to(DEV), w.to(DEV), 1e-6), ref) < 2e-6
    s = R.h3_scale(math.sqrt(H) * w.abs().max().item())
    y3 = ops.rmsnorm(x.to(DEV), w.to(DEV), 1e-6, h3=s)
    assert y3.dtype == torch.float16 and y3.shape == (300, 2 * H)
    assert rel_err(R.h3_to_f32(y3, s), ref) < 2e-6
    rows = torch.tensor([5, 0, 299, 17])
    y3r = ops.rmsnorm(x.to(DEV), w.to(DEV), 1e-6, rows.to(DEV), h3=s)
    assert rel_err(R.h3_to_f32(y3r, s), ref[rows]) < 2e-6
    # the row normalisers as a side output (the AttnLRP forward saves them): same planes, rstd at fp32 level
    rs = torch.empty(300, device=DEV)
    y3s = ops.rmsnorm(x.to(DEV), w.to(DEV), 1e-6, h3=s, rstd_out=rs)
    assert torch.equal(y3s, y3)
    assert rel_err(rs, R.row_rstd(x, 1e-6)) < 1e-6


def test_layernorm_dual_f32():
    x = rnd(257, 512, seed=5) * 3 + 1
    w1, b1, w2, b2 = (rnd(512, s=0.3, seed=s) for s in range(6, 10))
    s1, s2 = 2.0 ** 9, 2.0 ** 7
    y1, y2 = ops.layernorm_dual(*(t.to(DEV) for t in (x, w1, b1, w2, b2)), 1e-5, h3=(s1, s2))
    r1, r2 = R.layernorm_dual(x, w1, b1, w2, b2, 1e-5)
    assert rel_err(R.h3_to_f32(y1, s1), r1) < 3e-6 and rel_err(R.h3_to_f32(y2, s2), r2) < 3e-6
    z = ops.layernorm(x.to(DEV), w1.to(DEV), b1.to(DEV), 1e-5)
    assert rel_err(z, r1) < 3e-6


def _f32_matmul_err(x, w):
    """Max error of the CPU fp32 matmul itself vs fp64 (the yardstick for 'fp32-level')."""
    ref = x.double() @ w.double().t()
    return rel_err(x @ w.t(), ref)


@pytest.mark.parametrize("M,N,K,epi", [
    (300, 896, 896, "resid"), (32768, 896, 896, "resid"), (32768, 896, 4864, "resid"),   # 256x224 (w7) kernel
    (4096, 9728, 896, "swiglu"), (300, 1152, 896, "none"), (2048, 2048, 512, "gelu"),    # 256x256 / 128x128
    (700, 512, 2048, "bias_resid"), (8192, 1024, 640, "bias"), (1000, 512, 512, "bias_resid")])
def test_linear_h3_fp32_accuracy(M, N, K, epi, slack=0, two_term=False):
    """h3 GEMM vs fp64; ``slack`` binades of headroom between the activation's scaled maximum and the fp16 range
    (the model's scales come from bounds, not from the data: the planes stay accurate far below the bound).
    ``two_term``: bf16-valued weights (checkpoint values), exact in fp16 -> the K' = 2K GEMM."""
    x = rnd(M, K, seed=10)
    w = rnd(N, K, s=1 / math.sqrt(K), seed=11)
    if two_term:
        w = w.to(torch.bfloat16).float()
    b = rnd(N, s=0.1, seed=12) if "bias" in epi or epi == "gelu" else None
    r = rnd(M, N, seed=13) if "resid" in epi else None
    act = {"gelu": "gelu", "swiglu": "swiglu_il"}.get(epi)
    sx = R.h3_scale(x.abs().max().item()) / 2 ** slack
    w3, sw = R.h3_weight(w)
    assert w3.shape[1] == (1 if two_term else 3) * K
    ref = x.double() @ w.double().t()
    if b is not None:
        ref = ref + b.double()
    if act == "gelu":
        ref = torch.nn.functional.gelu(ref)
    elif act == "swiglu_il":
        g, u = R.deinterleave_gate_up(ref)
        ref = torch.nn.functional.silu(g) * u
    so = R.h3_scale(ref.abs().max().item())
    y = ops.linear_h3(R.h3_act(x, sx).to(DEV), w3.to(DEV), 1.0 / (sx * sw), None if b is None else b.to(DEV),
                      None if r is None else r.to(DEV), act, out_scale=so)
    if act is not None:
        y = R.h3_to_f32(y, so)
    if r is not None:
        ref = ref + r.double()
    yard = _f32_matmul_err(x[:512], w)
    err = rel_err(y, ref)
    # fp32-level: within a small factor of the CPU fp32 GEMM's own error (the h3 scheme drops 2^-22 terms and
    # rounds the residual plane at 2^-23; the h3 re-split of the epilogue output adds one more such rounding)
    assert err < max(4 * yard, 2e-6), (err, yard)


@pytest.mark.parametrize("M,N,K,epi", [(32768, 896, 896, "resid"), (32768, 896, 4864, "resid"),
                                       (4096, 9728, 896, "swiglu"), (300, 1152, 896, "none"), (2048, 2048, 512, "gelu"),
                                       (700, 512, 2048, "bias_resid")])
def test_linear_h3_two_term(M, N, K, epi):
    """Weights exact in fp16 (bf16 checkpoint values): the two-product GEMM, same fp32-level accuracy."""
    test_linear_h3_fp32_accuracy(M, N, K, epi, two_term=True)


@pytest.mark.parametrize("M", [1000, 257])
@pytest.mark.parametrize("two_term", [False, True])
def test_linear_h3_swiglu_partial_tiles(M, two_term):
    """SwiGLU h3 epilogue of the four-wave 256x256 kernel (full-line stores: rows r and r ^ 8 of a 16-row group
    exchange chunks) forced at M not a multiple of 256: the guarded rows of the partial last tile."""
    ops.set_gemm_tile(256)
    try:
        test_linear_h3_fp32_accuracy(M, 9728, 896, "swiglu", two_term=two_term)
    finally:
        ops.set_gemm_tile(0)


@pytest.mark.parametrize("slack", [8, 14])
def test_linear_h3_loose_scale(slack):
    """Scales 2^8 / 2^14 below the data's own (the model's bounds are loose): still fp32-level."""
    test_linear_h3_fp32_accuracy(2048, 896, 4864, "resid", slack)


@pytest.mark.parametrize("M,N,K", [(32768, 896, 9728), (8192, 896, 1152), (300, 896, 896), (2048, 1024, 640)])
def test_linear_h3_colscale(M, N, K):
    """colscale[n] * rscale[m] * (x @ w.T) + residual (the relevance engine's norm-weighted input gradients): the
    four-wave 256x224 kernel (M = 32768), the 128x128 kernel (small M) and the 256-wide generic path, two products
    (bf16-valued weights), in place on the residual, fp32-level against fp64."""
    x, w, r = rnd(M, K, seed=40), rnd(N, K, s=0.03, seed=41).bfloat16().float(), rnd(M, N, seed=42)
    cs, rs = 1 + 0.3 * rnd(N, seed=43), torch.rand(M, generator=torch.Generator().manual_seed(44)) + 0.5
    sx = R.h3_scale(x.abs().max().item())
    w3, sw = R.h3_weight(w)
    rd = r.to(DEV)
    y = ops.linear_h3(R.h3_act(x, sx).to(DEV), w3.to(DEV), 1.0 / (sx * sw), residual=rd, out=rd, rscale=rs.to(DEV),
                      colscale=cs.to(DEV))
    assert y.data_ptr() == rd.data_ptr()
    ref = (x.double() @ w.double().t()) * rs.double().view(-1, 1) * cs.double().view(1, -1) + r.double()
    assert rel_err(y, ref) < 4e-6     # fp32 level at K up to 9728 (a CPU fp32 GEMM: ~2e-6 there)


@pytest.mark.parametrize("M,N,K", [(32768, 896, 9728), (300, 896, 896), (2048, 1024, 640)])
def test_linear_h3_colscale_planes(M, N, K):
    """The column-scaled GEMM that also writes its result as h3 planes at bound-derived row scales (the AttnLRP dy):
    the fp32 output unchanged, the planes the exact split of s_m * row m with s_m from the bound (CPU oracle), below
    2^15, and rinv = 1 / s_m - the 256x224 kernel, the 128x128 kernel and the 256-wide generic path."""
    x, w, r = rnd(M, K, seed=40), rnd(N, K, s=0.03, seed=41).bfloat16().float(), rnd(M, N, seed=42)
    cs, rs = 1 + 0.3 * rnd(N, seed=43), torch.rand(M, generator=torch.Generator().manual_seed(44)) + 0.5
    sx = R.h3_scale(x.abs().max().item())
    w3, sw = R.h3_weight(w)
    a3, w3d = R.h3_act(x, sx).to(DEV), w3.to(DEV)
    g = torch.Generator().manual_seed(45)
    ba = (r.abs().amax(1) * (1 + torch.rand(M, generator=g))) / 32768   # |resid row| < 2^15 ba
    bb = rs.clone()
    bc = float(((x.abs().amax() * sx) * w.abs().sum(1).max() * cs.abs().max()) / sx)   # |product| / rs per row
    args = dict(residual=r.to(DEV), rscale=rs.to(DEV), colscale=cs.to(DEV))
    y0 = ops.linear_h3(a3, w3d, 1.0 / (sx * sw), **args)
    y, pl, pr = ops.linear_h3(a3, w3d, 1.0 / (sx * sw), planes_bound=(ba.to(DEV), bb.to(DEV), bc), **args)
    torch.cuda.synchronize()
    assert torch.equal(y, y0)
    _, want_pr = R.bound_planes(y.cpu(), ba, bb, bc)
    # the bound may be formed with an fma on the device: a row exactly at a power of two may land one binade over
    assert (pr.cpu() == want_pr).float().mean() > 0.999
    assert torch.all((pr.cpu() == want_pr) | (pr.cpu() == 2 * want_pr) | (pr.cpu() == want_pr / 2))
    assert torch.equal(pl.cpu(), R.h3_act(y.cpu() / pr.cpu().view(-1, 1), 1.0))
    assert float(pl.float().abs().max()) < 2 ** 15


@pytest.mark.parametrize("M,K,two_term", [(32768, 896, True), (32768, 4864, True), (16384, 896, False)])
def test_linear_h3_np(M, K, two_term):
    """The O-projection / down GEMM with the next RMSNorm's producer side in its epilogue (EPI_F32_RESID_NP): the fp32
    output bit-identical to the plain residual GEMM, the planes the exact split of p_m (y_m * g) and 1 / p_m exactly the
    CPU oracle's (R.np_planes on the GPU's y: same fp32 bound arithmetic), below 2^14, the sum-of-squares partials the
    row sums of y^2 per 112-column slab; and the consumer side (row_rscale_mul + the gate/up GEMM on the planes) equal
    to rmsnorm -> gate/up within fp32 accuracy."""
    N = 896
    x, w, r = rnd(M, K, seed=60), rnd(N, K, s=0.03, seed=61), rnd(M, N, seed=62)
    if two_term:
        w = w.bfloat16().float()
    g = 1 + 0.2 * rnd(N, seed=63)
    g[7] = 9.0                                   # an outlier norm channel
    sx = R.h3_scale(x.abs().max().item())
    w3, sw = R.h3_weight(w)
    a3, w3d, rd = R.h3_act(x, sx).to(DEV), w3.to(DEV), r.to(DEV)
    rstd = torch.rsqrt(r.pow(2).mean(1) + 1e-6)
    pb = float(x.abs().max() * w.abs().sum(1).max())          # |x @ w.T| bound
    assert ops.gemm_np_supported(M, N, 2 * K)
    al = 1.0 / (sx * sw)
    y0 = ops.linear_h3(a3, w3d, al, residual=rd)
    y, pl, pr, ssq = ops.linear_h3_np(a3, w3d, al, rd, g.to(DEV), rstd.to(DEV), float(g.abs().max()), pb)
    torch.cuda.synchronize()
    assert torch.equal(y, y0)
    want_pl, want_pr, want_ssq = R.np_planes(y.cpu(), g, rstd, float(g.abs().max()), pb)
    assert torch.equal(pr.cpu(), want_pr) and torch.equal(pl.cpu(), want_pl)
    assert float(pl.float().abs().max()) < 2 ** 14
    assert rel_err(ssq, want_ssq.double()) < 1e-6
    # consumer: the gate/up GEMM on the planes with the fused row scale == on rmsnorm(y) * g planes (fp32 accuracy)
    wg = rnd(2 * 4864, N, s=0.03, seed=64).bfloat16().float()
    wg3, swg = R.h3_weight(wg)
    rs = ops.row_rscale_mul(ssq, pr, N, 1e-6)
    yd = y.cpu().double()
    yn = yd * torch.rsqrt(yd.pow(2).mean(1, keepdim=True) + 1e-6) * g.double()
    got_gu = ops.linear_h3(pl, wg3.to(DEV), 1.0 / swg, rscale=rs)   # the plain GEMM: the pre-activations
    assert rel_err(got_gu, yn @ wg.double().t()) < 4e-6


@pytest.mark.parametrize("M,two_term", [(32768, True), (32768, False), (1000, True), (257, False)])
def test_linear_h3_swiglu_raw(M, two_term):
    """One GEMM for the SwiGLU planes and the saved pre-activations (AttnLRP forward): the planes bit-identical to
    act="swiglu_il" and the pre-activations bit-identical to the plain fp32 GEMM - four-wave 256x256 (M = 32768),
    the small-M kernels and partial row tiles, two and three products."""
    K, N = 896, 2 * 4864
    x, w = rnd(M, K, seed=50), rnd(N, K, s=0.03, seed=51)
    if two_term:
        w = w.bfloat16().float()
    sx = R.h3_scale(x.abs().max().item())
    w3, sw = R.h3_weight(w)
    a3, w3 = R.h3_act(x, sx).to(DEV), w3.to(DEV)
    rs = (torch.rand(M, generator=torch.Generator().manual_seed(52)) + 0.5).to(DEV)
    al = 1.0 / (sx * sw)
    planes, raw = ops.linear_h3_swiglu_raw(a3, w3, al, 64.0, rscale=rs)
    assert torch.equal(planes, ops.linear_h3(a3, w3, al, act="swiglu_il", out_scale=64.0, rscale=rs))
    assert torch.equal(raw, ops.linear_h3(a3, w3, al, rscale=rs))


def test_linear_h3_inplace_residual():
    M, K, N = 32768, 896, 896
    x, w, r = rnd(M, K, seed=20), rnd(N, K, s=0.03, seed=21), rnd(M, N, seed=22)
    rd = r.to(DEV)
    sx = R.h3_scale(x.abs().max().item())
    w3, sw = R.h3_weight(w)
    y = ops.linear_h3(R.h3_act(x, sx).to(DEV), w3.to(DEV), 1.0 / (sx * sw), residual=rd, out=rd)
    assert y.data_ptr() == rd.data_ptr()
    assert rel_err(y, x.double() @ w.double().t() + r.double()) < 2e-6


# 192-wide tiles need N % 192 == 0: the (8, 8) head layouts (N = 1536) run the auto and 256 tiles only
QKV_CELLS = [(B, S, Hq, Hkv, rot, tile)
             for (B, S, Hq, Hkv, rot) in [(2, 512, 14, 2, 64), (2, 100, 14, 2, 64), (1, 2048, 8, 8, 16),
                                          (64, 512, 14, 2, 64), (24, 2048, 8, 8, 16), (2, 512, 14, 2, 0)]
             for tile in ["auto", "192", "256"]
             if tile != "192" or ((Hq + 2 * Hkv) * 64) % 192 == 0]


@pytest.mark.parametrize("B,S,Hq,Hkv,rot,tile", QKV_CELLS)
@pytest.mark.parametrize("two_term", [False, True])
def test_qkv_rope_h3(B, S, Hq, Hkv, rot, tile, two_term):
    """fp32 QKV+RoPE from h3 operands: 128x128 tiles (small M), the four-wave 256x192 kernel with permuted weight rows
    (N = 1152, production M; forced at small M with tile 192) and the 256x256 kernel (tile 256), three- and
    two-product weights."""
    H = 896 if Hq == 14 else 512
    Nq = (Hq + 2 * Hkv) * 64
    x = rnd(B * S, H, seed=30)
    w = rnd(Nq, H, s=1 / math.sqrt(H), seed=31)
    if two_term:
        w = w.to(torch.bfloat16).float()
    b = rnd(Nq, s=0.1, seed=32)
    cos, sin = R.rope_tables(4096, max(rot, 2), 1e6 if rot == 64 else 1e4)
    sx = R.h3_scale(x.abs().max().item())
    w3, sw = R.h3_weight(w)
    try:
        if tile in ("192", "256"):
            ops.set_gemm_tile(int(tile))
        q, k, vt = ops.qkv_rope_h3(R.h3_act(x, sx).to(DEV), w3.to(DEV), 1.0 / (sx * sw), b.to(DEV), cos.to(DEV),
                                   sin.to(DEV), B, S, Hq, Hkv, 64, rot, 0.125)
        torch.cuda.synchronize()
    finally:
        ops.set_gemm_tile(0)
    rq, rk, rv = R.qkv_rope(x.double(), w.double(), b.double(), cos.double(), sin.double(), B, S, Hq, Hkv, 64, rot,
                            0.125)
    assert rel_err(q, rq) < 4e-6 and rel_err(k, rk) < 4e-6 and rel_err(vt, rv) < 4e-6


@pytest.mark.parametrize("B,S,Hq,Hkv,rot", [(2, 512, 14, 2, 64), (2, 100, 14, 2, 64), (1, 2048, 8, 8, 16),
                                             (3, 200, 14, 2, 0), (64, 512, 14, 2, 64)])
@pytest.mark.parametrize("tile", ["auto", "192", "256"])
def test_qkv_kv_planes(B, S, Hq, Hkv, rot, tile):
    """K / V^T h3 planes from the fp32 QKV epilogues (128x128, 256x192 and 256x256 tiles) are the split of the fp32
    K / V^T, bit for bit, V^T keys in the attention kernel's P^T order and zero key padding; q and K unchanged; the
    optional row-major V equals the fp32 V^T."""
    H = 896 if Hq == 14 else 512
    Nq = (Hq + 2 * Hkv) * 64
    x = rnd(B * S, H, seed=33)
    w = rnd(Nq, H, s=1 / math.sqrt(H), seed=34).to(torch.bfloat16).float()
    b = rnd(Nq, s=0.1, seed=35)
    cos, sin = R.rope_tables(4096, max(rot, 2), 1e6 if rot == 64 else 1e4)
    sx = R.h3_scale(x.abs().max().item())
    w3, sw = R.h3_weight(w)
    sk, sv = 2.0 ** 9, 2.0 ** 11
    try:
        if tile in ("192", "256"):
            ops.set_gemm_tile(int(tile))
        q, k, vt, kp, vp, v = ops.qkv_rope_h3(R.h3_act(x, sx).to(DEV), w3.to(DEV), 1.0 / (sx * sw), b.to(DEV),
                                              cos.to(DEV), sin.to(DEV), B, S, Hq, Hkv, 64, rot, 0.125,
                                              kv_scales=(sk, sv), v_rows=True)
        q2, k2, vt2 = ops.qkv_rope_h3(R.h3_act(x, sx).to(DEV), w3.to(DEV), 1.0 / (sx * sw), b.to(DEV), cos.to(DEV),
                                      sin.to(DEV), B, S, Hq, Hkv, 64, rot, 0.125)
        torch.cuda.synchronize()
    finally:
        ops.set_gemm_tile(0)
    assert vt is None and torch.equal(q, q2) and torch.equal(k, k2)   # the planes replace the fp32 V^T
    rkp, rvp = R.kv_planes(k.cpu(), vt2.cpu(), sk, sv)
    assert torch.equal(kp.cpu(), rkp)
    assert torch.equal(vp.cpu(), rvp)
    assert torch.equal(v, vt2[..., :S].transpose(-1, -2))   # V row-major (AttnLRP), the same values as V^T


@pytest.mark.parametrize("B,S,rot", [(2, 512, 64), (3, 98, 64), (64, 512, 64), (3, 200, 0)])
def test_qkv_planes_only(B, S, rot):
    """The planes-only QKV of the model's layers (need_k=False: q + K / V^T planes, no fp32 K / V^T / V rows) on the
    256x192 tiles: q and the planes equal the need_k=True call's bit for bit (partial row tiles, S % 4 != 0, no
    rotary).  (A separate planes-only instantiation with the unused outputs compiled out was measured 2-4 % slower on
    the bench-shape probe than this one and removed: docs/RESULTS.md section 6.)"""
    Hq, Hkv, H = 14, 2, 896
    Nq = (Hq + 2 * Hkv) * 64
    x = rnd(B * S, H, seed=36)
    w = rnd(Nq, H, s=1 / math.sqrt(H), seed=37).to(torch.bfloat16).float()
    b = rnd(Nq, s=0.1, seed=38)
    cos, sin = R.rope_tables(4096, max(rot, 2), 1e6)
    sx = R.h3_scale(x.abs().max().item())
    w3, sw = R.h3_weight(w)
    args = (R.h3_act(x, sx).to(DEV), w3.to(DEV), 1.0 / (sx * sw), b.to(DEV), cos.to(DEV), sin.to(DEV), B, S, Hq, Hkv,
            64, rot, 0.125)
    try:
        ops.set_gemm_tile(192)
        q1, k1, _, kp1, vp1 = ops.qkv_rope_h3(*args, kv_scales=(2.0 ** 9, 2.0 ** 11), need_k=True)
        q2, k2, _, kp2, vp2 = ops.qkv_rope_h3(*args, kv_scales=(2.0 ** 9, 2.0 ** 11), need_k=False)
        torch.cuda.synchronize()
    finally:
        ops.set_gemm_tile(0)
    assert k1 is not None and k2 is None
    assert torch.equal(q1, q2) and torch.equal(kp1, kp2) and torch.equal(vp1, vp2)


@pytest.mark.parametrize("B,S,Hq,Hkv", [(2, 512, 14, 2), (3, 100, 14, 2), (1, 2048, 8, 8), (2, 64, 4, 1),
                                         (2, 200, 14, 2)])
@pytest.mark.parametrize("h3", [False, True])
def test_attention_kv_planes_bit_identical(B, S, Hq, Hkv, h3):
    """The LDS-DMA plane-staged attention (K / V^T planes from the QKV epilogue) equals the kernel that splits the
    fp32 K / V^T itself (variant 2, 128 query rows, fp16 planes): output and LSE bit for bit, and the scored-rows mode
    on its rows."""
    q = rnd(B, Hq, S, 64, seed=46) * 0.5
    k = rnd(B, Hkv, S, 64, seed=47) * 2
    v = rnd(B, Hkv, S, 64, seed=48)
    sp = R.s_pad(S)
    vt = torch.zeros(B, Hkv, 64, sp)
    vt[..., :S] = v.transpose(-1, -2)
    s = R.h3_scale(v.abs().max().item()) if h3 else 0.0
    sc = tuple(R.h3_scale(t.abs().max().item()) for t in (q, k, v))
    kp, vp = R.kv_planes(k, vt, sc[1], sc[2])
    args = (q.to(DEV), k.to(DEV), vt.to(DEV), S)
    planes = (kp.to(DEV), vp.to(DEV))
    o1, l1 = ops.attention(*args, need_lse=True, h3=s, in_scales=sc)
    o2, l2 = ops.attention(q.to(DEV), k.to(DEV), None, S, need_lse=True, h3=s, in_scales=sc, kv_planes=planes)
    assert torch.equal(o1, o2) and torch.equal(l1, l2)
    if h3:   # the planes plus fp32 rows (AttnLRP forward): the planes unchanged, the rows = the fp32 kernel's output
        o4, l4, o32 = ops.attention(q.to(DEV), k.to(DEV), None, S, need_lse=True, h3=s, in_scales=sc,
                                    kv_planes=planes, f32_out=True)
        of, _ = ops.attention(*args, need_lse=True, in_scales=sc, kv_planes=planes)
        assert torch.equal(o4, o1) and torch.equal(l4, l1) and torch.equal(o32, of)
        assert torch.equal(ops.split_h3(o32, s), o1)   # the planes are the split of those rows
    n_rows = torch.tensor([float(min(31 + 40 * i, S - 2)) for i in range(B)], device=DEV)
    o3, _ = ops.attention(*args, n_rows=n_rows, h3=s, in_scales=sc, kv_planes=planes)
    W = o1.shape[1]
    for bi in range(B):
        lo = S - 1 - int(n_rows[bi])
        assert torch.equal(o3.view(B, S, W)[bi, lo:], o1.view(B, S, W)[bi, lo:])


@pytest.mark.parametrize("B,S,Hq,Hkv", [(2, 512, 14, 2), (3, 100, 14, 2), (1, 2048, 8, 8), (2, 64, 4, 1)])
@pytest.mark.parametrize("h3", [False, True])
@pytest.mark.parametrize("planes", ["bf16", "fp16"])
def test_attention_f32(B, S, Hq, Hkv, h3, planes):
    """fp32 attention vs fp64: the split-plane MFMA kernel (128 query rows per workgroup) on three bf16 planes or two
    scaled fp16 planes (h3).  The error is dominated by the fp32 exp2 (~5e-6 relative L2; bf16 attention is ~1e-3)."""
    _attention_f32_case(B, S, Hq, Hkv, h3, planes == "fp16")


def _attention_f32_case(B, S, Hq, Hkv, h3, fp16=False, slack=0):
    q = rnd(B, Hq, S, 64, seed=40) * 0.5
    k = rnd(B, Hkv, S, 64, seed=41) * 2
    v = rnd(B, Hkv, S, 64, seed=42)
    sp = R.s_pad(S)
    vt = torch.zeros(B, Hkv, 64, sp)
    vt[..., :S] = v.transpose(-1, -2)
    s = R.h3_scale(v.abs().max().item()) if h3 else 0.0
    sc = tuple(R.h3_scale(t.abs().max().item()) / 2 ** slack for t in (q, k, v)) if fp16 else None
    o, lse = ops.attention(q.to(DEV), k.to(DEV), vt.to(DEV), S, need_lse=True, h3=s, in_scales=sc)
    ro, rl = R.attention(q.double(), k.double(), vt.double(), S, need_lse=True)
    if h3:
        o = R.h3_to_f32(o, s)
    assert rel_err(o, ro) < 1e-5
    assert float((lse.cpu().double() - rl).abs().max()) < 5e-5


def test_attention_h3_loose_scales():
    """fp16-plane attention with its input scales 10 binades below the data's (the model's bounds are loose)."""
    _attention_f32_case(2, 512, 14, 2, True, fp16=True, slack=10)


def test_attention_f32_scored_rows_only():
    B, S, Hq, Hkv = 3, 512, 14, 2
    q, k = rnd(B, Hq, S, 64, seed=43), rnd(B, Hkv, S, 64, seed=44)
    vt = rnd(B, Hkv, 64, S, seed=45)
    n_rows = torch.tensor([31.0, 5.0, 100.0])
    o, _ = ops.attention(q.to(DEV), k.to(DEV), vt.to(DEV), S, n_rows=n_rows.to(DEV))
    ro, _ = R.attention(q.double(), k.double(), vt.double(), S)
    for b in range(B):
        lo = S - 1 - int(n_rows[b])
        sl = slice(b * S + lo, (b + 1) * S)
        assert rel_err(o[sl], ro[sl]) < 5e-6


@pytest.mark.parametrize("B,S,Hq,Hkv", [(2, 512, 14, 2), (1, 2048, 8, 8), (2, 100, 4, 2)])
def test_importance_stats_f32(B, S, Hq, Hkv):
    q = rnd(B, Hq, S, 64, seed=50) * 0.5
    k = rnd(B, Hkv, S, 64, seed=51)
    _, rl = R.attention(q.double(), k.double(), torch.zeros(B, Hkv, 64, R.s_pad(S), dtype=torch.float64), S,
                        need_lse=True)
    lr = ops.attn_lastrow(q.to(DEV), k.to(DEV), S)
    assert rel_err(lr, R.attn_lastrow(q.double(), k.double(), S)) < 2e-6
    cs = ops.attn_colsum(q.to(DEV), k.to(DEV), rl.float().to(DEV), S)
    assert rel_err(cs, R.attn_colsum(q.double(), k.double(), rl, S)) < 5e-6
    # the split-plane matrix-core kernels (the model's fp32 path): scores on h3 planes at the bound scales
    sc = (R.h3_scale(q.abs().max().item()), R.h3_scale(k.abs().max().item()))
    lr = ops.attn_lastrow(q.to(DEV), k.to(DEV), S, in_scales=sc)
    assert rel_err(lr, R.attn_lastrow(q.double(), k.double(), S)) < 2e-6
    cs = ops.attn_colsum(q.to(DEV), k.to(DEV), rl.float().to(DEV), S, in_scales=sc)
    assert rel_err(cs, R.attn_colsum(q.double(), k.double(), rl, S)) < 5e-6


@pytest.mark.parametrize("R_", [200, 2048])
def test_head_nll_h3(R_):
    """fp32 LM head + CE from h3 operands: 128x128 tiles (200 rows) and the four-wave 256x256 kernel (2048 rows,
    partial last vocabulary tile); the first 96 rows against fp64."""
    H, V = 896, 151936
    h = rnd(R_, H, seed=60)
    w = rnd(V, H, s=0.05, seed=61)
    t = torch.randint(0, V, (R_,))
    t[:3] = torch.tensor([0, V - 1, V - 100])
    sh = R.h3_scale(h.abs().max().item())
    w3, sw = R.h3_weight(w)
    nll = ops.head_nll_h3(R.h3_act(h, sh).to(DEV), w3.to(DEV), 1.0 / (sh * sw), t.to(DEV))
    ref = R.head_nll(h[:96].double(), w.double(), t[:96])
    assert float((nll[:96].cpu().double() - ref).abs().max()) < 2e-5


@pytest.mark.parametrize("codec", ["ref_int4_global", "mixed_int4_int8", "int4_token", "passthrough", "channel_4",
                                   "channel_1_mean", "int8_token_keep"])
def test_codec_fp32_bitexact_vs_cpu(codec):
    """fp32 activations: GPU message bytes == CPU reference bytes; the hi class of ref_int4_global stays fp32
    (reference Q1, Experiments/Qwen2-0.5B/qwen_layer_wise.py:54-70)."""
    B, S, H = 3, 512, 896
    x = rnd(B * S, H, seed=70) * 3
    x[5, 7] = 80.0
    imp = torch.rand(B, S, generator=torch.Generator().manual_seed(71))
    spec = C.get_codec(codec)
    m_cpu, L = C.encode(x, spec, B, S, 0.5, imp)
    m_gpu, L2 = C.encode(x.to(DEV), spec, B, S, 0.5, imp.to(DEV))
    assert L == L2
    y_cpu = C.decode(m_cpu, spec, L, torch.float32)
    y_gpu = C.decode(m_gpu, spec, L, torch.float32)
    if codec == "channel_1_mean":
        # the channel MEAN is a sum in a different order on the GPU (not bitwise); the ternary codes agree except
        # where x / mean sits on a rounding boundary
        assert (y_gpu.cpu() - y_cpu).abs().gt(1e-5).float().mean() < 1e-4
        return
    assert torch.equal(m_gpu.cpu(), m_cpu)
    assert torch.equal(y_gpu.cpu(), y_cpu)
    if codec == "ref_int4_global":
        # reference Q1 formula on the lo tokens, hi tokens untouched fp32
        k = int(0.5 * S)
        for b in range(B):
            xb = x.view(B, S, H)[b]
            idx = torch.sort(imp[b], stable=True).indices[:k]
            m = xb[idx].abs().max()
            q = torch.round(torch.clamp(xb[idx] / m * 7.0, -8.0, 7.0))
            exp = xb.clone()
            exp[idx] = q / 7.0 * m
            assert torch.equal(y_gpu.view(B, S, H)[b].cpu(), exp)


# ---- whole models at full size: GPU fp32 mode vs the CPU fp32 model on the same random weights -----------------
def _full_model_nll(cfg, B, S, seed=0, values=None):
    from llm_inference_in_distributed_edge_networks_amd.eval.data import synthetic_stream
    from llm_inference_in_distributed_edge_networks_amd.eval.windows import batches, sliding_windows, window_nll
    from llm_inference_in_distributed_edge_networks_amd.models import DecoderLM
    toks = synthetic_stream(S * 4, cfg.vocab_size, seed)
    wins = [w for w in sliding_windows(toks.shape[1], S, 32) if w.length == S][:B]
    b = next(batches(toks, wins, B))
    out = {}
    for dev in ("cpu", DEV):
        m = DecoderLM.random_init(cfg, seed, device=dev, dtype=torch.float32, values=values)
        bb = b.to(dev)
        x = m.forward_hidden(bb.ids)
        out[dev] = window_nll(m.row_nll(x, bb.rows, bb.targets), bb).double().cpu()
        del m
    return out["cpu"], out[DEV]


@pytest.mark.parametrize("name,B,S,values", [("qwen2-0.5b", 2, 512, None), ("pythia-70m", 2, 2048, None),
                                            ("qwen2-0.5b", 2, 512, torch.bfloat16),
                                            ("pythia-70m", 2, 2048, torch.float16)])
def test_full_model_nll_matches_cpu_fp32(name, B, S, values):
    """Full 24-layer Qwen2-0.5B / 6-layer Pythia-70M: per-window NLL of the GPU fp32 mode within 1e-4 relative of
    the CPU fp32 oracle (random-init weights of the exact architecture, full fp32 values or the checkpoints' bf16 /
    fp16 values - the two-product GEMMs; the CPU run is itself fp32)."""
    from llm_inference_in_distributed_edge_networks_amd.models import get_config
    cpu, gpu = _full_model_nll(get_config(name), B, S, values=values)
    rel = ((gpu - cpu).abs() / cpu.abs()).max().item()
    assert rel < 1e-4, (rel, cpu.tolist(), gpu.tolist())


def test_full_model_fused_norm_equals_separate_pass():
    """Qwen2-0.5B fp32 mode with RMSNorm-2 fused into the O projection's epilogue (opt-in) vs the separate norm pass:
    the final hidden state and the row NLL agree to fp32 accuracy (the planes carry a per-row instead of a per-layer
    scale, and the row sums of squares come from the epilogue's 112-column partials)."""
    from llm_inference_in_distributed_edge_networks_amd.eval.data import synthetic_stream
    from llm_inference_in_distributed_edge_networks_amd.eval.windows import batches, sliding_windows
    from llm_inference_in_distributed_edge_networks_amd.models import DecoderLM, get_config
    cfg = get_config("qwen2-0.5b")
    S = 512
    toks = synthetic_stream(S * 40, cfg.vocab_size, 0)
    b = next(batches(toks, [w for w in sliding_windows(toks.shape[1], S, 32) if w.length == S][:32], 32)).to(DEV)
    m = DecoderLM.random_init(cfg, 0, device=DEV, dtype=torch.float32, values=torch.bfloat16)
    m.fuse_norm_f32 = True                       # opt-in (EDGE_FUSED_NORM_F32=1): slower on the bench, kept tested
    assert m._np_fused(32 * S)
    out = {}
    for flag in (True, False):
        m.fuse_norm_f32 = flag
        x = m.forward_hidden(b.ids)
        out[flag] = (x.double().cpu(), m.row_nll(x, b.rows, b.targets).double().cpu())
    assert _l2(out[True][0], out[False][0]) < 2e-6 and _l2(out[True][1], out[False][1]) < 1e-6


@pytest.mark.parametrize("name", ["qwen2-0.5b", "pythia-70m"])
def test_full_model_kv_planes_identical(name, monkeypatch):
    """The fp32 model with the plane-staged attention (default) equals the per-tile-split attention bit for bit."""
    from llm_inference_in_distributed_edge_networks_amd.eval.data import synthetic_stream
    from llm_inference_in_distributed_edge_networks_amd.eval.windows import batches, sliding_windows
    from llm_inference_in_distributed_edge_networks_amd.models import DecoderLM, get_config
    from llm_inference_in_distributed_edge_networks_amd.models import model as MM
    cfg = get_config(name)
    S = 512
    toks = synthetic_stream(S * 4, cfg.vocab_size, 0)
    b = next(batches(toks, [w for w in sliding_windows(toks.shape[1], S, 32) if w.length == S][:3], 3)).to(DEV)
    m = DecoderLM.random_init(cfg, 0, device=DEV, dtype=torch.float32, values=torch.bfloat16)
    out = {}
    for flag in (True, False):
        monkeypatch.setattr(MM, "_KV_PLANES", flag)
        x = m.forward_hidden(b.ids)
        out[flag] = (x.clone(), m.row_nll(x, b.rows, b.targets).clone())
    assert torch.equal(out[True][0], out[False][0]) and torch.equal(out[True][1], out[False][1])


@pytest.mark.parametrize("M,N,K,epi", [(32768, 9728, 896, "swiglu"), (4096, 2048, 512, "gelu"),
                                       (1000, 1024, 896, "resid"), (700, 2048, 512, "bias")])
def test_linear_h3_four_wave(M, N, K, epi):
    """The h3 (fp32-mode) GEMMs on the persistent four-wave kernel, forced at every M."""
    ops.set_gemm_tile(256)
    try:
        test_linear_h3_fp32_accuracy(M, N, K, {"resid": "resid", "gelu": "gelu", "swiglu": "swiglu",
                                                "bias": "bias"}[epi])
    finally:
        ops.set_gemm_tile(0)


@pytest.mark.parametrize("M,N,K", [(300, 896, 896), (32768, 896, 896), (32768, 896, 4864), (256 * 3 + 5, 2688, 128)])
def test_linear_h3_four_wave_224(M, N, K):
    """The fp32-residual O-proj / down GEMMs on the four-wave 256x224 kernel."""
    ops.set_gemm_tile(224)
    try:
        test_linear_h3_fp32_accuracy(M, N, K, "resid")
    finally:
        ops.set_gemm_tile(0)


@pytest.mark.parametrize("M,N,K,epi,tile", [
    (32768, 896, 896, "resid", 0), (32768, 896, 4864, "resid", 0), (4096, 9728, 896, "swiglu", 0),
    (1000, 9728, 896, "swiglu", 256), (257, 896, 896, "resid", 224), (700, 512, 2048, "bias_resid", 256),
    (300, 512, 128, "none", 256), (5000, 896, 128, "resid", 224)])
@pytest.mark.parametrize("knob", ["ring", "spread2", "store_wait", "ring+store_wait"])
def test_linear_h3_ring_bit_identical(M, N, K, epi, tile, knob):
    """The paired-B h3 GEMMs on the three-slot A ring (DMA three K-tiles ahead, opt-in) and / or with a full tile's
    last epilogue stores left in flight across the next tile's first wait equal the default kernel bit for bit: same
    MFMA order, only the staging and the waits change (partial tiles, one K pair, many tiles per workgroup)."""
    x = rnd(M, K, seed=20)
    w = rnd(N, K, s=1 / math.sqrt(K), seed=21).to(torch.bfloat16).float()
    b = rnd(N, s=0.1, seed=22).to(DEV) if "bias" in epi else None
    r = rnd(M, N, seed=23).to(DEV) if "resid" in epi else None
    act = {"swiglu": "swiglu_il"}.get(epi)
    sx = R.h3_scale(x.abs().max().item())
    w3, sw = R.h3_weight(w)
    a3, w3 = R.h3_act(x, sx).to(DEV), w3.to(DEV)
    out = {}
    ops.set_gemm_tile(tile)
    try:
        for on in (0, 1):
            _knob(knob, on)
            out[on] = ops.linear_h3(a3, w3, 1.0 / (sx * sw), b, r, act, out_scale=1.0)
        torch.cuda.synchronize()
    finally:
        _knob(knob, -1)
        ops.set_gemm_tile(0)
    assert torch.equal(out[0], out[1])


def _knob(knob: str, on: int) -> None:
    """on: 1 the variant, 0 the two-buffer kernels with draining waits, -1 the defaults."""
    ring = {"ring": 111, "ring+store_wait": 111, "spread2": 222}.get(knob)
    ops.set_gemm_ring(-1 if on < 0 else ring * on if ring else 0)
    ops.set_gemm_store_wait(on if "store_wait" in knob else (-1 if on < 0 else 0))


@pytest.mark.parametrize("knob", ["ring", "spread2", "store_wait"])
def test_full_model_ring_identical(knob):
    """Qwen2-0.5B fp32 mode (QKV, O-proj, gate/up, down and the LSE head all paired-B): the three-slot A ring / the
    store-tolerant post-epilogue wait equal the default kernels bit for bit on the final hidden state and row NLL."""
    from llm_inference_in_distributed_edge_networks_amd.eval.data import synthetic_stream
    from llm_inference_in_distributed_edge_networks_amd.eval.windows import batches, sliding_windows
    from llm_inference_in_distributed_edge_networks_amd.models import DecoderLM, get_config
    cfg = get_config("qwen2-0.5b")
    S = 512
    toks = synthetic_stream(S * 20, cfg.vocab_size, 0)
    b = next(batches(toks, [w for w in sliding_windows(toks.shape[1], S, 32) if w.length == S][:16], 16)).to(DEV)
    m = DecoderLM.random_init(cfg, 0, device=DEV, dtype=torch.float32, values=torch.bfloat16)
    out = {}
    try:
        for on in (0, 1):
            _knob(knob, on)
            x = m.forward_hidden(b.ids)
            out[on] = (x.clone(), m.row_nll(x, b.rows, b.targets).clone())
    finally:
        _knob(knob, -1)
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])


@pytest.mark.parametrize("codec", ["mxfp4", "mxfp8", "mixed_mxfp4_mxfp8", "mxfp4_keep"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_mx_codecs_gpu_equal_cpu(codec, dtype):
    """gfx950 scaled converts (v_cvt_scalef32_pk_*) decode to exactly the CPU oracle's values."""
    B, S, H = 3, 256, 896
    x = (rnd(B * S, H, seed=80) * 3).to(dtype)
    x[:, 5] *= 40
    imp = torch.rand(B, S, generator=torch.Generator().manual_seed(81))
    spec = C.get_codec(codec)
    m_cpu, L = C.encode(x.float(), spec, B, S, 0.5, imp)
    m_gpu, L2 = C.encode(x.to(DEV), spec, B, S, 0.5, imp.to(DEV))
    y_cpu = C.decode(m_cpu, spec, L, torch.float32)
    y_gpu = C.decode(m_gpu, spec, L2, dtype).float().cpu()
    if dtype == torch.float32:
        assert torch.equal(y_gpu, y_cpu)
    else:   # bf16 activations: the hi class is bf16 on the GPU, the MX values are exact in bf16 or rounded once
        assert (y_gpu - y_cpu).abs().max() <= 0.01 * y_cpu.abs().max()


# ---- discriminating whole-model checks: final hidden state, peaked-output NLL, and their sensitivity ------------
# (reference oracle: the monolithic fp32 model, Experiments/Qwen2-0.5B/qwen_layer_wise.py:78-104)
HIDDEN_TOL, NLL_TOL = 1e-5, 3e-6     # measured clean: <= 1.9e-6 / 5.7e-7; 1e-4-perturbed: >= 2.3e-5 / 6.0e-6


def _model(cfg, seed, dev, values, head_scale):
    """Random model of the exact architecture; ``head_scale`` multiplies the LM head (a power of two, so bf16 / fp16
    values stay exact): logits then spread over tens of nats, the output distribution is peaked and the per-row NLL
    moves with the hidden state instead of sitting at ~ln |V| (std-0.02 random heads give a near-uniform softmax)."""
    from llm_inference_in_distributed_edge_networks_amd.models import DecoderLM
    m = DecoderLM.random_init(cfg, seed, device=dev, dtype=torch.float32, values=values, h3=False)
    w = m.w
    w["head"] = w["head"] * head_scale
    return DecoderLM(cfg, w, dev, torch.float32)


def _hidden_and_nll(m, b):
    from llm_inference_in_distributed_edge_networks_amd.eval.windows import window_nll
    x = m.forward_hidden(b.ids)
    rows = m.row_nll(x, b.rows, b.targets)
    return x.double().cpu(), rows.double().cpu(), window_nll(rows, b).double().cpu()


def _l2(a, b):
    return float((a - b).norm() / b.norm())


class _PerturbOneGemm:
    """Wraps ops.linear_h3: the ``which``-th fp32 GEMM of a forward gets its product scaled by (1 + eps)."""

    def __init__(self, which, eps):
        self.which, self.eps, self.n, self.orig = which, eps, 0, ops.linear_h3

    def __call__(self, a3, w3, alpha, *args, **kw):
        self.n += 1
        if self.n == self.which:
            alpha = alpha * (1.0 + self.eps)
        return self.orig(a3, w3, alpha, *args, **kw)


@pytest.mark.parametrize("name,B,S,values", [("qwen2-0.5b", 2, 512, torch.bfloat16), ("qwen2-0.5b", 1, 512, None),
                                            ("pythia-70m", 1, 2048, torch.float16)])
def test_full_model_hidden_state_and_peaked_nll(name, B, S, values, monkeypatch):
    """GPU fp32 mode vs the CPU fp32 model (same weights, same windows), whole model (24-layer Qwen2-0.5B, 6-layer
    Pythia-70M): the final hidden state within 1e-5 relative L2 and, with a peaked output distribution (row NLLs
    spread over tens of nats), the per-row NLL of every scored row within 3e-6 relative L2.  Sensitivity: the same checks run on a GPU forward whose layer-3
    output projection is perturbed by 1e-4 relative must FAIL both tolerances (else they could not see an error of
    that size)."""
    from llm_inference_in_distributed_edge_networks_amd.eval.data import synthetic_stream
    from llm_inference_in_distributed_edge_networks_amd.eval.windows import batches, sliding_windows
    from llm_inference_in_distributed_edge_networks_amd.models import get_config
    cfg = get_config(name)
    toks = synthetic_stream(S * 4, cfg.vocab_size, 5)
    wins = [w for w in sliding_windows(toks.shape[1], S, 32) if w.length == S][:B]
    b = next(batches(toks, wins, B))
    xc, nc, wc = _hidden_and_nll(_model(cfg, 1, "cpu", values, 32.0), b)
    mg = _model(cfg, 1, DEV, values, 32.0)
    bg = b.to(DEV)
    xg, ng, wg = _hidden_and_nll(mg, bg)
    e_h, e_n = _l2(xg, xc), _l2(ng, nc)
    spread = float(nc.std())       # nats; ~0 for a near-uniform softmax (random head), tens of nats here
    # the (3 per_layer + 1)-th ops.linear_h3 GEMM of the forward (QKV has its own entry point): 3 per Qwen2 / NeoX
    # layer after the QKV - layer 3's O projection; 2 with RMSNorm-2 fused into the O projection (ops.linear_h3_np),
    # the O projection then has its own entry point too - layer 3's gate/up GEMM
    per_layer = 2 if (cfg.arch == "qwen2" and mg.fuse_norm_f32) else 3
    pert = _PerturbOneGemm(3 * per_layer + 1, 1e-4)
    monkeypatch.setattr(ops, "linear_h3", pert)
    xp, npp, _ = _hidden_and_nll(mg, bg)
    monkeypatch.setattr(ops, "linear_h3", pert.orig)
    p_h, p_n = _l2(xp, xc), _l2(npp, nc)
    print(f"{name} values={values}: row-NLL spread {spread:.1f} nats (mean {float(nc.mean()):.1f}, ln|V| "
          f"{math.log(cfg.vocab_size):.1f}); clean: hidden {e_h:.2e}, "
          f"row NLL {e_n:.2e}; layer-3 O-proj x (1 + 1e-4): hidden {p_h:.2e}, row NLL {p_n:.2e}")
    assert spread > 1.0
    assert e_h < HIDDEN_TOL and e_n < NLL_TOL
    assert p_h > HIDDEN_TOL and p_n > NLL_TOL, "the tolerances do not detect a 1e-4 GEMM perturbation"
