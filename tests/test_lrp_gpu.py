"""AttnLRP relevance kernels (csrc/lrp.hip) and the batched RelevanceEngine on gfx950 vs the fp32 oracle."""
import pytest
import torch

from llm_inference_in_distributed_edge_networks_amd import ops
from llm_inference_in_distributed_edge_networks_amd.models import TINY_NEOX, TINY_QWEN2, DecoderLM
from llm_inference_in_distributed_edge_networks_amd.ops import reference as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rnd(*shape, s=1.0, seed=0, dtype=torch.bfloat16):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * s).to(dtype)


def rel_err(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    assert torch.isfinite(a).all()
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


@pytest.mark.parametrize("B,Hq,Hkv,S", [(2, 14, 2, 512), (1, 8, 8, 200), (3, 4, 2, 96), (1, 2, 1, 37)])
def test_lrp_attn_bwd(B, Hq, Hkv, S):
    q = rnd(B, Hq, S, 64, s=0.5, seed=1) * 0.125
    k = rnd(B, Hkv, S, 64, s=0.5, seed=2)
    v = rnd(B, Hkv, S, 64, seed=3)
    dO = rnd(B * S, Hq * 64, seed=4)
    vt = torch.zeros(B, Hkv, 64, R.s_pad(S), dtype=torch.bfloat16)
    vt[..., :S] = v.transpose(-1, -2)
    o, lse = R.attention(q, k, vt, S, need_lse=True)
    ref = R.lrp_attn_bwd(q, k, v, o, dO, lse)
    got = ops.lrp_attn_bwd(*(t.to(DEV) for t in (q, k, v, o, dO)), lse.float().contiguous().to(DEV))
    names = ["D", "rel", "dq", "dk", "dv"]
    for n, g_, r_ in zip(names, got, ref):
        assert g_.shape == r_.shape, n
        e = rel_err(g_, r_)
        assert e < 2e-2, f"{n}: rel err {e:.3g}"


def test_lrp_rope_pack():
    B, S, Hq, Hkv = 2, 70, 4, 2
    for rot in (64, 16):
        cos, sin = R.rope_tables(128, rot, 1e4)
        dq, dk, dv = (rnd(B, Hq, S, 64, seed=sd, dtype=torch.float32) for sd in (5, 6, 7))
        ref = R.lrp_rope_pack(dq, dk, dv, cos, sin, B, S, Hq, Hkv, rot, 0.125)
        got = ops.lrp_rope_pack(dq.to(DEV), dk.to(DEV), dv.to(DEV), cos.to(DEV), sin.to(DEV), B, S, Hq, Hkv, rot, 0.125)
        assert rel_err(got, ref) < 5e-3


def test_swiglu_and_gelu_rules():
    gu = rnd(300, 1024, seed=8)
    dm = rnd(300, 512, seed=9)
    assert rel_err(ops.swiglu_il(gu.to(DEV)), R.swiglu_il(gu)) < 1e-2
    assert rel_err(ops.lrp_swiglu_bwd(dm.to(DEV), gu.to(DEV)), R.lrp_swiglu_bwd(dm, gu)) < 1e-2
    a = rnd(300, 512, seed=10)
    assert rel_err(ops.lrp_gelu_bwd(dm.to(DEV), a.to(DEV)), R.lrp_gelu_bwd(dm, a)) < 1e-2
    x = rnd(300, 256, seed=11) * 2 + 0.5
    rs = ops.ln_rstd(x.to(DEV), 1e-5)
    assert rel_err(rs, R.ln_rstd(x, 1e-5)) < 1e-3
    dy1, dy2, res = rnd(300, 256, seed=12), rnd(300, 256, seed=13), rnd(300, 256, seed=14)
    w1, w2 = rnd(256, seed=15), rnd(256, seed=16)
    r = R.lrp_ln_bwd(dy1, rs.cpu(), w1, dy2, rs.cpu(), w2, res)
    got = ops.lrp_ln_bwd(*(t.to(DEV) for t in (dy1,)), rs, w1.to(DEV), dy2.to(DEV), rs, w2.to(DEV), res.to(DEV))
    assert rel_err(got, r) < 1e-2


def test_linear_rowscale():
    x, w = rnd(512, 1024, seed=17), rnd(256, 1024, s=0.05, seed=18)
    rs = torch.rand(512) + 0.5
    res = rnd(512, 256, seed=19)
    got = ops.linear_rowscale(x.to(DEV), w.to(DEV), rs.to(DEV), residual=res.to(DEV))
    assert rel_err(got, R._f(x) @ R._f(w).t() * rs.view(-1, 1) + R._f(res)) < 1e-2


@pytest.mark.parametrize("cfg", [TINY_QWEN2, TINY_NEOX], ids=lambda c: c.name)
def test_relevance_engine_gpu_vs_cpu(cfg):
    """bf16 HIP relevance pass vs the fp32 CPU engine (== autograd oracle) on the same weights."""
    from llm_inference_in_distributed_edge_networks_amd.relevance.engine import RelevanceEngine
    mg = DecoderLM.random_init(cfg, 3, device=DEV, dtype=torch.bfloat16, std=0.05)
    mc = DecoderLM.random_init(cfg, 3, std=0.05)
    # identical (bf16-rounded) weights on both sides
    for Lg, Lc in zip(mg.layers, mc.layers):
        for kk in Lc:
            Lc[kk] = Lg[kk].float().cpu() if kk in Lg else Lc[kk]
    for kk in ("embed", "head", "norm_w", "norm_b"):
        if mc.w.get(kk) is not None:
            mc.w[kk] = mg.w[kk].float().cpu()
    mc.layers = mc.w["layers"]
    ids = torch.randint(0, cfg.vocab_size, (4, 128), generator=torch.Generator().manual_seed(2))
    rg, ing, mxg = RelevanceEngine(mg).head_relevance(ids.to(DEV))
    rc, inc, mxc = RelevanceEngine(mc).head_relevance(ids)
    assert rel_err(mxg, mxc) < 1e-2
    # measured on MI355X (profiles/history/r03m_lrp_bf16_err.jsonl, seeds 2-4): per-head relevance <= 0.76 %, normalised
    # table <= 2.8 % (the 3.2 % of docs/RESULTS.md is the full-size Qwen2 table)
    assert rel_err(rg, rc) < 0.02, rel_err(rg, rc)
    # the calibrated table (normalised per layer over all windows) is what weighted_importance consumes
    wg, wc = rg.sum(0), rc.sum(0)
    assert rel_err(wg / wg.sum(-1, keepdim=True), wc / wc.sum(-1, keepdim=True)) < 0.04


@pytest.mark.parametrize("B,Hq,Hkv,S", [(2, 14, 2, 512), (1, 8, 8, 200), (3, 4, 2, 96), (1, 2, 1, 37)])
@pytest.mark.parametrize("scales", ["given", "derived"])
def test_lrp_attn_bwd_f32(B, Hq, Hkv, S, scales):
    """fp32 attention LRP backward vs the fp64 reference: fp32-rounding agreement of the matrix-core sweeps on scaled
    fp16 planes (three products), at the given plane scales (the engine's path: the forward attention's) or at
    scales derived from the tensors' maxima."""
    _lrp_attn_bwd_f32_case(B, Hq, Hkv, S, scales == "given")


def test_lrp_attn_bwd_dynamic_range():
    """Gradients have no a-priori bound: dO's plane scale is a power of two from its per-head maxima, so every output is
    exactly equivariant under a power-of-two scaling of dO (2^-40 and 2^+40: bit-identical after unscaling), and rows
    of dO spread over 80 binades keep the fp32-level error (on the global scale) of the unit-scale case."""
    B, Hq, Hkv, S = 1, 4, 2, 160
    f = torch.float32
    q = rnd(B, Hq, S, 64, s=0.5, seed=11, dtype=f) * 0.125
    k = rnd(B, Hkv, S, 64, s=0.5, seed=12, dtype=f)
    v = rnd(B, Hkv, S, 64, seed=13, dtype=f)
    dO = rnd(B * S, Hq * 64, seed=14, dtype=f)
    vt = torch.zeros(B, Hkv, 64, R.s_pad(S), dtype=f)
    vt[..., :S] = v.transpose(-1, -2)
    o, lse = R.attention(q, k, vt, S, need_lse=True)
    dev = [t.to(DEV) for t in (q, k, v, o)]
    lse_d = lse.float().contiguous().to(DEV)
    sc = tuple(R.h3_scale(t.abs().max().item()) for t in (q, k, v))
    base = ops.lrp_attn_bwd(*dev, dO.to(DEV), lse_d, in_scales=sc)
    for e in (-40, 40):
        got = ops.lrp_attn_bwd(*dev, (dO * 2.0 ** e).to(DEV), lse_d, in_scales=sc)
        for n, g_, b_ in zip(["D", "rel", "dq", "dk", "dv"], got, base):
            assert torch.equal(g_ * 2.0 ** -e, b_), f"{n}: not equivariant under dO x 2^{e}"
    # mixed magnitudes: dO rows over 2^-40 .. 2^40; the error measured against fp64 on the global scale
    dOm = dO * (2.0 ** torch.linspace(-40, 40, B * S).round()).view(-1, 1)
    ref = R.lrp_attn_bwd(q.double(), k.double(), v.double(), o.double(), dOm.double(), lse.double())
    got = ops.lrp_attn_bwd(*dev, dOm.to(DEV), lse_d, in_scales=sc)
    for n, g_, r_ in zip(["D", "rel", "dq", "dk", "dv"], got, ref):
        assert rel_err(g_, r_) < 2e-6, n


def _lrp_attn_bwd_f32_case(B, Hq, Hkv, S, h3=False):
    f = torch.float32
    q = rnd(B, Hq, S, 64, s=0.5, seed=1, dtype=f) * 0.125
    k = rnd(B, Hkv, S, 64, s=0.5, seed=2, dtype=f)
    v = rnd(B, Hkv, S, 64, seed=3, dtype=f)
    dO = rnd(B * S, Hq * 64, seed=4, dtype=f)
    vt = torch.zeros(B, Hkv, 64, R.s_pad(S), dtype=f)
    vt[..., :S] = v.transpose(-1, -2)
    o, lse = R.attention(q, k, vt, S, need_lse=True)
    ref = R.lrp_attn_bwd(q.double(), k.double(), v.double(), o.double(), dO.double(), lse.double())
    sc = tuple(R.h3_scale(t.abs().max().item()) for t in (q, k, v)) if h3 else None
    got = ops.lrp_attn_bwd(*(t.to(DEV) for t in (q, k, v, o, dO)), lse.float().contiguous().to(DEV), in_scales=sc)
    for n, g_, r_ in zip(["D", "rel", "dq", "dk", "dv"], got, ref):
        assert g_.shape == r_.shape and g_.dtype == torch.float32, n
        e = rel_err(g_, r_)
        assert e < 2e-6, f"{n}: rel err {e:.3g}"
    # dk, dv summed over each GQA group (one workgroup per kv head sweeping its q heads)
    got = ops.lrp_attn_bwd(*(t.to(DEV) for t in (q, k, v, o, dO)), lse.float().contiguous().to(DEV), gqa_sum=True,
                           in_scales=sc)
    for n, g_, r_ in zip(["dk", "dv"], got[3:], ref[3:]):
        r_ = r_.view(B, Hkv, Hq // Hkv, S, 64).sum(2)
        assert g_.shape == r_.shape, n
        e = rel_err(g_, r_)
        assert e < 2e-6, f"{n} (GQA sum): rel err {e:.3g}"


def test_fp32_lrp_rule_kernels():
    """Per-row-scaled h3 outputs of the fp32 rules: planes bit-identical to the reference split (split_h3_dyn,
    rope pack) or within fp32 rounding of the rule (SwiGLU / GELU transcendentals), every row's max below 2^15."""
    f = torch.float32
    x = rnd(301, 896, seed=20, dtype=f) * torch.logspace(-6, 6, 301).view(-1, 1)
    x[7] = 0.0
    post = torch.rand(301) + 0.5
    g3, gi = ops.split_h3_dyn(x.to(DEV), post.to(DEV))
    r3, ri = R.split_h3_dyn(x, post)
    assert torch.equal(g3.cpu(), r3) and torch.equal(gi.cpu(), ri)
    assert g3.float().abs().max() < 2 ** 15
    back = R.h3_to_f32(g3.cpu()) * (gi.cpu() / post).view(-1, 1)
    assert rel_err(back, x) < 1e-7
    # SwiGLU rule
    gu, dm = rnd(97, 2 * 512, seed=21, dtype=f) * 3, rnd(97, 512, seed=22, dtype=f)
    d3, di = ops.lrp_swiglu_bwd_h3(dm.to(DEV), gu.to(DEV), post[:97].to(DEV))
    val = R.h3_to_f32(d3.cpu()) * di.cpu().view(-1, 1)
    assert rel_err(val, R.lrp_swiglu_bwd(dm.double(), gu.double()) * post[:97].double().view(-1, 1)) < 1e-6
    # GELU rule
    a = rnd(97, 512, seed=23, dtype=f) * 3
    d3, di = ops.lrp_gelu_bwd_h3(dm.to(DEV), a.to(DEV))
    assert rel_err(R.h3_to_f32(d3.cpu()) * di.cpu().view(-1, 1), R.lrp_gelu_bwd(dm.double(), a.double())) < 1e-6
    # forward activations at a fixed scale
    for act, inp in (("swiglu_il", gu), ("gelu", a)):
        got = R.h3_to_f32(ops.act_h3(inp.to(DEV), act, 2.0 ** 6).cpu(), 2.0 ** 6)   # |act| < 2^9 here
        want = R.swiglu_il(inp.double()) if act == "swiglu_il" else R.gelu(inp.double())
        assert rel_err(got, want) < 1e-6, act
    # inverse RoPE + GQA sum + pack
    B, S, Hq, Hkv = 2, 70, 4, 2
    for rot in (64, 16):
        cos, sin = R.rope_tables(128, rot, 1e4)
        dq, dk, dv = (rnd(B, Hq, S, 64, seed=sd, dtype=f) for sd in (5, 6, 7))
        want = R.lrp_rope_pack(dq.double(), dk.double(), dv.double(), cos.double(), sin.double(), B, S, Hq, Hkv,
                               rot, 0.125)
        g3, gi = ops.lrp_rope_pack_h3(dq.to(DEV), dk.to(DEV), dv.to(DEV), cos.to(DEV), sin.to(DEV), B, S, Hq, Hkv,
                                      rot, 0.125)
        assert rel_err(R.h3_to_f32(g3.cpu()) * gi.cpu().view(-1, 1), want) < 1e-6
        # from dk / dv already summed over each GQA group
        dks, dvs = (t.view(B, Hkv, Hq // Hkv, S, 64).sum(2).contiguous() for t in (dk, dv))
        g3, gi = ops.lrp_rope_pack_h3(dq.to(DEV), dks.to(DEV), dvs.to(DEV), cos.to(DEV), sin.to(DEV), B, S, Hq, Hkv,
                                      rot, 0.125)
        assert rel_err(R.h3_to_f32(g3.cpu()) * gi.cpu().view(-1, 1), want) < 1e-6
    # norm statistics, LayerNorm rule, channel-group sums
    y = rnd(300, 256, seed=24, dtype=f) * 2 + 0.5
    for center in (False, True):
        assert rel_err(ops.row_rstd(y.to(DEV), 1e-5, center), R.row_rstd(y.double(), 1e-5, center)) < 1e-6
    rs = R.row_rstd(y, 1e-5, True)
    dy1, dy2, res = (rnd(300, 256, seed=sd, dtype=f) for sd in (25, 26, 27))
    w1, w2 = rnd(256, seed=28, dtype=f), rnd(256, seed=29, dtype=f)
    got = ops.lrp_ln_bwd_f32(dy1.to(DEV), rs.to(DEV), w1.to(DEV), dy2.to(DEV), w2.to(DEV), res.to(DEV))
    assert rel_err(got, R.lrp_ln_bwd(dy1.double(), rs.double(), w1.double(), dy2.double(), rs.double(),
                                     w2.double(), res.double())) < 1e-6
    xx, dd = rnd(3 * 50, 256, seed=30, dtype=f), rnd(3 * 50, 256, seed=31, dtype=f)
    assert rel_err(ops.group_absprod(xx.to(DEV), dd.to(DEV), 3, 50), R.group_absprod(xx.double(), dd.double(), 3,
                                                                                    50)) < 1e-6
    sens = torch.empty(3, 4, device=DEV)
    ops.group_absprod(xx.to(DEV), dd.to(DEV), 3, 50, sens_out=sens)
    assert rel_err(sens, R.group_sens(xx.double(), dd.double(), 3, 50)) < 1e-6


@pytest.mark.parametrize("M,N,K,tile,bf16w", [(300, 512, 256, 0, False), (300, 512, 256, 256, True),
                                               (520, 640, 192, 0, True), (300, 640, 192, 256, False),
                                               (4096, 4096, 256, 0, True)])
def test_fp32_lrp_swiglu_gemm_epilogue(M, N, K, tile, bf16w):
    """dm GEMM + SwiGLU rule in one kernel (EPI_H3_LRP_SWIGLU) vs the fp64 rule on the fp64 product: every row within
    4e-6 of its own max (rows spanning 12 decades), planes below 2^15 at the weights' bound scale; the 128x128 and
    the persistent 256x256 kernels (forced at small M, a half-empty last column tile at N = 640, and chosen by shape
    at 4096 x 4096), three- and two-product (bf16-valued) weights."""
    f = torch.float32
    dx = rnd(M, K, seed=40, dtype=f) * torch.logspace(-6, 6, M).view(-1, 1)
    wd = rnd(K, N, seed=41, dtype=f) * 0.05      # down projection [H, I]
    wgu = rnd(2 * N, K, seed=42, dtype=f) * 0.05  # interleaved gate|up [2I, H]
    if bf16w:
        wd, wgu = wd.bfloat16().float(), wgu.bfloat16().float()
    nw = torch.rand(K, generator=torch.Generator().manual_seed(43)) + 0.5
    x = rnd(M, K, seed=44, dtype=f) * 3
    gu = (x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-6) * nw) @ wgu.t()
    post = torch.rand(M, generator=torch.Generator().manual_seed(45)) + 0.5
    c0 = ops.lrp_swiglu_scale(wd, wgu, nw)
    w3, s = R.h3_weight(wd.t().contiguous())
    a3, rinv = ops.split_h3_dyn(dx.to(DEV))
    ops.set_gemm_tile(tile)
    try:
        d3, rs = ops.linear_h3_lrp_swiglu(a3, w3.to(DEV), 1.0 / s, gu.to(DEV), c0, rinv, post=post.to(DEV))
        torch.cuda.synchronize()
    finally:
        ops.set_gemm_tile(0)
    assert d3.shape == (M, 4 * N) and float(d3.float().abs().max()) < 2 ** 15
    got = R.h3_to_f32(d3.cpu()).double() * rs.cpu().double().view(-1, 1)
    want = R.lrp_swiglu_bwd(dx.double() @ wd.double(), gu.double()) * post.double().view(-1, 1)
    row_err = (got - want).abs().amax(1) / want.abs().amax(1)
    assert float(row_err.max()) < 4e-6, float(row_err.max())   # the h3 product's own error (K terms)
    # the CPU route of the same op (the engine's CPU path) agrees
    c3, crs = R.linear_h3_lrp_swiglu(a3.cpu(), w3, 1.0 / s, gu, c0, rinv.cpu(), post)
    assert torch.equal(crs, rs.cpu())
    assert rel_err(R.h3_to_f32(c3) * crs.view(-1, 1), want) < 4e-6


@pytest.mark.parametrize("cfg", [TINY_QWEN2, TINY_NEOX], ids=lambda c: c.name)
def test_relevance_engine_h3_tiny_vs_autograd(cfg):
    """fp32 HIP relevance engine vs the autograd oracle (fp64 on the CPU, same weights)."""
    from llm_inference_in_distributed_edge_networks_amd.relevance.attnlrp import head_relevance_batched
    from llm_inference_in_distributed_edge_networks_amd.relevance.engine_f32 import RelevanceEngineH3
    mg = DecoderLM.random_init(cfg, 3, device=DEV, std=0.05)
    mc = DecoderLM.random_init(cfg, 3, std=0.05)
    ids = torch.randint(0, cfg.vocab_size, (4, 128), generator=torch.Generator().manual_seed(2))
    rg, ing, mxg, cg, sg = RelevanceEngineH3(mg).head_relevance(ids.to(DEV), want_channels=True, want_sens=True)
    rc, inc, mxc, cc, sc = head_relevance_batched(mc, ids, dtype=torch.float64, want_sens=True)
    for n, a, b in (("rel", rg, rc), ("in_rel", ing, inc), ("seed", mxg, mxc), ("chan", cg, cc), ("sens", sg, sc)):
        e = rel_err(a, b)
        assert e < 1e-5, f"{n}: {e:.3g}"


def test_fp32_calibration_table_matches_cpu_full_qwen2():
    """The reference-precision calibration on the full 24-layer Qwen2-0.5B (one 512-token window, bf16-valued random
    weights as the HF checkpoint): the fp32 HIP engine's normalised head table and channel-group table within 1e-4
    (relative L2) of the CPU fp32 autograd oracle on the same weights (measured 2e-6); the bf16 HIP engine's table
    is pinned at its measured deviation on this window (5.0 %: bf16 storage of every saved tensor)."""
    from llm_inference_in_distributed_edge_networks_amd.models import get_config
    from llm_inference_in_distributed_edge_networks_amd.relevance.attnlrp import (head_relevance_batched,
                                                                                  normalize_per_layer)
    from llm_inference_in_distributed_edge_networks_amd.relevance.engine import RelevanceEngine
    from llm_inference_in_distributed_edge_networks_amd.relevance.engine_f32 import RelevanceEngineH3
    cfg = get_config("qwen2-0.5b")
    mc = DecoderLM.random_init(cfg, 7, std=0.02, values=torch.bfloat16)
    mg = DecoderLM.random_init(cfg, 7, device=DEV, std=0.02, values=torch.bfloat16)
    ids = torch.randint(0, cfg.vocab_size, (1, 512), generator=torch.Generator().manual_seed(3))
    rc, _, _, cc = head_relevance_batched(mc, ids)
    rg, _, _, cg = RelevanceEngineH3(mg).head_relevance(ids.to(DEV), want_channels=True)
    tc = normalize_per_layer(rc.sum(0))
    e_head = rel_err(normalize_per_layer(rg.sum(0)), tc)
    e_chan = rel_err(normalize_per_layer(cg.sum(0)), normalize_per_layer(cc.sum(0)))
    e_raw = rel_err(rg, rc)
    del mg
    mb = DecoderLM.random_init(cfg, 7, device=DEV, dtype=torch.bfloat16, std=0.02)
    rb, _, _ = RelevanceEngine(mb).head_relevance(ids.to(DEV))
    e_bf16 = rel_err(normalize_per_layer(rb.sum(0)), tc)
    print(f"normalised head table vs CPU fp32: fp32 HIP engine {e_head:.2e} (raw {e_raw:.2e}), bf16 HIP engine "
          f"{e_bf16:.2e}; channel groups {e_chan:.2e}")
    assert e_head < 1e-4 and e_chan < 1e-4 and e_raw < 1e-4
    assert e_bf16 < 0.06


def test_fp32_calibration_table_matches_cpu_full_pythia():
    """The same check on the full 6-layer Pythia-70M (GPT-NeoX: parallel residual, LayerNorm rule, GELU identity
    rule, 25 % rotary), fp16-valued weights as the HF checkpoint, one 1024-token window."""
    from llm_inference_in_distributed_edge_networks_amd.models import get_config
    from llm_inference_in_distributed_edge_networks_amd.relevance.attnlrp import (head_relevance_batched,
                                                                                  normalize_per_layer)
    from llm_inference_in_distributed_edge_networks_amd.relevance.engine_f32 import RelevanceEngineH3
    cfg = get_config("pythia-70m")
    mc = DecoderLM.random_init(cfg, 4, std=0.02, values=torch.float16)
    mg = DecoderLM.random_init(cfg, 4, device=DEV, std=0.02, values=torch.float16)
    ids = torch.randint(0, cfg.vocab_size, (1, 1024), generator=torch.Generator().manual_seed(5))
    rc, _, _, cc = head_relevance_batched(mc, ids)
    rg, _, _, cg = RelevanceEngineH3(mg).head_relevance(ids.to(DEV), want_channels=True)
    e_head = rel_err(normalize_per_layer(rg.sum(0)), normalize_per_layer(rc.sum(0)))
    e_chan = rel_err(normalize_per_layer(cg.sum(0)), normalize_per_layer(cc.sum(0)))
    print(f"pythia-70m normalised head table vs CPU fp32: {e_head:.2e} (raw {rel_err(rg, rc):.2e}); channel groups "
          f"{e_chan:.2e}")
    assert e_head < 1e-4 and e_chan < 1e-4


@pytest.mark.parametrize("heavy", [100.0])
def test_fp32_lrp_swiglu_gemm_heavy_tailed_weights(heavy):
    """The fused dm GEMM + SwiGLU rule scales its planes from an a-priori bound of the weights (lrp_swiglu_scale), not
    from each row's max.  Trained checkpoints have outlier channels: here 3 of 256 channels carry 100x norm weights,
    10x gate/up columns and 100x down-projection rows (the bound grows ~10^4x).  Per-row error against the fp64 rule
    stays at the h3 product's level (CPU emulation of the same planes: 2.1e-6 at 100x, 0.85e-6 without outliers) and
    the planes stay far from both fp16 overflow and the subnormal range."""
    f = torch.float32
    M, N, K = 300, 512, 256
    dx = rnd(M, K, seed=40, dtype=f) * torch.logspace(-6, 6, M).view(-1, 1)
    wd = rnd(K, N, seed=41, dtype=f) * 0.05
    wgu = rnd(2 * N, K, seed=42, dtype=f) * 0.05
    nw = torch.rand(K, generator=torch.Generator().manual_seed(43)) + 0.5
    ch = torch.tensor([3, 77, 200])
    nw[ch] *= heavy
    wd[:, ch] *= heavy ** 0.5
    wgu[:, ch] *= heavy ** 0.5
    wd[ch, :] *= heavy
    x = rnd(M, K, seed=44, dtype=f) * 3
    gu = (x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-6) * nw) @ wgu.t()
    post = torch.rand(M, generator=torch.Generator().manual_seed(45)) + 0.5
    c0 = ops.lrp_swiglu_scale(wd, wgu, nw)
    w3, s = R.h3_weight(wd.t().contiguous())
    a3, rinv = ops.split_h3_dyn(dx.to(DEV))
    d3, rs = ops.linear_h3_lrp_swiglu(a3, w3.to(DEV), 1.0 / s, gu.to(DEV), c0, rinv, post=post.to(DEV))
    torch.cuda.synchronize()
    planes = R.h3_to_f32(d3.cpu())
    pmax = float(planes.abs().max())
    assert 2 ** 4 < pmax < 2 ** 15, pmax          # headroom both ways: no overflow, far above fp16 subnormals
    got = planes.double() * rs.cpu().double().view(-1, 1)
    want = R.lrp_swiglu_bwd(dx.double() @ wd.double(), gu.double()) * post.double().view(-1, 1)
    row_err = (got - want).abs().amax(1) / want.abs().amax(1)
    assert float(row_err.max()) < 4e-6, float(row_err.max())
