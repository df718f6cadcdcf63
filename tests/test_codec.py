"""Boundary codec: wire format, reference-formula parity, property tests (hypothesis)."""
import math

import pytest
import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from llm_inference_in_distributed_edge_networks_amd import codec as C
from llm_inference_in_distributed_edge_networks_amd.codec import wire as W


def ref_q1(h, imp, ratio):
    """Reference Q1 (Experiments/Qwen2-0.5B/qwen_layer_wise.py:54-70), B=1, verbatim semantics."""
    h = h.clone()
    idx = torch.sort(imp, stable=True).indices[: int(ratio * h.size(1))]
    max_val = torch.max(torch.abs(h[:, idx, :]))
    num_levels = 16
    scaled = torch.clamp(h[:, idx, :] / max_val * (num_levels / 2 - 1), -(num_levels / 2), (num_levels / 2 - 1))
    h[:, idx, :] = torch.round(scaled) / (num_levels / 2 - 1) * max_val
    return h


@pytest.mark.parametrize("ratio", [0.25, 0.5, 0.75, 1.0])
def test_q1_bitexact_vs_reference(ratio):
    S, H = 64, 96
    h = torch.randn(1, S, H) * 2
    h[0, 3] *= 50
    imp = torch.rand(S)
    y, _ = C.fake_quant(h.view(S, H), C.get_codec("ref_int4_global"), 1, S, ratio, imp.view(1, S))
    assert torch.equal(y.view(1, S, H), ref_q1(h, imp, ratio))


def ref_channel(h, method):
    """Reference Q5/Q6 (qwen_layer_wise.py:106-152)."""
    h = h.clone()
    M = 127 if method == "channel_8" else 7
    for c in range(h.shape[2]):
        ch = h[:, :, c]
        if method in ("channel_8", "channel_4"):
            m = torch.max(torch.abs(ch))
            d = torch.round(ch / m * M) * m / M
        elif method == "channel_1_mean":
            mu = torch.mean(ch) + 1e-8
            d = torch.clamp(torch.round(ch / mu), -1, 1) * mu
        else:
            m = torch.max(torch.abs(ch))
            d = torch.clamp(torch.round(ch / m), -1, 1) * m
        h[:, :, c] = d
    return h


@pytest.mark.parametrize("method", ["channel_8", "channel_4", "channel_1_mean", "channel_1_max"])
def test_channel_codecs_vs_reference(method):
    S, H = 50, 64
    h = torch.randn(1, S, H)
    y, nb = C.fake_quant(h.view(S, H), C.get_codec(method), 1, S)
    r = ref_channel(h, method)
    assert torch.allclose(y.view(1, S, H), r, atol=1e-6, rtol=1e-5)
    codes = {"channel_8": 1, "channel_4": 0.5, "channel_1_mean": 0.25, "channel_1_max": 0.25}[method]
    assert nb >= S * H * codes


def test_passthrough_identity_and_size():
    x = torch.randn(2 * 33, 64)
    y, nb = C.fake_quant(x, C.get_codec("passthrough"), 2, 33)
    assert torch.equal(x, y)
    L = C.layout(C.get_codec("passthrough"), 2, 33, 64, 0, torch.float32)
    assert L.total == nb and L.total >= 2 * 33 * 64 * 4


def test_ratio_zero_is_identity_for_keep_codecs():
    x = torch.randn(64, 64)
    for name in ("ref_int4_global", "int4_token", "int8_token_keep"):
        y, _ = C.fake_quant(x, C.get_codec(name), 1, 64, 0.0, torch.rand(1, 64))
        assert torch.equal(x, y)


def test_header_and_layout():
    spec = C.get_codec("mixed_int4_int8")
    x = torch.randn(3 * 100, 128).to(torch.bfloat16)
    msg, L = C.encode(x, spec, 3, 100, 0.5, torch.rand(3, 100))
    hdr = msg[:32].view(torch.int32).tolist()
    assert hdr == [W.MAGIC, W.VERSION, spec.cid, 3, 100, 128, 50, W.FMT_INT8]
    assert L.total == msg.numel() and all(o % 16 == 0 for o in (L.off_mask, L.off_scale, L.off_hi, L.off_lo))
    # int8 rows + int4 rows + scales + mask
    assert L.total >= 3 * (50 * 128 + 50 * 64) + 3 * 100 * 4


def test_select_mask_is_k_least_important_stable():
    imp = torch.tensor([[0.5, 0.1, 0.1, 0.9, 0.0, 0.3]])
    lo = C.select_mask(imp, 3)
    assert lo.tolist() == [[False, True, True, False, True, False]]
    lo2 = C.select_mask(torch.tensor([[0.2, 0.2, 0.2, 0.2]]), 2)   # ties by position
    assert lo2.tolist() == [[True, True, False, False]]


def test_mask_words_roundtrip():
    lo = torch.rand(3, 130) > 0.5
    w = W._mask_words(lo, 6)
    assert torch.equal(W._words_to_mask(w, 130), lo)


@settings(max_examples=40, deadline=None)
@given(S=st.integers(2, 80), H=st.sampled_from([32, 64, 96]), ratio=st.floats(0, 1),
       name=st.sampled_from(["int4_token", "mixed_int4_int8", "int8_token", "mixed_int2_int8", "int8_token_keep"]),
       seed=st.integers(0, 10_000))
def test_per_token_roundtrip_error_bound(S, H, ratio, name, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(S, H, generator=g) * torch.rand(S, 1, generator=g) * 10
    spec = C.get_codec(name)
    imp = torch.rand(1, S, generator=g)
    y, _ = C.fake_quant(x, spec, 1, S, ratio, imp)
    k = W.num_lo(spec, ratio, S)
    lo = C.select_mask(imp, k)[0] if spec.uses_ratio else torch.zeros(S, dtype=torch.bool)
    for is_lo, qmax in ((True, spec.qmax_lo), (False, spec.qmax_hi)):
        sel = lo if is_lo else ~lo
        if sel.sum() == 0:
            continue
        err = (y[sel] - x[sel]).abs().amax(-1)
        if qmax == 0:                               # native rows are exact
            assert err.max() == 0
        else:
            bound = x[sel].abs().amax(-1) / qmax * 0.5 * (1 + 1e-5) + 1e-7
            if qmax == 1:
                bound = x[sel].abs().amax(-1)        # ternary: |x - q*m| <= m/2 .. m
            assert (err <= bound + 1e-6).all()


@settings(max_examples=30, deadline=None)
@given(S=st.integers(1, 70), ratio=st.floats(0, 1), seed=st.integers(0, 1000))
def test_lo_count_is_reference_truncation(S, ratio, seed):
    spec = C.get_codec("mixed_int4_int8")
    x = torch.randn(S, 32)
    msg, L = C.encode(x, spec, 1, S, ratio, torch.rand(1, S))
    words = msg[L.off_mask:L.off_mask + L.mw * 4].view(torch.int32).view(1, -1)
    assert int(W._words_to_mask(words, S).sum()) == int(ratio * S) == L.k


def test_compression_ordering():
    B, S, H = 1, 512, 896
    bpt = {n: C.message_bytes(C.get_codec(n), B, S, H, 0.5) / S for n in C.CODECS}
    assert bpt["passthrough"] > bpt["ref_int4_global"] > bpt["int8_token"] > bpt["mixed_int4_int8"] > \
        bpt["mixed_int2_int8"]
    assert abs(bpt["passthrough"] - 2 * H) < 2


def test_select_mask_nan_and_ties():
    """Selection order = stable ascending sort with NaN last and -0 == +0 (what the GPU bitonic kernel does)."""
    imp = torch.tensor([[0.5, float("nan"), -0.0, 0.0, 0.5, -1.0, float("inf")]])
    lo = C.wire.select_mask(imp, 4)
    assert lo.tolist() == [[True, False, True, True, False, True, False]]
    assert C.wire.select_mask(imp, [6]).sum() == 6 and not C.wire.select_mask(imp, [6])[0, 1]


@pytest.mark.parametrize("mass,exp", [(1.0, 0), (0.0, 6), (-0.5, 6), (0.5, 5), (0.55, 4), (0.9, 2)])
def test_top_rho_k(mass, exp):
    """keep = first i with sum_{j<i} desc_j >= mass (pythia_model.py:92-112, B21 fixed): mass <= 0 keeps none."""
    imp = torch.tensor([[0.05, 0.5, 0.1, 0.2, 0.1, 0.05]])   # desc 0.5 0.2 0.1 0.1 0.05 0.05
    assert int(C.wire.top_rho_k(imp, mass)) == exp


@pytest.mark.parametrize("codec", ["ref_int4_global", "mixed_int4_int8", "int8_token_keep"])
def test_top_rho_message_roundtrip(codec):
    B, S, H = 3, 64, 128
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B * S, H, generator=g)
    imp = torch.softmax(torch.randn(B, S, generator=g) * 2, -1)
    spec = C.get_codec(codec)
    msg, L = C.encode(x, spec, B, S, 0.4, imp, selection="top_rho")
    ks = C.wire.top_rho_k(imp, 0.6)
    assert L.kvar and C.wire.message_k(msg, L).tolist() == ks.tolist()
    y = C.decode(msg, spec, L, torch.float32)
    lo = C.wire.select_mask(imp, ks)
    # hi tokens exact (fp32 rows) unless the hi class is int8; lo tokens changed
    if spec.hi_fmt == C.wire.NATIVE:
        assert torch.equal(y.view(B, S, H)[~lo], x.view(B, S, H)[~lo])
    # same result as the fixed-k codec applied window by window with that window's k
    for b in range(B):
        yb, _ = C.fake_quant(x.view(B, S, H)[b], spec, 1, S, importance=imp[b:b + 1], k=int(ks[b]))
        if codec != "ref_int4_global":
            assert torch.equal(yb, y.view(B, S, H)[b])
    kt = int(ks.sum())
    assert C.wire.message_payload(msg, L) == L.payload_bytes(kt) <= L.total


def test_mx_formats_oracle():
    """OCP MX rows: E8M0 block scale 2^(floor(log2 amax) - emax); E2M1 / E4M3 round-to-nearest-even, saturating."""
    x = torch.tensor([[0.0, 0.25, 0.5, 0.75, 1.0, 1.25, 1.5, 2.5, 3.0, 5.0, 6.0, 7.0, -1.0, -3.5, 100.0, 0.3] * 2])
    y4, nb4 = C.fake_quant(x, C.get_codec("mxfp4"), 1, 1)
    # amax 100 -> scale 2^(6 - 2) = 16: 100/16 = 6.25 -> 6 (96); 7/16 -> 0.5 (8); 5/16 = 0.3125 -> 0.5 (8)
    assert y4[0, :16].tolist() == [0, 0, 0, 0, 0, 0, 0, 0, 0, 8, 8, 8, 0, 0, 96, 0]
    y8, nb8 = C.fake_quant(x, C.get_codec("mxfp8"), 1, 1)
    assert y8[0, 14] == 96 and y8[0, 15] == 0.3125 and torch.equal(y8[0, :14], x[0, :14])
    assert nb4 > 32 // 2 and nb8 > 32


@pytest.mark.parametrize("codec", ["mxfp4", "mxfp8", "mixed_mxfp4_mxfp8", "mxfp4_keep"])
def test_mx_codecs_error_and_bytes(codec):
    g = torch.Generator().manual_seed(0)
    B, S, H = 2, 64, 256
    x = torch.randn(B * S, H, generator=g)
    x[:, 7] *= 50          # an outlier channel: block scales confine it to its 32-channel block
    imp = torch.rand(B, S, generator=g)
    spec = C.get_codec(codec)
    y, nb = C.fake_quant(x, spec, B, S, 0.5, imp)
    err = ((y - x) ** 2).mean() / (x ** 2).mean()
    assert err < (0.03 if "fp4" in codec else 0.002)
    bits = 8 * nb / (B * S * H)
    assert bits < {"mxfp4": 4.6, "mxfp8": 8.6, "mixed_mxfp4_mxfp8": 6.6, "mxfp4_keep": 18.5}[codec]
    # block scaling beats one per-token scale under the outlier channel at equal nominal width
    if codec == "mxfp4":
        yt, _ = C.fake_quant(x, C.get_codec("int4_token"), B, S, 1.0, imp)
        assert err < ((yt - x) ** 2).mean() / (x ** 2).mean()


@pytest.mark.parametrize("model", ["linear", "mse"])
def test_group_bits_allocation(model):
    from llm_inference_in_distributed_edge_networks_amd.codec.wire import GROUP_BITS, allocate_group_bits
    rel = [0.30, 0.01, 0.20, 0.02, 0.25, 0.01, 0.10, 0.11]
    bits = allocate_group_bits(rel, 4.0, model=model)
    assert sum(bits) == 4 * len(rel) and set(bits) <= ({2, 4, 8} if model == "linear" else set(GROUP_BITS))
    order = sorted(range(len(rel)), key=lambda g: -rel[g])
    # more relevant groups never get fewer bits than less relevant ones
    assert all(bits[order[i]] >= bits[order[i + 1]] for i in range(len(rel) - 1)), bits
    assert allocate_group_bits([1.0] * 14, 4.0, model=model) == (4,) * 14
    assert allocate_group_bits([0.0] * 6, 2.0, model=model) == (2,) * 6
    assert sum(allocate_group_bits(rel, 3.0, model=model)) <= 3 * len(rel)


def test_group_bits_mse_model():
    """The MSE allocation: the error of b bits is W / qmax_b^2 (qmax 1, 3, 7, 15, 31, 127), so a step pays where the
    sensitivity ratio beats the ~5x error drop of the next bit; the plan minimises sum_g W_g / qmax^2 at the budget
    (checked against every plan of two groups), and a 1.2x spread - the surrogate model's relevance spread - stays
    uniform at 4 bits while an outlier-sized (100x) group takes bits from the others."""
    import itertools
    from llm_inference_in_distributed_edge_networks_amd.codec.wire import GROUP_BITS, allocate_group_bits
    q = {b: (1 << (b - 1)) - 1 for b in GROUP_BITS}
    assert allocate_group_bits([1.0, 1.2, 1.1, 1.0], 4.0) == (4, 4, 4, 4)
    hot = allocate_group_bits([100.0, 1.0, 1.0, 1.0], 4.0)
    assert hot[0] > 4 and min(hot[1:]) < 4 and sum(hot) == 16
    for w in ([50.0, 1.0], [1.0, 7.0], [3.0, 3.0], [400.0, 0.5]):
        for avg in (3.0, 4.0, 5.0):
            got = allocate_group_bits(w, avg)
            err = lambda p: sum(wi / q[b] ** 2 for wi, b in zip(w, p))   # noqa: E731
            best = min((p for p in itertools.product(GROUP_BITS, repeat=2) if sum(p) <= avg * 2), key=err)
            assert err(got) <= err(best) * (1 + 1e-12), (w, avg, got, best)


def test_boundary_group_plan_tables(tmp_path):
    """A sensitivity table beside the relevance table switches the plan to the MSE allocation over it."""
    import json
    from llm_inference_in_distributed_edge_networks_amd.codec.wire import (allocate_group_bits, boundary_group_plan,
                                                                            load_group_tables)
    rel = [[1.0, 1.1, 0.9, 1.0]] * 3
    sens = [[1.0, 1.0, 1.0, 1.0], [80.0, 1.0, 1.0, 1.0], [1.0, 1.0, 1.0, 90.0]]
    (tmp_path / "channel_group_relevance.json").write_text(json.dumps(rel))
    assert load_group_tables(str(tmp_path / "channel_group_relevance.json"))["sensitivity"] is None
    assert boundary_group_plan(rel, 0, 4) == allocate_group_bits(rel[1], 4.0, model="linear")
    (tmp_path / "channel_group_sensitivity.json").write_text(json.dumps(sens))
    t = load_group_tables(str(tmp_path / "channel_group_relevance.json"))
    assert boundary_group_plan(t, 0, 4) == allocate_group_bits(sens[1], 4.0) and boundary_group_plan(t, 0, 4)[0] > 4
    assert boundary_group_plan(t, 1, 4)[3] > 4 and boundary_group_plan(None, 1, 4) == (4, 4, 4, 4)
    # no table: the uniform plan at any width of the ladder (3 bits included, not a 4 / 2 split)
    assert boundary_group_plan(None, 1, 4, 3.0) == (3, 3, 3, 3)


def test_boundary_group_relevance_rows():
    """Boundary after layer L -> the table row of the stream entering L + 1; after the LAST layer (the reference's
    layer 23 of 24) the table's last row - the quality sweep at boundary 23 indexed past the table before."""
    from llm_inference_in_distributed_edge_networks_amd.codec.wire import boundary_group_relevance
    table = [[float(10 * i + g) for g in range(3)] for i in range(24)]
    assert boundary_group_relevance(table, 11, 3) == table[12]
    assert boundary_group_relevance(table, 22, 3) == table[23]
    assert boundary_group_relevance(table, 23, 3) == table[23]
    assert boundary_group_relevance(None, 23, 3) == [1.0, 1.0, 1.0]


@pytest.mark.parametrize("name", ["rgroup", "mixed_rgroup_int8"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("plan", [(8, 2, 4, 4), (3, 5, 6, 2), (6, 3, 8, 5)])
def test_group_codec_roundtrip(name, dtype, plan):
    from llm_inference_in_distributed_edge_networks_amd.codec.wire import with_plan
    B, S, H = 2, 48, 256
    g = torch.Generator().manual_seed(5)
    x = (torch.randn(B * S, H, generator=g) * 2).to(dtype)
    x[:, 64:128] *= 10          # a loud group
    imp = torch.rand(B, S, generator=g)
    spec = with_plan(C.get_codec(name), plan)
    msg, L = C.encode(x, spec, B, S, 0.5, imp)
    assert L.plan == plan and L.total == msg.numel()
    assert bytes(msg[L.off_plan:L.off_plan + 4].tolist()) == bytes(plan)
    y = C.decode(msg, spec, L, torch.float32)
    xf = x.float()
    lo = torch.ones(B * S, dtype=torch.bool) if name == "rgroup" else C.wire.select_mask(imp, S // 2).reshape(-1)
    for gi, b in enumerate(plan):
        blk = slice(64 * gi, 64 * gi + 64)
        qmax = (1 << (b - 1)) - 1
        step = xf[lo][:, blk].abs().amax(-1, keepdim=True) / qmax
        assert ((y[lo][:, blk] - xf[lo][:, blk]).abs() <= step / 2 + 1e-6).all(), gi
    if name == "mixed_rgroup_int8":
        step = xf[~lo].abs().amax(-1, keepdim=True) / 127
        assert ((y[~lo] - xf[~lo]).abs() <= step / 2 + 1e-6).all()
    # row bytes: codes 8 * sum(bits) + 4 scale bytes per group
    assert L.row_bytes(C.wire.FMT_GRP) == 8 * sum(plan) + 16
    # default plan without relevance: 4 bits everywhere
    L4 = C.layout(C.get_codec(name), B, S, H, S // 2 if name != "rgroup" else 0, dtype)
    assert L4.plan == (4, 4, 4, 4)


# sha1 prefixes of the CPU oracle's messages for a fixed input (B 2, S 128, H 896, ratio 0.5; head-group plan
# 2,4,8,4,4,2,8,4,4,4,2,8,4,4): the wire format of every codec, pinned - identical to round 4's tree when taken
WIRE_FINGERPRINTS = {
    "channel_1_max": (64576, "7dd6daea9df2e70e"),
    "channel_1_mean": (64576, "e6e44f6621c8a0da"),
    "channel_4": (121920, "53e7214e1d216a68"),
    "channel_8": (236608, "8b3fc6c69b72de9b"),
    "int4_token": (517184, "fff48e3c9ad2e77b"),
    "int8_token": (230464, "aabcbc228d1b0ee3"),
    "int8_token_keep": (574528, "6f7852e159488c62"),
    "mixed_int2_int8": (144448, "c1e854f4598cae86"),
    "mixed_int4_int8": (173120, "9fea4432e6d76a0c"),
    "mixed_mxfp4_mxfp8": (179264, "6b22e50680302847"),
    "mixed_rgroup_int8": (186448, "deaeac663805b663"),
    "mxfp4": (121920, "5c658c6ec1c707ad"),
    "mxfp4_keep": (519744, "e1df63008ca1bf20"),
    "mxfp8": (236608, "9f69368d50b1cc8d"),
    "passthrough": (917568, "9565e5c72b2b360c"),
    "ref_int4_global": (516176, "0b749fe758cea6cf"),
    "rgroup": (141392, "9adc7787e6ad8fa1"),
}


def test_wire_format_fingerprints():
    import hashlib
    from llm_inference_in_distributed_edge_networks_amd.codec import wire as W
    torch.manual_seed(0)
    B, S, H = 2, 128, 896
    x = (torch.randn(B * S, H) * torch.logspace(-2, 2, H)).float()
    imp = torch.rand(B, S)
    for name, (n, h) in WIRE_FINGERPRINTS.items():
        spec = W.CODECS[name]
        if W.needs_plan(spec):
            spec = W.with_plan(spec, (2, 4, 8, 4, 4, 2, 8, 4, 4, 4, 2, 8, 4, 4))
        msg, _ = W.encode(x, spec, B, S, 0.5, imp)
        assert msg.numel() == n and hashlib.sha1(msg.numpy().tobytes()).hexdigest()[:16] == h, name
