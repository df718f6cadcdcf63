"""Own model implementations vs HF transformers (random-init tiny configs, fp32, CPU)."""
import pytest
import torch
import torch.nn.functional as F

from llm_inference_in_distributed_edge_networks_amd.models import TINY_NEOX, TINY_QWEN2, DecoderLM, get_config
from llm_inference_in_distributed_edge_networks_amd.models.configs import PYTHIA_70M, QWEN2_0_5B

from helpers import hf_neox, hf_qwen2, ours_from_hf


@pytest.mark.parametrize("cfg,mk", [(TINY_QWEN2, hf_qwen2), (TINY_NEOX, hf_neox)])
def test_logits_match_hf(cfg, mk):
    hf = mk(cfg)
    ours = ours_from_hf(cfg, hf)
    ids = torch.randint(0, cfg.vocab_size, (2, 50), generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        ref = hf(ids).logits
    got = ours.logits(ours.forward_hidden(ids)).view_as(ref)
    assert (got - ref).abs().max() < 1e-4


@pytest.mark.parametrize("cfg,mk", [(TINY_QWEN2, hf_qwen2), (TINY_NEOX, hf_neox)])
def test_row_nll_matches_hf_ce(cfg, mk):
    hf = mk(cfg)
    ours = ours_from_hf(cfg, hf)
    ids = torch.randint(0, cfg.vocab_size, (1, 64), generator=torch.Generator().manual_seed(2))
    with torch.no_grad():
        ref = F.cross_entropy(hf(ids).logits[0, :-1], ids[0, 1:], reduction="none")
    got = ours.row_nll(ours.forward_hidden(ids), torch.arange(63), ids[0, 1:])
    assert (got - ref).abs().max() < 1e-4


def test_layer_range_equals_monolithic():
    m = DecoderLM.random_init(TINY_QWEN2, 3)
    ids = torch.randint(0, 512, (2, 40))
    full = m.forward_hidden(ids)
    x = m.embed(ids)
    for i in range(2):
        x, _ = m.layer(i, x, 2, 40)
    for i in range(2, 4):
        x, _ = m.layer(i, x, 2, 40)
    assert torch.equal(x, full)


@pytest.mark.parametrize("cfg", [TINY_QWEN2, TINY_NEOX])
def test_partial_stage_weights_identical(cfg):
    full = DecoderLM.random_init(cfg, 7)
    s1 = DecoderLM.random_init(cfg, 7, layers=range(2, 4), with_embed=False)
    for i in range(2, 4):
        for k, v in full.layers[i].items():
            assert torch.equal(v, s1.layers[i][k])
    assert s1.layers[0] is None
    assert torch.equal(full.w["head"], s1.w["head"])


def test_layer_does_not_modify_input():
    m = DecoderLM.random_init(TINY_NEOX, 0)
    x = torch.randn(2 * 30, 256)
    x0 = x.clone()
    m.layer(0, x, 2, 30)
    assert torch.equal(x, x0)


def test_presets():
    q = get_config("Qwen/Qwen2-0.5B")
    assert q is QWEN2_0_5B and q.qkv_size == 1152 and q.group_size == 7
    assert 490e6 < q.num_params() < 500e6    # 494M params
    p = get_config("pythia")
    assert p is PYTHIA_70M and p.rotary_dim == 16 and p.parallel_residual
    assert 69e6 < p.num_params() < 72e6


@pytest.mark.parametrize("cfg", [TINY_QWEN2, TINY_NEOX])
def test_h3_execution_path_matches_fp32(cfg):
    """The fp32 GPU mode's op sequence (h3 split-fp16 GEMM operands, ops.*_h3) run on CPU equals plain fp32."""
    ref_m = DecoderLM.random_init(cfg, 5)
    h3_m = DecoderLM.random_init(cfg, 5, h3=True)
    ids = torch.randint(0, cfg.vocab_size, (2, 48), generator=torch.Generator().manual_seed(3))
    B, S = ids.shape
    xr, xx = ref_m.embed(ids), h3_m.embed(ids)
    for i in range(cfg.num_layers):
        xr, sr = ref_m.layer(i, xr, B, S, stats=("lastrow", "colsum"))
        xx, sx = h3_m.layer(i, xx, B, S, stats=("lastrow", "colsum"))
        assert torch.allclose(sx.lastrow, sr.lastrow, atol=1e-6) and torch.allclose(sx.colsum, sr.colsum, atol=1e-5)
    assert (xx - xr).abs().max() < 1e-4
    rows = torch.arange(S - 8, S).repeat(B) + torch.arange(B).repeat_interleave(8) * S
    tg = torch.randint(0, cfg.vocab_size, (rows.numel(),))
    assert torch.allclose(h3_m.row_nll(xx, rows, tg), ref_m.row_nll(xr, rows, tg), atol=1e-4)
    # last-layer scored-rows shortcut
    xl = h3_m.layer_rows(cfg.num_layers - 1, h3_m.forward_hidden(ids, 0, cfg.num_layers - 1), B, S, rows)
    assert torch.allclose(xl, xr.index_select(0, rows), atol=1e-4)


@pytest.mark.parametrize("cfg", [TINY_QWEN2, TINY_NEOX])
def test_h3_bounds_hold(cfg):
    """Every GEMM input of the fp32 mode stays below its bound (so s * |x| <= 2^15, inside fp16), for inputs far
    outside the trained range: huge residual streams, one-hot rows, all-equal rows."""
    from llm_inference_in_distributed_edge_networks_amd import ops
    from llm_inference_in_distributed_edge_networks_amd.models.model import _h3_bounds
    m = DecoderLM.random_init(cfg, 9)
    g = torch.Generator().manual_seed(1)
    B, S, H = 2, 40, cfg.hidden_size
    x = torch.randn(B * S, H, generator=g) * 1e4
    x[0] = 0.0
    x[0, 3] = 5e5
    x[1] = 7.0
    for i, L in enumerate(m.layers):
        bd = _h3_bounds(cfg, L)
        if cfg.arch == "qwen2":
            h = ops.rmsnorm(x, L["ln1_w"], cfg.norm_eps)
        else:
            h, h2 = ops.layernorm_dual(x, L["ln1_w"], L["ln1_b"], L["ln2_w"], L["ln2_b"], cfg.norm_eps)
        assert h.abs().max() <= bd["qkv"] * (1 + 1e-5)
        q, k, vt = ops.qkv_rope(h, L["wqkv"], L["bqkv"], m.cos, m.sin, B, S, cfg.num_heads, cfg.num_kv_heads,
                                cfg.head_dim, cfg.rotary_dim, m.q_scale)
        assert q.abs().max() <= bd["att_q"] * (1 + 1e-5) and k.abs().max() <= bd["att_k"] * (1 + 1e-5)
        assert vt.abs().max() <= bd["o"] * (1 + 1e-5)
        o, _ = ops.attention(q, k, vt, S)
        assert o.abs().max() <= bd["o"] * (1 + 1e-5)
        y = ops.linear(o, L["wo"], L.get("bo"), residual=x)
        if cfg.arch == "qwen2":
            h2 = ops.rmsnorm(y, L["ln2_w"], cfg.norm_eps)
            a = ops.linear(h2, L["wgu"], act="swiglu_il")
        else:
            a = ops.linear(h2, L["wfc"], L["bfc"], act="gelu")
        assert h2.abs().max() <= bd["mlp"] * (1 + 1e-5)
        assert a.abs().max() <= bd["down"] * (1 + 1e-5)
        x = y
