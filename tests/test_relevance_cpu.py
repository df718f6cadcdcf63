"""AttnLRP rules (own re-implementation of the lxt rule set used by Experiments/Relevance/main.py)."""
import torch
import pytest

from llm_inference_in_distributed_edge_networks_amd.models import TINY_NEOX, TINY_QWEN2, DecoderLM
from llm_inference_in_distributed_edge_networks_amd.relevance.attnlrp import (_IdentityAct, _UniformMatmul,
                                                                              _UniformMul, head_relevance,
                                                                              normalize_per_layer)


def _gxi(fn, *xs):
    xs = [x.clone().requires_grad_(True) for x in xs]
    y = fn(*xs)
    g = torch.randn_like(y)
    (y * g).sum().backward()
    return float((y * g).sum().detach()), sum(float((x * x.grad).sum().detach()) for x in xs)


def test_rules_conserve_relevance():
    a, b = torch.randn(5, 7), torch.randn(5, 7)
    out, inp = _gxi(_UniformMul.apply, a, b)
    assert abs(out - inp) < 1e-4
    out, inp = _gxi(lambda x: _IdentityAct.apply(x, "silu"), a)
    assert abs(out - inp) < 1e-4
    out, inp = _gxi(lambda x: _IdentityAct.apply(x, "gelu"), a)
    assert abs(out - inp) < 1e-4
    out, inp = _gxi(_UniformMatmul.apply, torch.randn(3, 4, 6), torch.randn(3, 6, 5))
    assert abs(out - inp) < 1e-3


def test_head_relevance_shapes_and_normalisation():
    for cfg in (TINY_QWEN2, TINY_NEOX):
        m = DecoderLM.random_init(cfg, 0, std=0.05)
        ids = torch.randint(0, cfg.vocab_size, (1, 40), generator=torch.Generator().manual_seed(0))
        rel, in_rel, seed = head_relevance(m, ids)
        assert rel.shape == (cfg.num_layers, cfg.num_heads) and torch.isfinite(rel).all()
        w = normalize_per_layer(rel)
        assert torch.allclose(w.sum(-1), torch.ones(cfg.num_layers), atol=1e-3)
        rel2, _, _ = head_relevance(m, ids)
        assert torch.allclose(rel, rel2)


def test_output_identity_equals_probability_hook():
    for cfg in (TINY_QWEN2, TINY_NEOX):
        m = DecoderLM.random_init(cfg, 3, std=0.05)
        ids = torch.randint(0, cfg.vocab_size, (1, 48), generator=torch.Generator().manual_seed(1))
        r_probs, _, _ = head_relevance(m, ids, via_probs=True)
        r_out, _, _ = head_relevance(m, ids)
        assert torch.allclose(r_probs, r_out, rtol=1e-4, atol=1e-6)


def test_engine_equals_autograd_oracle():
    """Explicit-backward RelevanceEngine (the production pass, batched) == autograd AttnLRP, per window."""
    from llm_inference_in_distributed_edge_networks_amd.relevance.engine import RelevanceEngine
    for cfg in (TINY_QWEN2, TINY_NEOX):
        m = DecoderLM.random_init(cfg, 3, std=0.05)
        ids = torch.randint(0, cfg.vocab_size, (3, 56), generator=torch.Generator().manual_seed(1))
        rel, in_rel, mx = RelevanceEngine(m).head_relevance(ids)
        assert rel.shape == (3, cfg.num_layers, cfg.num_heads)
        for b in range(3):
            r0, in0, mx0 = head_relevance(m, ids[b:b + 1])
            assert torch.allclose(rel[b], r0, rtol=1e-4, atol=1e-5)
            assert abs(float(in_rel[b]) - float(in0)) < 1e-3 * max(1.0, abs(float(in0)))
            assert abs(float(mx[b]) - float(mx0)) < 1e-4


def test_lrp_reference_ops_match_autograd():
    """The reference LRP attention backward == autograd through the uniform / softmax rules."""
    from llm_inference_in_distributed_edge_networks_amd.ops import reference as R
    from llm_inference_in_distributed_edge_networks_amd.relevance.attnlrp import _Softmax
    g = torch.Generator().manual_seed(0)
    B, Hq, Hkv, S, D = 2, 4, 2, 40, 64
    q = torch.randn(B, Hq, S, D, generator=g) * 0.3
    k = torch.randn(B, Hkv, S, D, generator=g) * 0.3
    v = torch.randn(B, Hkv, S, D, generator=g)
    dO = torch.randn(B * S, Hq * D, generator=g)
    qa, ka, va = (t.clone().requires_grad_(True) for t in (q, k, v))
    kk, vv = ka.repeat_interleave(2, 1), va.repeat_interleave(2, 1)
    sc = _UniformMatmul.apply(qa, kk.transpose(-1, -2)).masked_fill(torch.ones(S, S, dtype=torch.bool).triu(1),
                                                                    float("-inf"))
    A = _Softmax.apply(sc)
    A.retain_grad()
    oh = _UniformMatmul.apply(A, vv)
    o = oh.permute(0, 2, 1, 3).reshape(B * S, Hq * D)
    (o * dO).sum().backward()
    lse = torch.logsumexp(sc.detach(), -1)
    Dl, rel, dq, dk, dv = R.lrp_attn_bwd(q, k, v, o.detach(), dO, lse)
    assert torch.allclose(rel, (A * A.grad).sum((2, 3)), rtol=1e-4, atol=1e-4)
    assert torch.allclose(dq, qa.grad, rtol=1e-4, atol=1e-5)
    assert torch.allclose(dk.view(B, Hkv, 2, S, D).sum(2), ka.grad, rtol=1e-4, atol=1e-5)
    assert torch.allclose(dv.view(B, Hkv, 2, S, D).sum(2), va.grad, rtol=1e-4, atol=1e-5)


def test_batched_autograd_and_channel_relevance():
    """head_relevance_batched (the fp32 calibration path on any device) == per-window head_relevance, and its
    channel-group relevance == the explicit engine's (want_channels)."""
    from llm_inference_in_distributed_edge_networks_amd.relevance.attnlrp import head_relevance_batched
    from llm_inference_in_distributed_edge_networks_amd.relevance.engine import RelevanceEngine
    for cfg in (TINY_QWEN2, TINY_NEOX):
        m = DecoderLM.random_init(cfg, 4, std=0.05)
        ids = torch.randint(0, cfg.vocab_size, (3, 48), generator=torch.Generator().manual_seed(2))
        rel, in_rel, mx, chan = head_relevance_batched(m, ids)
        G = cfg.hidden_size // 64
        assert chan.shape == (3, cfg.num_layers, G) and (chan >= 0).all() and (chan.sum(-1) > 0).all()
        for b in range(3):
            r0, in0, mx0 = head_relevance(m, ids[b:b + 1])
            assert torch.allclose(rel[b], r0, rtol=1e-4, atol=1e-5)
            assert abs(float(in_rel[b]) - float(in0)) < 1e-3 * max(1.0, abs(float(in0)))
            assert abs(float(mx[b]) - float(mx0)) < 1e-4
        rel_e, _, _, chan_e, sens_e = RelevanceEngine(m).head_relevance(ids, want_channels=True, want_sens=True)
        assert torch.allclose(rel_e, rel, rtol=1e-4, atol=1e-5)
        assert torch.allclose(chan_e, chan, rtol=1e-4, atol=1e-6)
        # the groups' quantization sensitivity: the explicit engine == autograd, and == its definition
        *_, sens = head_relevance_batched(m, ids, want_sens=True)
        assert sens.shape == chan.shape and (sens > 0).all()
        assert torch.allclose(sens_e, sens, rtol=1e-3, atol=1e-12)


@pytest.mark.parametrize("arch", ["qwen2", "neox"])
def test_h3_relevance_engine_cpu_equals_autograd(arch):
    """The fp32 relevance engine's op sequence (forward with saves on h3 GEMMs, explicit LRP backward on the
    transposed h3 weights with per-row gradient scales) on the CPU reference ops == the autograd oracle."""
    from llm_inference_in_distributed_edge_networks_amd.models import TINY_NEOX, TINY_QWEN2, DecoderLM
    from llm_inference_in_distributed_edge_networks_amd.relevance.attnlrp import head_relevance_batched
    from llm_inference_in_distributed_edge_networks_amd.relevance.engine_f32 import RelevanceEngineH3
    cfg = TINY_QWEN2 if arch == "qwen2" else TINY_NEOX
    m = DecoderLM.random_init(cfg, 0, h3=True)
    ids = torch.randint(0, cfg.vocab_size, (3, 96), generator=torch.Generator().manual_seed(1))
    got = RelevanceEngineH3(m).head_relevance(ids, want_channels=True)
    want = head_relevance_batched(m, ids, dtype=torch.float64)
    for n, a, b in zip(("rel", "in_rel", "seed", "chan"), got, want):
        e = float((a.double() - b).norm() / b.norm())
        assert e < 1e-5, (n, e)
