"""AttnLRP rules (own re-implementation of the lxt rule set used by Experiments/Relevance/main.py)."""
import torch

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
