"""fp32 reference ops: layouts and identities the HIP kernels rely on."""
import math

import pytest
import torch

from llm_inference_in_distributed_edge_networks_amd import ops
from llm_inference_in_distributed_edge_networks_amd.ops import reference as R


def test_interleave_roundtrip():
    g, u = torch.randn(64, 32), torch.randn(64, 32)
    w = R.interleave_gate_up(g, u)
    x = torch.randn(5, 32)
    gg, uu = R.deinterleave_gate_up(x @ w.t())
    assert torch.allclose(gg, x @ g.t(), atol=1e-5) and torch.allclose(uu, x @ u.t(), atol=1e-5)


def test_swiglu_linear():
    g, u = torch.randn(32, 16), torch.randn(32, 16)
    x = torch.randn(4, 16)
    y = R.linear(x, R.interleave_gate_up(g, u), act="swiglu_il")
    assert torch.allclose(y, torch.nn.functional.silu(x @ g.t()) * (x @ u.t()), atol=1e-5)


def test_rope_tables_match_hf():
    from transformers import Qwen2Config
    from transformers.models.qwen2.modeling_qwen2 import Qwen2RotaryEmbedding
    hc = Qwen2Config(hidden_size=256, num_attention_heads=4, rope_theta=1e6, max_position_embeddings=128)
    rot = Qwen2RotaryEmbedding(hc)
    cos, sin = rot(torch.zeros(1, 1, 64), torch.arange(100).view(1, -1))
    c, s = R.rope_tables(128, 64, 1e6)
    assert torch.allclose(cos[0, :, :32], c[:100], atol=1e-6) and torch.allclose(sin[0, :, 32:], s[:100], atol=1e-6)


def test_attention_matches_naive_and_lse():
    B, Hq, Hkv, S = 2, 4, 2, 37
    q = torch.randn(B, Hq, S, 64) * 0.2
    k = torch.randn(B, Hkv, S, 64)
    v = torch.randn(B, Hkv, S, 64)
    vt = torch.zeros(B, Hkv, 64, R.s_pad(S))
    vt[..., :S] = v.transpose(-1, -2)
    o, lse = R.attention(q, k, vt, S, need_lse=True)
    P = R.attention_probs(q, k, S)
    ref = (P @ v.repeat_interleave(2, 1)).permute(0, 2, 1, 3).reshape(B * S, -1)
    assert torch.allclose(o, ref, atol=1e-5)
    assert torch.allclose(R.attn_colsum(q, k, lse, S), P.sum(-2), atol=1e-5)
    assert torch.allclose(R.attn_lastrow(q, k, S), P[:, :, -1], atol=1e-6)
    assert torch.allclose(P.sum(-2).sum(-1), torch.full((B, Hq), float(S)), atol=1e-3)


def test_head_nll():
    h, w = torch.randn(7, 16), torch.randn(50, 16)
    t = torch.randint(0, 50, (7,))
    ref = torch.nn.functional.cross_entropy(h @ w.t(), t, reduction="none")
    assert torch.allclose(R.head_nll(h, w, t), ref, atol=1e-5)


def test_head_combine_cpu():
    x = torch.rand(2, 3, 10)
    w = torch.tensor([1.0, -2.0, 0.5])
    assert torch.allclose(ops.head_combine(x, w, 0.1), 0.1 * (x * w.view(1, 3, 1)).sum(1))


def test_native_library_exports_every_bound_entry_point():
    """Every ctypes signature in ops/_native.py names a symbol of the in-tree library build (a stale entry fails
    every GPU op at load time)."""
    import ctypes
    import os

    from llm_inference_in_distributed_edge_networks_amd.ops import _native
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("kernel library not built")
    L = ctypes.CDLL(_native.LIB_PATH)
    assert [n for n in _native._SIGS if not hasattr(L, n)] == []


def test_x6_three_plane_activation_layout():
    """3-plane X6 activations [a0|a1|a2] expand to the A' K-concatenation the GEMM reads (blocks 2 0 1 1 0 0), and
    A' @ B'^T over the six bf16 products is fp32-accurate."""
    import torch

    from llm_inference_in_distributed_edge_networks_amd.ops import reference as R
    g = torch.Generator().manual_seed(0)
    x, w = torch.randn(64, 128, generator=g), torch.randn(96, 128, generator=g) / 11
    a3 = R.x6_act(x)
    assert a3.shape == (64, 384) and a3.dtype == torch.bfloat16
    assert torch.equal(R.x6_to_f32(a3), (a3[:, :128].float() + a3[:, 128:256].float()) + a3[:, 256:].float())
    assert (R.x6_to_f32(a3) - x).abs().max() <= 1e-6 * x.abs().max()
    ap = R.x6_expand(a3)
    for j, p in enumerate(R.X6_APLANES):
        assert torch.equal(ap[:, 128 * j:128 * (j + 1)], a3[:, 128 * p:128 * (p + 1)])
    y = ap.double() @ R.x6_weight(w).double().t()
    ref = x.double() @ w.double().t()
    assert ((y - ref).abs().max() / ref.abs().max()) < 1e-6
    assert torch.allclose(R.x6w_to_f32(R.x6_weight(w)), w, rtol=0, atol=1e-6)
