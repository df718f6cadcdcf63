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


def test_h3_two_plane_activation_layout():
    """2-plane h3 activations [hi|lo] of s x expand to the A' K-concatenation the GEMM reads (blocks 1 0 0), and
    alpha A' @ B'^T over the three fp16 products is fp32-accurate (below the fp32 GEMM's own error)."""
    import torch

    from llm_inference_in_distributed_edge_networks_amd.ops import reference as R
    g = torch.Generator().manual_seed(0)
    x, w = torch.randn(64, 896, generator=g), torch.randn(96, 896, generator=g) / 30
    s = R.h3_scale(x.abs().max().item())
    assert s * x.abs().max() <= 2 ** 15 < 2 * s * x.abs().max()
    a3 = R.h3_act(x, s)
    assert a3.shape == (64, 2 * 896) and a3.dtype == torch.float16
    assert (R.h3_to_f32(a3, s) - x).abs().max() <= 2 ** -21 * x.abs().max()
    ap = R.h3_expand(a3)
    for j, p in enumerate(R.H3_APLANES):
        assert torch.equal(ap[:, 896 * j:896 * (j + 1)], a3[:, 896 * p:896 * (p + 1)])
    w3, sw = R.h3_weight(w)
    y = ap.double() @ w3.double().t() / (s * sw)
    ref = x.double() @ w.double().t()
    e32 = ((x @ w.t()).double() - ref).norm() / ref.norm()
    assert ((y - ref).norm() / ref.norm()) < max(e32, 1e-7)
    assert (R.h3w_to_f32(w3, sw, 896) - w).abs().max() <= 2 ** -21 * w.abs().max()
    # a weight exact in fp16 after scaling (bf16 checkpoint values) -> the two-term layout [hi | hi], same product
    wb = w.to(torch.bfloat16).float()
    w2, sb = R.h3_weight(wb)
    assert w2.shape == (96, 896)
    assert torch.equal(R.h3w_to_f32(w2, sb, 896), wb)
    w3b, _ = R.h3_weight(wb, two_term=False)
    y2 = R.h3_expand(a3, 2).double() @ torch.cat([w2, w2], 1).double().t()   # the third product is exactly zero
    y3 = R.h3_expand(a3, 3).double() @ w3b.double().t()
    assert torch.allclose(y2, y3, rtol=1e-12, atol=0) and R.h3_terms(a3, w2) == 2 and R.h3_terms(a3, w3b) == 3


def test_h3_scale_keeps_fp16_range():
    from llm_inference_in_distributed_edge_networks_amd.ops import reference as R
    for b in (1e-30, 3e-5, 0.7, 1.0, 1.5, 30.0, 65504.0, 1e9):
        s = R.h3_scale(b)
        assert s * b <= 2 ** 15 < 2 * s * b or s in (2.0 ** 100, 2.0 ** -100)
    assert R.h3_scale(0.0) == 1.0 and R.h3_scale(float("inf")) == 1.0


def test_kv_plane_perm_is_the_attention_operand_order():
    """V^T plane key order (gemm.hip kv_plane_pos): key 32 s + 16 hf + 4 a + r of a 64-key tile at element
    8 (4 s + a) + 4 hf + r, a bijection on every tile; planes split2h of s x."""
    from llm_inference_in_distributed_edge_networks_amd.ops import reference as R
    perm = R.kv_plane_perm(128)
    assert sorted(perm.tolist()) == list(range(128))
    for key in range(128):
        t, kk = divmod(key, 64)
        s_, hf, a, r = kk >> 5, (kk >> 4) & 1, (kk >> 2) & 3, kk & 3
        assert perm[key] == 64 * t + 8 * (4 * s_ + a) + 4 * hf + r
    k = torch.randn(1, 2, 100, 64)
    vt = torch.zeros(1, 2, 64, 128)
    vt[..., :100] = torch.randn(1, 2, 64, 100)
    kp, vp = R.kv_planes(k, vt, 2.0 ** 3, 2.0 ** 4)
    assert kp.shape == (1, 2, 2, 100, 64) and vp.shape == (1, 2, 2, 64, 128)
    hi = (k * 8).half()
    assert torch.equal(kp[:, :, 0], hi) and torch.equal(kp[:, :, 1], (k * 8 - hi.float()).half())
    back = vp[..., perm]
    assert (back[:, :, 0].float() + back[:, :, 1].float() - vt * 16).abs().max() <= (vt * 16).abs().max() * 2 ** -20
    assert (back[:, :, 0].float() / 16 - vt).abs().max() <= vt.abs().max() * 2 ** -10
