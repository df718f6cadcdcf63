"""Epilogue desync of the four-wave GEMMs (csrc/gemm.hip GemmArgs::split_h): the odd workgroups of each XCD run the
first K-tiles of their last tile first, park the raw accumulators in a persistent per-device workspace and finish
that tile last.  The accumulation order of every output is unchanged, so the result must be bit-identical to the
plain persistent walk - for every epilogue family the bench runs at the bench's own shapes (M = 32768: SwiGLU h3
planes, fp32 residual in place, QKV + RoPE + K / V^T planes; the LM-head LSE at the 2048 scored rows x the full
vocabulary), the bf16 mode's gate/up and LSE, and split points other than the default half tile.

Round 3's version of this code faulted the GPU at the bench shape and on the LSE head; the cause was its inline-asm
park / restore taking an SGPR base fresh from v_readfirstlane without the 5 wait states (docs/ARCHITECTURE.md §GEMM).
A checked build (the tuning library, EDGE_GEMM_CHECKS) also bounds-checks every segment and park area on the device.
"""
import pytest
import torch

from llm_inference_in_distributed_edge_networks_amd import ops
from llm_inference_in_distributed_edge_networks_amd.ops import reference as R
from llm_inference_in_distributed_edge_networks_amd.ops._native import lib

pytestmark = pytest.mark.gpu
DEV = "cuda"
SPLITS = (0, -1, 2, 6)


def rnd(*shape, s=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g) * s


def h3_operands(M, N, K, seed):
    x = rnd(M, K, seed=seed)
    w = (rnd(N, K, s=0.02, seed=seed + 1)).bfloat16().float()   # bf16 values: the two-product (paired-B) GEMM
    w3, sw = R.h3_weight(w)
    s = 2.0 ** 10
    return R.h3_act(x, s).to(DEV), w3.to(DEV), 1.0 / (s * sw)


def each_split(fn):
    outs = {}
    prev = ops.get_gemm_split()
    try:
        for k in SPLITS:
            ops.set_gemm_split(k)
            r = fn()
            torch.cuda.synchronize()
            outs[k] = [t.clone() for t in (r if isinstance(r, (tuple, list)) else (r,)) if torch.is_tensor(t)]
    finally:
        ops.set_gemm_split(prev)
    if lib().edge_gemm_checked_build():
        assert ops.gemm_check_errors() == 0, "device bounds check failed"
    return outs


def assert_identical(outs):
    for k, o in outs.items():
        assert len(o) == len(outs[0])
        for a, b in zip(o, outs[0]):
            assert torch.equal(a, b), f"split {k} differs from the plain walk"


@pytest.mark.parametrize("M,N,K,kind", [(32768, 9728, 896, "swiglu"), (8192, 9728, 896, "swiglu"),
                                         (32768, 896, 896, "resid"), (32768, 896, 4864, "resid")])
def test_desync_bit_identical_linear(M, N, K, kind):
    a3, w3, alpha = h3_operands(M, N, K, 1)
    if kind == "swiglu":
        fn = lambda: ops.linear_h3(a3, w3, alpha, act="swiglu_il", out_scale=64.0)   # noqa: E731
    else:
        res = rnd(M, N, seed=5).to(DEV)
        fn = lambda: ops.linear_h3(a3, w3, alpha, residual=res)                       # noqa: E731
    assert_identical(each_split(fn))


def test_desync_bit_identical_inplace_residual():
    """C aliases the residual (the down projection's out=y): a parked tile's epilogue still reads its own rows."""
    M, N, K = 32768, 896, 896
    a3, w3, alpha = h3_operands(M, N, K, 2)
    y0 = rnd(M, N, seed=6).to(DEV)

    def fn():
        y = y0.clone()
        return ops.linear_h3(a3, w3, alpha, residual=y, out=y)
    assert_identical(each_split(fn))


def test_desync_bit_identical_qkv_planes():
    B, S, Hq, Hkv = 64, 512, 14, 2
    a3, w3, alpha = h3_operands(B * S, (Hq + 2 * Hkv) * 64, 896, 3)
    bias = rnd((Hq + 2 * Hkv) * 64, s=0.02, seed=7).to(DEV)
    cos, sin = R.rope_tables(4096, 64, 1e6)
    cos, sin = cos.to(DEV), sin.to(DEV)
    fn = lambda: ops.qkv_rope_h3(a3, w3, alpha, bias, cos, sin, B, S, Hq, Hkv, 64, 64, 0.125,   # noqa: E731
                                 kv_scales=(64.0, 64.0))
    assert_identical(each_split(fn))


@pytest.mark.parametrize("V", [18432, 151936])
def test_desync_bit_identical_lse_head(V):
    """The LM head + LSE at the bench's scored rows (64 windows x 32) and the full Qwen2 vocabulary."""
    R_, K = 2048, 896
    a3, w3, alpha = h3_operands(R_, V, K, 4)
    tgt = torch.randint(0, V, (R_,), generator=torch.Generator().manual_seed(8)).to(DEV)
    assert_identical(each_split(lambda: ops.head_nll_h3(a3, w3, alpha, tgt)))


def test_desync_bit_identical_bf16_mode():
    """bf16 mode: the gate/up SwiGLU GEMM and the LSE head on the same four-wave kernel."""
    M, N, K = 32768, 9728, 896
    x = rnd(M, K, seed=9).bfloat16().to(DEV)
    w = (rnd(N, K, s=0.02, seed=10)).bfloat16().to(DEV)
    assert_identical(each_split(lambda: ops.linear(x, w, act="swiglu_il")))
    h = rnd(2048, K, seed=11).bfloat16().to(DEV)
    wv = (rnd(151936, K, s=0.02, seed=12)).bfloat16().to(DEV)
    tgt = torch.randint(0, 151936, (2048,), generator=torch.Generator().manual_seed(13)).to(DEV)
    assert_identical(each_split(lambda: ops.head_nll(h, wv, tgt)))
