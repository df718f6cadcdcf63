"""CPU oracle of the fp32-mode fused RMSNorm-2 (ops.linear_h3_np / reference.np_planes, gemm.hip EPI_F32_RESID_NP):
the planes carry p_m (y_m * g) at a power-of-two row scale from a bound, the consumer undoes it with
rsqrt(mean(y^2) + eps) / p_m.  The h3 model with the fusion equals the separate-norm h3 model to fp32 accuracy."""

import torch

from llm_inference_in_distributed_edge_networks_amd import ops
from llm_inference_in_distributed_edge_networks_amd.models import DecoderLM, TINY_QWEN2
from llm_inference_in_distributed_edge_networks_amd.ops import reference as R


def test_np_planes_bound_and_split():
    g = torch.Generator().manual_seed(0)
    M, N = 64, 896
    x = torch.randn(M, N, generator=g)
    x[3] *= 1000.0                                   # a sink-like row
    prod = torch.randn(M, N, generator=g) * 0.5
    y = x + prod
    w = 1 + 0.1 * torch.randn(N, generator=g)
    w[5] = -12.0
    rstd = torch.rsqrt(x.pow(2).mean(1) + 1e-6)
    pb = float(prod.abs().max())
    planes, prinv, ssq = R.np_planes(y, w, rstd, float(w.abs().max()), pb)
    p = 1.0 / prinv
    scaled = (y * w) * p.view(-1, 1)
    assert float(scaled.abs().max()) < 2 ** 14                         # bound respected: no fp16 overflow
    assert float(scaled.abs().amax(1).min()) > 2 ** 5     # loose by at most ~2^9 here: the lo plane stays normal
    assert torch.equal(p, torch.exp2(torch.log2(p).round()))            # powers of two
    back = (planes[:, :N].float() + planes[:, N:].float()) / p.view(-1, 1)
    assert float(((back - y * w).abs() / (y * w).abs().amax(1, keepdim=True)).max()) < 2 ** -21
    assert torch.allclose(ssq.sum(1), y.pow(2).sum(1), rtol=1e-6)
    rs = R.row_rscale_mul(ssq, prinv, N, 1e-6)
    normed = back * torch.rsqrt(y.pow(2).mean(1) + 1e-6).view(-1, 1)
    assert torch.allclose((planes[:, :N].float() + planes[:, N:].float()) * rs.view(-1, 1), normed, rtol=1e-5,
                          atol=1e-6)


def test_fused_norm_model_equals_separate_pass_cpu():
    cfg = TINY_QWEN2
    m = DecoderLM.random_init(cfg, seed=3, dtype=torch.float32, values=torch.bfloat16, h3=True)
    assert not m.fuse_norm_f32                       # CPU models keep the separate pass unless asked
    ids = torch.randint(0, cfg.vocab_size, (2, 128), generator=torch.Generator().manual_seed(1))
    x0 = m.forward_hidden(ids)
    m.fuse_norm_f32 = True
    x1 = m.forward_hidden(ids)
    ref = DecoderLM.random_init(cfg, seed=3, dtype=torch.float32, values=torch.bfloat16, h3=False).forward_hidden(ids)
    e01 = float((x1 - x0).norm() / x0.norm())
    e1r = float((x1 - ref).norm() / ref.norm())
    assert e01 < 2e-6 and e1r < 2e-6, (e01, e1r)
    assert ops.linear_h3_np is not None
