"""The two reference models at their real shapes on the GPU (random weights, synthetic tokens):

* Pythia-70M with the reference's 2048-token windows (``Pythia-70M/last_row_exp.py:72-73``), split at layer 2
  with an int8 boundary, against the fp32 CPU oracle of the same split;
* Qwen2-0.5B at the bench micro-batch (64 windows x 512 tokens: the size that selects the production GEMM
  kernels, incl. the 256x224 residual GEMMs), per-window NLL with those kernels against the 256x256 ones.
"""
import pytest
import torch

from llm_inference_in_distributed_edge_networks_amd import ops
from llm_inference_in_distributed_edge_networks_amd.eval.data import synthetic_stream
from llm_inference_in_distributed_edge_networks_amd.eval.windows import batches, sliding_windows
from llm_inference_in_distributed_edge_networks_amd.models import PYTHIA_70M, QWEN2_0_5B, DecoderLM
from llm_inference_in_distributed_edge_networks_amd.parallel import BoundaryConfig, LocalPipeline, PipelinePlan

pytestmark = pytest.mark.gpu


def test_pythia70m_2048_windows_gpu_vs_cpu():
    cfg = PYTHIA_70M
    toks = synthetic_stream(2048 + 2 * 512, cfg.vocab_size, 7)
    wins = sliding_windows(toks.shape[1], 2048, 512)
    plan = PipelinePlan.from_split_layers(cfg.num_layers, [2])
    bcfg = BoundaryConfig("int8_token", 1.0, "last_row")
    mc = DecoderLM.random_init(cfg, 3, std=0.05)
    mg = DecoderLM.random_init(cfg, 3, device="cuda", dtype=torch.bfloat16, std=0.05)
    pc = LocalPipeline(mc, plan, bcfg).evaluate(batches(toks, wins, 2)).ppl()
    pg = LocalPipeline(mg, plan, bcfg).evaluate(batches(toks, wins, 2)).ppl()
    assert abs(pg - pc) / pc < 0.02, (pg, pc)


def test_qwen2_production_shapes_w7_vs_256():
    cfg = QWEN2_0_5B
    toks = synthetic_stream(64 * 32 + 512, cfg.vocab_size, 8)
    wins = [w for w in sliding_windows(toks.shape[1], 512, 32) if w.length == 512][:64]
    b = next(batches(toks, wins, 64)).to("cuda")
    assert b.B * 512 == 32768
    m = DecoderLM.random_init(cfg, 4, device="cuda", dtype=torch.bfloat16)
    plan = PipelinePlan.from_split_layers(cfg.num_layers, [11])
    bcfg = BoundaryConfig("mixed_int4_int8", 0.5, "regular_importance")
    assert ops.gemm_ssq_parts(32768, 896, 896, residual=True) == 8   # the 256x224 kernel is selected
    w7 = LocalPipeline(m, plan, bcfg, use_graphs=False).run_batch(b).clone()
    ops.set_gemm_tile(256)   # every GEMM on 256x256 tiles (N = 896: a half-used last column tile)
    try:
        assert ops.gemm_ssq_parts(32768, 896, 896, residual=True) == 14
        c256 = LocalPipeline(m, plan, bcfg, use_graphs=False).run_batch(b).clone()
    finally:
        ops.set_gemm_tile(0)
    assert torch.isfinite(w7).all()
    # same math, different tiling / partial-sum order: bf16-level differences through 24 layers
    assert torch.allclose(w7, c256, rtol=2e-2, atol=2e-2), (w7 - c256).abs().max()
