"""Shared-prefix sweep engine == independent split runs; checkpoint/resume."""
import json
import os

import torch

from llm_inference_in_distributed_edge_networks_amd.eval.data import synthetic_stream
from llm_inference_in_distributed_edge_networks_amd.eval.sweep import SweepConfig, SweepEngine, run_sweep
from llm_inference_in_distributed_edge_networks_amd.eval.windows import batches, sliding_windows
from llm_inference_in_distributed_edge_networks_amd.models import TINY_QWEN2, DecoderLM
from llm_inference_in_distributed_edge_networks_amd.parallel import BoundaryConfig, LocalPipeline, PipelinePlan
from llm_inference_in_distributed_edge_networks_amd.utils.checkpoint import SweepState

M = DecoderLM.random_init(TINY_QWEN2, 0, std=0.06)
TOK = synthetic_stream(1200, 512, 1)
WINS = sliding_windows(1200, 128, 32)


def test_sweep_equals_split_runner():
    methods = ["regular_importance", "last_row", "aggregate_till", "weighted_importance"]
    hw = torch.randn(4, 4)
    sc = SweepConfig(methods, [0, 2], [0, 0.25, 0.5, 1], codec="ref_int4_global", head_weights=hw, max_fork_tokens=512)
    res = run_sweep(SweepEngine(M, sc), batches(TOK, WINS, 4))
    for mi, meth in enumerate(methods):
        for li, L in enumerate([0, 2]):
            for ri, r in enumerate([0, 0.25, 0.5, 1]):
                pipe = LocalPipeline(M, PipelinePlan.from_split_layers(4, [L]),
                                     BoundaryConfig("ref_int4_global", r, meth, hw))
                ppl = pipe.evaluate(batches(TOK, WINS, 4)).ppl()
                assert abs(ppl - res["avg_ppl_results"][mi][li][ri]) / ppl < 1e-6, (meth, L, r)
    # ratio 0 identical across methods/layers, ratio 1 identical across methods
    p = res["avg_ppl_results"]
    assert len({round(p[mi][li][0], 9) for mi in range(4) for li in range(2)}) == 1
    assert len({round(p[mi][0][3], 9) for mi in range(4)}) == 1


def test_resume(tmp_path):
    sc = SweepConfig(["last_row"], [1], [0, 0.5], codec="mixed_int4_int8")
    full = run_sweep(SweepEngine(M, sc), batches(TOK, WINS, 2))
    st = SweepState(str(tmp_path / "ck.json"), "h1")
    e1 = SweepEngine(M, sc)
    # interrupt after 3 batches
    it = batches(TOK, WINS, 2)
    part = [next(it) for _ in range(3)]
    run_sweep(e1, iter(part), st, log_every=2)
    assert os.path.exists(tmp_path / "ck.json")
    e2 = SweepEngine(M, sc)
    res = run_sweep(e2, batches(TOK, WINS, 2), st, log_every=2)
    assert abs(res["avg_ppl_results"][0][0][1] - full["avg_ppl_results"][0][0][1]) < 1e-9
    assert res["windows"] == full["windows"]
    # different config hash -> not resumed
    assert SweepState(str(tmp_path / "ck.json"), "other").load() is None


def test_sweep_top_rho_equals_split_runner():
    """Top-rho rows of the sweep engine == the pipeline runtime with selection='top_rho'."""
    from llm_inference_in_distributed_edge_networks_amd.eval.sweep import SweepMethod
    rows = [SweepMethod("rho", "regular_importance", selection="top_rho"),
            SweepMethod("rho_last", "last_row", selection="top_rho")]
    sc = SweepConfig(rows, [1], [0.25, 0.75, 1.0], codec="mixed_int4_int8")
    res = run_sweep(SweepEngine(M, sc), batches(TOK, WINS, 4))
    for mi, meth in enumerate(["regular_importance", "last_row"]):
        for ri, r in enumerate([0.25, 0.75, 1.0]):   # 1.0: keep mass 0, no importance tracked
            pipe = LocalPipeline(M, PipelinePlan.from_split_layers(4, [1]),
                                 BoundaryConfig("mixed_int4_int8", r, meth, selection="top_rho"))
            ppl = pipe.evaluate(batches(TOK, WINS, 4)).ppl()
            assert abs(ppl - res["avg_ppl_results"][mi][0][ri]) / ppl < 1e-6
            assert abs(pipe.wire_bytes_per_token()[0] - res["wire_bytes_per_token"][mi][0][ri]) < 1e-6


def test_initial_rows_batched_equals_per_window():
    """The batched Pythia 'initial' (one stacked suffix per batch) == each window / ordering / ratio on its own."""
    from llm_inference_in_distributed_edge_networks_amd.eval.experiments import initial_rows
    from llm_inference_in_distributed_edge_networks_amd.eval.sweep import SweepMethod
    from llm_inference_in_distributed_edge_networks_amd.models import TINY_NEOX
    mn = DecoderLM.random_init(TINY_NEOX, 1, std=0.06)
    rows = initial_rows([3, "aggregate upto 2", "maximum aggregation", "upto ratio"])
    sc = SweepConfig(rows, [2], [0, 3, 7, 10], codec="int8_token_keep", ratio_scale=0.1)
    res = run_sweep(SweepEngine(mn, sc), batches(TOK, WINS, 4))
    ref = run_sweep(SweepEngine(mn, SweepConfig(rows, [2], [0, 3, 7, 10], codec="int8_token_keep", ratio_scale=0.1,
                                                max_fork_tokens=128)), batches(TOK, WINS, 1))
    a, b = torch.tensor(res["mean_window_nll"]), torch.tensor(ref["mean_window_nll"])
    assert torch.allclose(a, b, atol=2e-5), (a - b).abs().max()
    # ratio 10 with top-rho: mass 0 -> every token quantized == the ratio-form ratio 10
    assert abs(a[3, 0, 3] - a[0, 0, 3]) < 1e-6


def test_sweep_group_codec_equals_split_runner():
    """Head-group codec with relevance-allocated plans (per boundary layer): sweep engine == pipeline runtime, and
    the plans differ between boundaries when the relevance does."""
    G = TINY_QWEN2.hidden_size // 64
    grel = torch.rand(TINY_QWEN2.num_layers, G, generator=torch.Generator().manual_seed(3))
    grel[1] = torch.tensor([1.0] + [0.02] * (G - 1))    # one dominant group: 8 bits for it, 2 for some others
    sc = SweepConfig(["regular_importance"], [0, 2], [0.5, 1], codec="mixed_rgroup_int8", group_relevance=grel,
                     group_avg_bits=4.0)
    eng = SweepEngine(M, sc)
    res = run_sweep(eng, batches(TOK, WINS, 4))
    for li, L in enumerate([0, 2]):
        for ri, r in enumerate([0.5, 1]):
            bc = BoundaryConfig("mixed_rgroup_int8", r, "regular_importance", group_relevance=grel, group_avg_bits=4.0)
            pipe = LocalPipeline(M, PipelinePlan.from_split_layers(4, [L]), bc)
            assert pipe.stages[0].spec_out.plan == eng._spec_at("mixed_rgroup_int8", L).plan
            ppl = pipe.evaluate(batches(TOK, WINS, 4)).ppl()
            assert abs(ppl - res["avg_ppl_results"][0][li][ri]) / ppl < 1e-6, (L, r)
    assert eng._spec_at("mixed_rgroup_int8", 0).plan == (8, 4, 2, 2)
    # 3 stages: each boundary decodes with the plan its sender used
    bc = BoundaryConfig("mixed_rgroup_int8", 0.5, "regular_importance", group_relevance=grel)
    pipe = LocalPipeline(M, PipelinePlan.from_split_layers(4, [0, 2]), bc)
    assert pipe.stages[1].spec_in.plan == pipe.stages[0].spec_out.plan
    assert pipe.evaluate(batches(TOK, WINS, 4)).ppl() > 0
