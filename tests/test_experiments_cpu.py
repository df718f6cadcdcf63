"""Reference entry points (Experiments/*/main.py + params.json) run end-to-end on tiny models (CPU)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_main(exp, params, tmp_path):
    d = tmp_path / exp
    d.mkdir()
    base = {"dataset": "synthetic", "synthetic_tokens": 1200, "max_windows": 8, "device": "cpu",
            "window_batch": 4, "output_dir": str(d)}
    base.update(params)
    (d / "params.json").write_text(json.dumps(base))
    env = dict(os.environ, EDGE_NO_PROGRESS="1", WORLD_SIZE="1", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "Experiments", exp, "main.py")], cwd=d, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return d


def test_pythia_last_row(tmp_path):
    d = run_main("Pythia-70M", {"model": "tiny-neox", "experiment": "last_row", "max_length": 128,
                                "ratios": [0, 0.5, 1], "layers_of_interest": [1, 2],
                                "methods": ["regular_importance", "last_row", "aggregate_till"]}, tmp_path)
    res = json.loads((d / "avg_ppl_results_pythia_70m.json").read_text())
    p = res["avg_ppl_results"]
    assert len(p) == 3 and len(p[0]) == 2 and len(p[0][0]) == 3
    assert p[0][0][0] == p[1][1][0]


def test_pythia_initial(tmp_path):
    d = run_main("Pythia-70M", {"model": "tiny-neox", "experiment": "initial", "max_length": 128,
                                "ratios": [0, 5, 10],
                                "layers_of_interest": [1, "aggregate upto 2", "maximum aggregation", "upto ratio"]},
                 tmp_path)
    res = json.loads((d / "exp_1.json").read_text())["exp_1"]
    assert set(res) == {"1", "aggregate upto 2", "maximum aggregation", "upto ratio"}
    # ratio 0 is method independent for the ratio orderings; top-rho at mass 1 may still cut the tail tokens
    # whose mass lies beyond the rounded sum (as the reference's fp32 running total does)
    assert len({round(v["0"], 9) for k, v in res.items() if k != "upto ratio"}) == 1
    assert abs(res["upto ratio"]["0"] - res["1"]["0"]) < 1e-5


def test_pythia_unknown_experiment(tmp_path):
    with pytest.raises(AssertionError):
        run_main("Pythia-70M", {"model": "tiny-neox", "experiment": "bogus"}, tmp_path)


def test_qwen2_importance_and_relevance(tmp_path):
    d = run_main("Relevance", {"model": "tiny-qwen2", "max_length": 64, "max_windows": 3}, tmp_path)
    hw = json.loads((d / "attention_head_weights.json").read_text())
    assert len(hw) == 4 and len(hw[0]) == 4
    d2 = run_main("Qwen2-0.5B", {"model": "tiny-qwen2", "max_length": 128, "ratios": [0, 0.25, 1],
                                 "layers_of_interest": [1, 2],
                                 "methods": ["regular_importance", "weighted_importance", "last_row",
                                             "aggregate_till"],
                                 "head_weights": str(d / "attention_head_weights.json")}, tmp_path)
    res = json.loads((d2 / "avg_ppl_results.json").read_text())
    assert len(res["avg_ppl_results"]) == 4 and res["wire_bytes_per_token"][0][0][2] < res["wire_bytes_per_token"][0][0][0]
    # the relevance pass also writes the channel-group table; the config-5 pipeline uses it for its group plans
    gr = json.loads((d / "channel_group_relevance.json").read_text())
    assert len(gr) == 4 and len(gr[0]) == 4 and all(abs(sum(r) - 1) < 1e-3 for r in gr)
    d3 = run_main("Pipeline", {"model": "tiny-qwen2", "num_stages": 2, "codec": "mixed_rgroup_int8",
                               "methods": ["weighted_importance"], "ratios": [0, 1], "max_length": 64,
                               "head_weights": str(d / "attention_head_weights.json"),
                               "group_relevance": str(d / "channel_group_relevance.json")}, tmp_path)
    res = json.loads((d3 / "pipeline_results.json").read_text())["results"]["weighted_importance"]
    assert res["1"]["wire_bytes_per_token"] < res["0"]["wire_bytes_per_token"]


def test_qwen2_channel(tmp_path):
    d = run_main("Qwen2-0.5B", {"model": "tiny-qwen2", "max_length": 128, "layers_of_interest": [1, 3],
                                "methods": ["channel_8", "channel_4", "channel_1_mean", "channel_1_max"]}, tmp_path)
    res = json.loads((d / "avg_ppl_results_channel.json").read_text())
    assert len(res["avg_ppl_results"]) == 2 and len(res["avg_ppl_results"][0]) == 4


def test_analysis_js(tmp_path):
    d = run_main("Analysis", {"model": "tiny-neox", "max_lines": 6}, tmp_path)
    res = json.loads((d / "js_divergence.json").read_text())
    m = res["js_divergence"]
    assert len(m) == 4 and m[0][0] == 0 and abs(m[0][1] - m[1][0]) < 1e-12 and all(0 <= v <= 1 for r in m for v in r)


def test_top_rho_selection_from_params(tmp_path):
    """params['selection'] = 'top_rho' drives the sweep and the pipeline (variable-k boundary messages)."""
    d = run_main("Qwen2-0.5B", {"model": "tiny-qwen2", "max_length": 128, "ratios": [0.5], "layers_of_interest": [1],
                                "methods": ["last_row"], "codec": "mixed_int4_int8", "selection": "top_rho"},
                 tmp_path)
    sw = json.loads((d / "avg_ppl_results.json").read_text())
    p = run_main("Pipeline", {"model": "tiny-qwen2", "split_layers": [1], "codec": "mixed_int4_int8",
                              "methods": ["last_row"], "ratios": [0.5], "max_length": 128, "selection": "top_rho"},
                 tmp_path)
    res = json.loads((p / "pipeline_results.json").read_text())["results"]["last_row"]["0.5"]
    assert abs(res["ppl"] - sw["avg_ppl_results"][0][0][0]) / res["ppl"] < 1e-6


def test_rgroup_sweep_equals_pipeline_with_relevance_table(tmp_path):
    """The Qwen2 sweep driver and the pipeline driver load params['group_relevance'] the same way: with a skewed
    channel-group relevance table the mixed_rgroup_int8 boundary (relevance-allocated group widths) gives the same
    PPL and wire bytes through both."""
    from llm_inference_in_distributed_edge_networks_amd.models import TINY_QWEN2
    G = TINY_QWEN2.hidden_size // 64
    rel = [[(10.0 if g == G - 1 else 0.05) * (1 + l) for g in range(G)] for l in range(TINY_QWEN2.num_layers + 1)]
    from llm_inference_in_distributed_edge_networks_amd.codec import wire
    assert wire.allocate_group_bits(rel[2], 4.0) != wire.allocate_group_bits([1.0] * G, 4.0)   # the table matters
    tab = tmp_path / "grel.json"
    tab.write_text(json.dumps(rel))
    common = {"model": "tiny-qwen2", "max_length": 128, "ratios": [0.5, 1.0], "methods": ["last_row"],
              "codec": "mixed_rgroup_int8", "group_relevance": str(tab), "group_avg_bits": 4.0}
    sw = json.loads((run_main("Qwen2-0.5B", dict(common, layers_of_interest=[1]), tmp_path)
                     / "avg_ppl_results.json").read_text())
    pr = json.loads((run_main("Pipeline", dict(common, split_layers=[1]), tmp_path)
                     / "pipeline_results.json").read_text())["results"]["last_row"]
    for ri, r in enumerate(("0.5", "1.0")):
        assert abs(pr[r]["ppl"] - sw["avg_ppl_results"][0][0][ri]) / pr[r]["ppl"] < 1e-6
        assert pr[r]["wire_bytes_per_token"] == pytest.approx(sw["wire_bytes_per_token"][0][0][ri], rel=1e-6)


def test_pipeline_driver_resumes_mid_run(tmp_path, monkeypatch):
    """pipeline_experiment checkpoints after every chunk of checkpoint_every windows and after every (method,
    ratio); a run killed in the middle of its second configuration resumes to the uninterrupted result."""
    import sys as _sys
    _sys.path.insert(0, ROOT)
    from llm_inference_in_distributed_edge_networks_amd.config import Params
    from llm_inference_in_distributed_edge_networks_amd.eval import experiments as E
    from llm_inference_in_distributed_edge_networks_amd.parallel import pipeline as P

    def params(d):
        d.mkdir()
        # top_rho: variable-k messages, so the bytes per token differ per batch and a resumed run must carry the
        # byte and token sums of the chunks before the crash
        return Params.from_dict({"model": "tiny-qwen2", "split_layers": [1], "codec": "mixed_int4_int8",
                                 "methods": ["last_row"], "selection": "top_rho", "ratios": [0.25, 0.75],
                                 "max_length": 128, "stride": 32,
                                 "window_batch": 2, "dataset": "synthetic", "synthetic_tokens": 1200,
                                 "device": "cpu", "checkpoint_every": 4, "output_dir": str(d)})
    full = E.pipeline_experiment(params(tmp_path / "full"), "qwen2-0.5b")["results"]
    calls = {"n": 0}
    orig = P.LocalPipeline.evaluate

    def flaky(self, *a, **k):
        calls["n"] += 1
        if calls["n"] == 14:                 # inside the second ratio's run
            raise KeyboardInterrupt("simulated crash")
        return orig(self, *a, **k)
    p = params(tmp_path / "crash")
    monkeypatch.setattr(P.LocalPipeline, "evaluate", flaky)
    with pytest.raises(KeyboardInterrupt):
        E.pipeline_experiment(p, "qwen2-0.5b")
    ck = json.loads((tmp_path / "crash" / "pipeline_results.rank0.ckpt.json").read_text())
    assert "0.25" in ck["results"]["last_row"] and ck["partial"]["key"] == ["last_row", "0.75"]
    monkeypatch.setattr(P.LocalPipeline, "evaluate", orig)
    res = E.pipeline_experiment(p, "qwen2-0.5b")["results"]
    for r in ("0.25", "0.75"):
        assert res["last_row"][r]["ppl"] == pytest.approx(full["last_row"][r]["ppl"], rel=1e-9)
        assert res["last_row"][r]["n_tokens"] == full["last_row"][r]["n_tokens"]
        assert res["last_row"][r]["wire_bytes_per_token"] == pytest.approx(
            full["last_row"][r]["wire_bytes_per_token"], rel=1e-12)
    # a partial entry in round 3's format (wire_sum / wire_n instead of wire_bytes / wire_tokens) is not resumed
    # from: that (method, ratio) restarts from batch 0 and still ends at the uninterrupted result
    ck = tmp_path / "crash" / "pipeline_results.rank0.ckpt.json"
    state = json.loads(ck.read_text())
    state["results"]["last_row"].pop("0.75")
    state["partial"] = {"key": ["last_row", "0.75"], "total_nll": 123.0, "n_tokens": 7.0, "seconds": 0.1,
                        "wire_sum": 1.0, "wire_n": 1.0, "next_batch": 4}
    ck.write_text(json.dumps(state))
    res = E.pipeline_experiment(p, "qwen2-0.5b")["results"]
    assert res["last_row"]["0.75"]["ppl"] == pytest.approx(full["last_row"]["0.75"]["ppl"], rel=1e-9)
