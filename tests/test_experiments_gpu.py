"""Reference entry points on the GPU (tiny models, synthetic tokens): the drivers pick bf16 + the HIP kernels,
and the pipeline driver runs every importance method with HIP graphs (the LRP head table must already be on the
device when a graph is captured)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_main(exp, params, tmp_path, name=None):
    d = tmp_path / (name or exp)
    d.mkdir()
    base = {"dataset": "synthetic", "synthetic_tokens": 3000, "max_windows": 24, "device": "cuda",
            "window_batch": 8, "output_dir": str(d)}
    base.update(params)
    (d / "params.json").write_text(json.dumps(base))
    env = dict(os.environ, EDGE_NO_PROGRESS="1", WORLD_SIZE="1", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "Experiments", exp, "main.py")], cwd=d, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return d


def test_relevance_then_weighted_pipeline_and_sweep(tmp_path):
    d = run_main("Relevance", {"model": "tiny-qwen2", "max_length": 128}, tmp_path)
    hwp = str(d / "attention_head_weights.json")
    hw = json.loads(open(hwp).read())
    assert len(hw) == 4 and all(abs(sum(r) - 1) < 1e-3 for r in hw)
    p = run_main("Pipeline", {"model": "tiny-qwen2", "num_stages": 2, "codec": "mixed_int4_int8",
                              "methods": ["weighted_importance", "last_row", "aggregate_till", "regular_importance"],
                              "ratios": [0, 0.5, 1], "max_length": 128, "head_weights": hwp}, tmp_path)
    res = json.loads((p / "pipeline_results.json").read_text())["results"]
    assert set(res) == {"weighted_importance", "last_row", "aggregate_till", "regular_importance"}
    ppl0 = {round(v["0"]["ppl"], 6) for v in res.values()}
    assert len(ppl0) == 1  # ratio 0 is method independent
    q = run_main("Qwen2-0.5B", {"model": "tiny-qwen2", "max_length": 128, "ratios": [0, 0.5],
                                "layers_of_interest": [1], "methods": ["weighted_importance", "last_row"],
                                "head_weights": hwp}, tmp_path)
    sweep = json.loads((q / "avg_ppl_results.json").read_text())["avg_ppl_results"]
    assert len(sweep) == 2 and all(v > 0 for row in sweep for r in row for v in r)
    # config 5 style: relevance-weighted importance + the head-group codec with the LRP channel-group plans
    grp = str(d / "channel_group_relevance.json")
    gr = json.loads(open(grp).read())
    assert len(gr) == 4 and all(len(r) == 256 // 64 for r in gr)
    g = run_main("Pipeline", {"model": "tiny-qwen2", "num_stages": 3, "codec": "mixed_rgroup_int8",
                              "methods": ["weighted_importance"], "ratios": [0, 0.5, 1], "max_length": 128,
                              "head_weights": hwp, "group_relevance": grp, "group_avg_bits": 3}, tmp_path,
                 name="Pipeline_rgroup")
    res = json.loads((g / "pipeline_results.json").read_text())["results"]["weighted_importance"]
    assert res["1"]["wire_bytes_per_token"] < res["0"]["wire_bytes_per_token"] and res["1"]["ppl"] > 0


def test_pythia_entry_point_gpu(tmp_path):
    d = run_main("Pythia-70M", {"model": "tiny-neox", "experiment": "last_row", "max_length": 256,
                                "ratios": [0, 0.5], "layers_of_interest": [1],
                                "methods": ["regular_importance", "last_row"]}, tmp_path)
    res = json.loads((d / "avg_ppl_results_pythia_70m.json").read_text())["avg_ppl_results"]
    assert res[0][0][0] == res[1][0][0]
