"""Tracing, watchdog, config, graph-cache fallbacks."""
import json
import time

import pytest
import torch

from llm_inference_in_distributed_edge_networks_amd.config import Params
from llm_inference_in_distributed_edge_networks_amd.utils import trace
from llm_inference_in_distributed_edge_networks_amd.utils.graphs import GraphCache
from llm_inference_in_distributed_edge_networks_amd.utils.watchdog import Watchdog


def test_trace_ranges_and_counters():
    trace.reset()
    trace.enable(True)
    with trace.range("a"):
        time.sleep(0.01)
    with trace.range("a"):
        pass
    trace.counter("bytes", 10)
    trace.counter("bytes", 5)
    s = trace.summary()
    assert s["a"]["count"] == 2 and s["a"]["total_s"] >= 0.01 and s["counters"]["bytes"] == 15
    trace.enable(False)
    with trace.range("b"):
        pass
    assert "b" not in trace.summary()


def test_watchdog_fires_and_beats():
    fired = []
    wd = Watchdog(0.3, on_timeout=lambda: fired.append(1)).start()
    for _ in range(5):
        time.sleep(0.1)
        wd.beat()
    assert not fired
    time.sleep(0.8)
    assert fired and wd.fired
    wd.stop()


def test_params_reference_files_load(tmp_path):
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for exp in ("Pythia-70M", "Qwen2-0.5B", "Relevance"):
        p = Params.load(os.path.join(root, "Experiments", exp, "params.json"))
        assert p.stride == 32
    f = tmp_path / "p.json"
    f.write_text(json.dumps({"ratios": [0, 1], "unknown_key": 3}))
    p = Params.load(str(f))
    assert p.extra == {"unknown_key": 3} and p.to_dict()["unknown_key"] == 3
    assert p.config_hash() != Params.from_dict({"ratios": [0, 0.5]}).config_hash()
    with pytest.raises(ValueError):
        Params.from_dict({"stride": 0})


def test_graph_cache_cpu_passthrough():
    calls = []
    g = GraphCache(lambda x: calls.append(1) or x * 2)
    for _ in range(3):
        assert torch.equal(g(torch.ones(3)), torch.full((3,), 2.0))
    assert len(calls) == 3 and not g.graphs
