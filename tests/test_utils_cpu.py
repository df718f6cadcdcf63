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


def test_checkpoint_refuses_other_sharding(tmp_path):
    """A data-parallel checkpoint written at world=2 cannot be resumed at world=1 or 4."""
    import pytest
    from llm_inference_in_distributed_edge_networks_amd.utils.checkpoint import ShardMismatch, SweepState
    p = str(tmp_path / "ck.json")
    SweepState(p, "h", shard=(0, 2, "batch-mod/8")).save({"windows_done": 16})
    assert SweepState(p, "h", shard=(0, 2, "batch-mod/8")).load()["windows_done"] == 16
    for other in ((0, 1, "batch-mod/8"), (0, 4, "batch-mod/8"), (0, 2, "batch-mod/4")):
        with pytest.raises(ShardMismatch):
            SweepState(p, "h", shard=other).load()
    assert SweepState(p, "other-config", shard=(0, 1, "x")).load() is None


def test_window_weight_stride_longer_than_window():
    """stride > max_length: the reference masks nothing (target[:, :-trg_len] with trg_len > S), weight S - 1."""
    from llm_inference_in_distributed_edge_networks_amd.eval.windows import sliding_windows
    ws = sliding_windows(1000, 64, 100)
    assert ws[1].trg_len > ws[1].length and ws[1].weight == ws[1].length - 1
    assert ws[0].weight == 63


def test_normalize_per_layer_zero_sum():
    import torch
    from llm_inference_in_distributed_edge_networks_amd.relevance.attnlrp import normalize_per_layer
    r = normalize_per_layer(torch.tensor([[1.0, -1.0], [1.0, 3.0]]))
    assert torch.isfinite(r).all() and torch.allclose(r[1], torch.tensor([0.25, 0.75]))


def test_wikitext_fallback_is_loud(capsys):
    import pytest
    from llm_inference_in_distributed_edge_networks_amd.eval.data import DatasetUnavailable, token_stream
    with pytest.warns(RuntimeWarning):
        ids, prov = token_stream("wikitext", "no/such-model", 512, 1000)
    assert prov.startswith("synthetic") and "WARNING" in capsys.readouterr().out
    with pytest.raises(DatasetUnavailable):
        token_stream("wikitext", "no/such-model", 512, 1000, strict=True)
    with pytest.raises(ValueError):
        token_stream("wikitxt", "x", 512)
