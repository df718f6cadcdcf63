"""LRP head-weight tables in the reference's pickle form (``attention_head_weights.pkl``: the notebook writes it with
``pickle.dump``, ``Experiments/Qwen2-0.5B/main.py:129-130`` reads it from ``../../``).  The loader must read a
[layers][heads] list of numbers at any pickle protocol, refuse everything else, and never execute anything from the
file."""
import json
import os
import pickle

import pytest
import torch

from llm_inference_in_distributed_edge_networks_amd.eval import experiments
from llm_inference_in_distributed_edge_networks_amd.importance import load_head_weights


def table(layers=24, heads=14):
    g = torch.Generator().manual_seed(0)
    w = torch.randn(layers, heads, generator=g, dtype=torch.float64)
    w = w / w.sum(dim=1, keepdim=True)    # signed, each layer sums to 1 (Relevance/main.py:111-118)
    rows = w.tolist()
    rows[-1][-1] = 0                       # an int left from the notebook's [[0 ...]] initialisation
    return rows


@pytest.mark.parametrize("protocol", [2, 3, 4, 5])
def test_pickle_table_loads(tmp_path, protocol):
    rows = table()
    p = tmp_path / "attention_head_weights.pkl"
    with open(p, "wb") as f:
        pickle.dump(rows, f, protocol=protocol)
    w = load_head_weights(str(p))
    assert w.shape == (24, 14) and w.dtype == torch.float32
    assert torch.equal(w, torch.tensor(rows, dtype=torch.float32))


def test_pickle_tuple_rows_and_torch_save(tmp_path):
    rows = table(4, 3)
    p = tmp_path / "t.pkl"
    with open(p, "wb") as f:
        pickle.dump(tuple(tuple(r) for r in rows), f)
    assert torch.equal(load_head_weights(str(p)), torch.tensor(rows, dtype=torch.float32))
    q = tmp_path / "s.pkl"
    torch.save(torch.tensor(rows), q)     # torch.save of a tensor: torch.load(weights_only=True) reads it
    assert torch.allclose(load_head_weights(str(q)), torch.tensor(rows, dtype=torch.float32))


class _Payload:
    def __init__(self, marker):
        self.marker = marker

    def __reduce__(self):
        return (open, (self.marker, "w"))   # would create the marker file if anything unpickled it


@pytest.mark.parametrize("bad", ["reduce", "nested_reduce", "dict", "string", "ragged", "bool", "empty"])
def test_pickle_refuses_anything_else(tmp_path, bad):
    marker = tmp_path / "executed"
    obj = {"reduce": _Payload(str(marker)), "nested_reduce": [[1.0, _Payload(str(marker))]],
           "dict": {"layer0": [1.0]}, "string": [["a", 1.0]], "ragged": [[1.0, 2.0], [3.0]], "bool": [[True, 1.0]],
           "empty": []}[bad]
    p = tmp_path / "attention_head_weights.pkl"
    with open(p, "wb") as f:
        pickle.dump(obj, f)
    with pytest.raises(ValueError):
        load_head_weights(str(p))
    assert not marker.exists()


def test_json_still_loads(tmp_path):
    rows = table(2, 14)
    p = tmp_path / "attention_head_weights.json"
    p.write_text(json.dumps(rows))
    assert torch.equal(load_head_weights(str(p)), torch.tensor(rows, dtype=torch.float32))


def test_default_lookup_finds_reference_pickle_location(tmp_path, monkeypatch):
    """The reference's Qwen2 sweep runs in Experiments/Qwen2-0.5B and reads ../../attention_head_weights.pkl."""
    rows = table()
    with open(tmp_path / "attention_head_weights.pkl", "wb") as f:
        pickle.dump(rows, f)
    run_dir = tmp_path / "Experiments" / "Qwen2-0.5B"
    os.makedirs(run_dir)
    monkeypatch.chdir(run_dir)
    path = experiments._default_head_weights()
    assert path == "../../attention_head_weights.pkl"
    assert torch.equal(load_head_weights(path), torch.tensor(rows, dtype=torch.float32))
