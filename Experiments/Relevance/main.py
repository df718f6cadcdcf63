"""LRP (AttnLRP) per-head relevance calibration for Qwen2-0.5B (reference: Experiments/Relevance/main.py).

Reads ``./params.json`` (``max_length``, ``stride``; the reference wrongly read the Pythia file, B13)
and writes ``attention_head_weights.json`` = [layer][head] relevance shares (each layer sums to 1),
the table ``weighted_importance`` consumes.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from llm_inference_in_distributed_edge_networks_amd.config import Params  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.relevance.attnlrp import relevance_main  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.parallel.dist import shutdown  # noqa: E402

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", default="params.json")
    ap.add_argument("--device", default=None)
    ap.add_argument("--max-windows", type=int, default=None)
    a = ap.parse_args()
    p = Params.load(a.params, device=a.device, max_windows=a.max_windows)
    p.model = p.model or "qwen2-0.5b"
    relevance_main(p)
    shutdown()  # all ranks done: barrier + destroy the process group before interpreter exit
