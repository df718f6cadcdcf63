"""Qwen2-0.5B experiments (reference: Experiments/Qwen2-0.5B/main.py + channel_wise.py).

``python main.py`` reads ``./params.json``: if the first method is a channel quantizer
(channel_8 / channel_4 / channel_1_mean / channel_1_max) the per-channel sweep runs
(results ``[layer][method]``), otherwise the importance sweep over
``methods x layers_of_interest x ratios`` (regular_importance, weighted_importance, last_row,
aggregate_till; results ``avg_ppl_results[method][layer][ratio]``).  weighted_importance needs the
LRP head table written by ``../Relevance/main.py``.
Data-parallel over GPUs: ``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 main.py``.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from llm_inference_in_distributed_edge_networks_amd.config import Params  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.experiments import qwen2_main  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.parallel.dist import shutdown  # noqa: E402

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", default="params.json")
    ap.add_argument("--device", default=None)
    ap.add_argument("--max-windows", type=int, default=None)
    a = ap.parse_args()
    p = Params.load(a.params, device=a.device, max_windows=a.max_windows)
    p.model = p.model or "qwen2-0.5b"
    if p.max_length is None:
        p.max_length = 512
    qwen2_main(p)
    shutdown()  # all ranks done: barrier + destroy the process group before interpreter exit
