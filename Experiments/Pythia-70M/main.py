"""Pythia-70M experiments (reference: Experiments/Pythia-70M/main.py).

Run from this directory: ``python main.py`` reads ``./params.json`` (reference schema:
``experiment`` in {"last_row", "initial"}, ``ratios``, ``layers_of_interest``, ``methods``, ``stride``;
optional new keys documented in ``llm_inference_in_distributed_edge_networks_amd/config.py``).
Data-parallel over GPUs: ``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 main.py``.

ratios: fraction of the boundary tokens quantized (``last_row``), or 0..10 meaning 0.1*ratio
(``initial``).  Special ``layers_of_interest`` of the ``initial`` experiment: 'aggregate upto 2',
'maximum aggregation', 'upto ratio' (top-rho).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from llm_inference_in_distributed_edge_networks_amd.config import Params  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.experiments import pythia_main  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.parallel.dist import shutdown  # noqa: E402

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", default="params.json")
    ap.add_argument("--device", default=None)
    ap.add_argument("--max-windows", type=int, default=None)
    a = ap.parse_args()
    p = Params.load(a.params, device=a.device, max_windows=a.max_windows)
    p.model = p.model or "pythia-70m"
    pythia_main(p)
    shutdown()  # all ranks done: barrier + destroy the process group before interpreter exit
