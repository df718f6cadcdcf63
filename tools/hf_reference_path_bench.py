"""Same-node baseline: the reference's computation, written on stock HF transformers + PyTorch eager, on this GPU.

BASELINE.md's numbers are from a T4.  To compare against the reference's *implementation strategy* on the same
MI355X, this runs what the reference does per 512-token window (``/root/reference/Experiments/Qwen2-0.5B/main.py:
151-180``: one HF forward with ``output_attentions=True`` for the importance maps; then, per configuration, a
layer-by-layer HF forward that quantizes the ``ratio`` least important tokens of the boundary layer with one global
int4 scale, ``qwen_layer_wise.py:41-76``; shifted CE with the sliding-window targets) with HF Qwen2 modules of the
Qwen2-0.5B shape (random init, fp32, no download).  The code here is written for this harness from that description,
not taken from the reference.

``--configs 1`` is the work of one evaluated configuration (what ``bench.py`` does per window: config 3, column-mean
importance at layer 11, ratio 0.5); ``--configs 100`` is the reference's notebook sweep (4 methods x 5 layers x 5
ratios per window).  ``--batch 1`` is the reference's loop (one window per call); ``--batch 64`` the same work batched,
the best plain PyTorch eager can do with it.  Prints one JSON line.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from llm_inference_in_distributed_edge_networks_amd.eval.hf_reference import ReferencePath  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.models import get_config  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen2-0.5b")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--windows", type=int, default=32, help="timed windows")
    ap.add_argument("--warmup", type=int, default=2, help="untimed batches")
    ap.add_argument("--configs", type=int, default=1, help="quantized forwards per window (1 = bench, 100 = sweep)")
    ap.add_argument("--layer", type=int, default=11)
    ap.add_argument("--ratio", type=float, default=0.5)
    a = ap.parse_args()
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    cfg = get_config(a.model)
    ref = ReferencePath(cfg, dev)
    r = ref.throughput(a.batch, a.windows, a.warmup, a.configs, a.layer, a.ratio)
    print(json.dumps({"what": "reference computation on HF transformers + PyTorch eager (fp32)", "device": dev,
                      "gpu": torch.cuda.get_device_name(0) if dev == "cuda" else "cpu", "model": cfg.name, **r,
                      "torch": torch.__version__}), flush=True)


if __name__ == "__main__":
    main()
