"""Throughput of the reference's own workload: the Qwen2-0.5B importance sweep of
``Notebooks/qwen2-0.5B_experiment.ipynb`` (4 methods x layers [22,18,3,23,11] x ratios
[0,.25,.5,.75,1], int4 global-scale boundary quantization, max_length 512, stride 32).

The reference ran 1 eager + 100 split forwards per window at 16.03-16.35 s/window on a T4
(BASELINE.md).  Here the shared-prefix sweep engine runs one prefix forward per window batch plus
one stacked suffix forward per boundary layer.  Reports windows/s and the speed-up vs 16.19 s/window.
Random-init weights + synthetic tokens (throughput only; PPL values are not comparable)."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_inference_in_distributed_edge_networks_amd.eval.data import synthetic_stream  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.sweep import SweepConfig, SweepEngine  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.windows import batches, sliding_windows  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.models import build_model, get_config  # noqa: E402

T4_SECONDS_PER_WINDOW = 16.19


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen2-0.5b")
    ap.add_argument("--windows", type=int, default=256)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--warmup-batches", type=int, default=2)
    ap.add_argument("--json-out", default="")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"],
                    help="fp32 = the reference's precision (h3 GEMMs); bf16 = the bf16 mode")
    ap.add_argument("--weight-values", default="bf16", choices=["bf16", "fp32"],
                    help="random weight values: bf16 as the HF checkpoint the reference upcasts, or full fp32")
    a = ap.parse_args()
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    dtype = torch.bfloat16 if (dev == "cuda" and a.dtype == "bf16") else torch.float32
    cfg = get_config(a.model)
    model, prov = build_model(cfg, dev, dtype, seed=0,
                              values=torch.bfloat16 if a.weight_values == "bf16" else None)
    layers = [22, 18, 3, 23, 11] if cfg.num_layers == 24 else [1, 2]
    hw = torch.full((cfg.num_layers, cfg.num_heads), 1.0 / cfg.num_heads)
    sc = SweepConfig(["regular_importance", "weighted_importance", "last_row", "aggregate_till"], layers,
                     [0, 0.25, 0.5, 0.75, 1], codec="ref_int4_global", head_weights=hw)
    toks = synthetic_stream(299_078, cfg.vocab_size, 0)
    wins = [w for w in sliding_windows(toks.shape[1], 512, 32) if w.length == 512][1:]
    bl = [b.to(dev) for b in batches(toks, wins[: (a.windows + a.warmup_batches * a.batch)], a.batch)]
    eng = SweepEngine(model, sc)
    for b in bl[: a.warmup_batches]:
        eng.run_batch(b)
    if dev == "cuda":
        torch.cuda.synchronize()
    eng = SweepEngine(model, sc)
    t0 = time.perf_counter()
    for b in bl[a.warmup_batches:]:
        eng.run_batch(b)
    if dev == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    n = eng.windows_done
    out = {"workload": "Qwen2 notebook sweep (4 methods x 5 layers x 5 ratios, ref_int4_global)",
           "windows": n, "seconds": dt, "windows_per_s": n / dt, "s_per_window": dt / n,
           "speedup_vs_T4_reference": T4_SECONDS_PER_WINDOW / (dt / n),
           "forward_tokens_per_s": eng.forward_tokens / dt, "dtype": str(dtype), "weights": prov,
           "data": "synthetic", "batch": a.batch}
    print(json.dumps(out))
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
