"""AttnLRP head-relevance calibration throughput (reference C8: Experiments/Relevance/main.py).

Reference: 9,331 windows of 512 tokens in 1 h 17 m 20 s on a T4 with lxt + gradient checkpointing
(``Notebooks/attention_head_weights_via_relevance.ipynb`` JSON lines 5674, 18358) = ~1.0k tokens/s.
Here: Qwen2-0.5B architecture, random-init weights, synthetic windows of 512 tokens, the batched
RelevanceEngine (forward with saves + explicit AttnLRP backward on the gfx950 kernels).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from llm_inference_in_distributed_edge_networks_amd.models import DecoderLM, get_config  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.relevance.engine import RelevanceEngine  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.relevance.engine_f32 import RelevanceEngineH3  # noqa: E402

REF_TOKENS_PER_S = 9331 * 512 / (77 * 60 + 20)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen2-0.5b")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"],
                    help="fp32: the reference-precision engine (h3 GEMMs, fp32 attention rule); bf16: bf16 storage")
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    cfg = get_config(a.model)
    if a.dtype == "fp32":   # bf16-valued fp32 weights: what the reference computes with (HF bf16 checkpoint upcast)
        m = DecoderLM.random_init(cfg, 0, device="cuda", dtype=torch.float32, values=torch.bfloat16)
        eng = RelevanceEngineH3(m)
    else:
        m = DecoderLM.random_init(cfg, 0, device="cuda", dtype=torch.bfloat16)
        eng = RelevanceEngine(m)
    ids = torch.randint(0, cfg.vocab_size, (a.batch, a.seq), generator=torch.Generator().manual_seed(0)).cuda()
    for _ in range(a.warmup):
        rel, _, _ = eng.head_relevance(ids)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        rel, _, _ = eng.head_relevance(ids)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.iters
    tps = a.batch * a.seq / dt
    out = {"metric": "AttnLRP head-relevance pass throughput (fwd + LRP bwd)", "model": cfg.name,
           "batch_windows": a.batch, "seq_len": a.seq, "ms_per_batch": round(dt * 1e3, 3),
           "tokens_per_s": round(tps, 1), "reference_tokens_per_s_T4": round(REF_TOKENS_PER_S, 1),
           "vs_reference": round(tps / REF_TOKENS_PER_S, 1), "finite": bool(torch.isfinite(rel).all()),
           "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2**30, 2),
           "data": "synthetic ids, random-init weights", "dtype": a.dtype}
    print(json.dumps(out), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
