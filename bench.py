#!/usr/bin/env python
"""Headline benchmark: Qwen2-0.5B 2-stage split inference with an importance-quantized boundary.

Metric (BASELINE.json): WikiText-2 sliding-window PPL + inter-stage bytes/token, Qwen2-0.5B 2-stage
split; tokens/sec.  One step = ``--microbatches`` window batches of ``--batch`` windows
(max_length 512, stride 32: the reference recipe, ``Experiments/Qwen2-0.5B/params.json``) per
data-parallel replica, pushed through the 2-stage pipeline:

    stage 0: embed -> layers 0..L (importance at L) -> boundary codec encode -> RCCL send
    stage 1: RCCL recv -> decode -> layers L+1..23 -> final norm + LM head + CE on the scored rows

N GPUs -> pp=2 stages x dp=N/2 replicas (N=1: both stages on the one GPU, boundary still encoded
and decoded).  ``value`` = window tokens processed per second over the whole job (every window is
a full 512-token forward, as in the reference); scored tokens/s, PPL and measured wire bytes/token
are reported alongside.  Data: synthetic token stream of the WikiText-2 test length, random-init
weights of the exact Qwen2-0.5B architecture (no network / HF cache on the benchmark machines).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from llm_inference_in_distributed_edge_networks_amd import codec as C  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.data import synthetic_stream  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.windows import (batches, sliding_windows,  # noqa: E402
                                                                           window_nll)
from llm_inference_in_distributed_edge_networks_amd.models import build_model, get_config  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.parallel import (BoundaryConfig, DistributedPipeline,  # noqa: E402
                                                                      Grid, LocalPipeline, PipelinePlan,
                                                                      init_distributed)
from llm_inference_in_distributed_edge_networks_amd.parallel.dist import all_reduce_max_  # noqa: E402

# Reference throughput on its own hardware: the Qwen2 sweep ran 1 eager + 100 split
# forwards of 512 tokens per window at 16.03-16.35 s/window on a T4 = ~3.2k forward tokens/s.
BASELINE_TOKENS_PER_S = 3200.0


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--model", default="qwen2-0.5b")
    p.add_argument("--batch", type=int, default=64, help="windows per micro-batch")
    p.add_argument("--microbatches", type=int, default=0,
                   help="micro-batches per step per replica (default 4 x pipeline depth: every GPU does the "
                        "work of 4 full-model micro-batches per step at any N, i.e. weak scaling)")
    p.add_argument("--max-length", type=int, default=512)
    p.add_argument("--stride", type=int, default=32)
    p.add_argument("--split", type=int, default=11, help="last layer of stage 0 (reference layer_of_interest)")
    p.add_argument("--codec", default="mixed_int4_int8")
    p.add_argument("--ratio", type=float, default=0.5)
    p.add_argument("--method", default="regular_importance")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--transport", default="torch", choices=["torch", "rccl"],
                   help="stage hand-off: torch.distributed p2p (RCCL) or the native RCCL wrapper")
    p.add_argument("--no-graphs", action="store_true")
    p.add_argument("--json-out", default="")
    return p.parse_args()


def main():
    a = parse()
    env = init_distributed("auto")
    dev = env.device
    cfg = get_config(a.model)
    world = env.world_size
    pp = 2 if world >= 2 else 1
    grid = Grid(world, pp)
    if a.microbatches <= 0:
        a.microbatches = 4 * pp
    plan2 = PipelinePlan.from_split_layers(cfg.num_layers, [a.split])
    dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
    if pp == 1:
        model, prov = build_model(cfg, dev, dtype, seed=a.seed)
        runner = LocalPipeline(model, plan2, BoundaryConfig(a.codec, a.ratio, a.method), use_graphs=not a.no_graphs)
    else:
        dp_idx, stage = grid.coords(env.rank)
        lay = plan2.stage_layers(stage)
        model, prov = build_model(cfg, dev, dtype, seed=a.seed, layers=lay, with_embed=(stage == 0),
                                  with_head=(stage == pp - 1))
        runner = DistributedPipeline(model, plan2, BoundaryConfig(a.codec, a.ratio, a.method), grid, env.rank,
                                     use_graphs=not a.no_graphs, transport=a.transport)

    # ---- data: synthetic stream of WikiText-2 test length, HF sliding windows, staged on device
    tokens = synthetic_stream(299_078, cfg.vocab_size, a.seed)
    wins = [w for w in sliding_windows(tokens.shape[1], a.max_length, a.stride) if w.length == a.max_length]
    need = a.batch * a.microbatches * grid.dp
    pool = list(batches(tokens, wins[: need * 4], a.batch))
    pool = [b.to(dev) for b in pool]
    pool_w = [b.weights.to(dev) for b in pool]   # per-window loss weights, resident (no H2D copy per step)
    nll_acc = torch.zeros(2, dtype=torch.float64, device=dev)

    per_step = a.microbatches * grid.dp

    def mbs_for(first_step: int, nsteps: int):
        return [pool[(first_step * per_step + i) % len(pool)] for i in range(nsteps * per_step)]

    def wts_for(first_step: int, nsteps: int):
        return [pool_w[(first_step * per_step + i) % len(pool)] for i in range(nsteps * per_step)]

    def run_steps(first_step: int, nsteps: int):
        """nsteps consecutive steps.  pp=1: micro-batch by micro-batch on the local 2-stage pipeline.
        pp>1: one continuous pipeline over all nsteps*microbatches (stages stay busy across step
        boundaries; the only fill/drain is at the ends of the timed region)."""
        mbs = mbs_for(first_step, nsteps)
        if pp == 1:
            for b, w in zip(mbs, wts_for(first_step, nsteps)):
                wn = runner.run_batch(b)
                nll_acc[0] += (wn.double() * w).sum()   # device-side accumulation: no host sync per micro-batch
                nll_acc[1] += w.sum()
        else:
            acc, _ = runner.evaluate(mbs)
            nll_acc[0] += acc.total_nll
            nll_acc[1] += acc.n_tokens

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()
        if env.is_dist:
            torch.distributed.barrier()
            if dev.type == "cuda":
                torch.cuda.synchronize()

    run_steps(0, a.warmup)
    sync()
    nll_acc.zero_()
    t0 = time.perf_counter()
    run_steps(a.warmup, a.steps)
    sync()
    dt = time.perf_counter() - t0
    if env.is_dist:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        all_reduce_max_(t)
        dt = float(t.item())

    tok_per_step = grid.dp * a.microbatches * a.batch * a.max_length
    scored_per_step = grid.dp * a.microbatches * a.batch * a.stride
    value = tok_per_step * a.steps / dt
    spec = C.get_codec(a.codec)
    wire = C.message_bytes(spec, a.batch, a.max_length, cfg.hidden_size, a.ratio) / (a.batch * a.max_length)
    ppl = math.exp(float(nll_acc[0]) / float(nll_acc[1])) if (pp == 1 or env.rank == world - 1) and \
        float(nll_acc[1]) > 0 else None
    if env.is_dist:
        t = torch.tensor([ppl or 0.0], dtype=torch.float64, device=dev)
        all_reduce_max_(t)
        ppl = float(t.item())
    out = {
        "metric": "Qwen2-0.5B 2-stage split sliding-window PPL eval throughput (window tokens/sec)",
        "value": round(value, 1), "unit": "tokens/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(1000 * dt / a.steps, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": round(value / BASELINE_TOKENS_PER_S, 2), "dtype": "bf16" if dtype == torch.bfloat16 else "fp32",
        "data": "synthetic (WikiText-2-test-length Zipf token stream), random-init weights",
        "config": {"model": cfg.name, "global_batch": grid.dp * a.microbatches * a.batch, "seq_len": a.max_length,
                   "stride": a.stride, "parallelism": f"pp{pp}xdp{grid.dp}", "split_after_layer": a.split,
                   "codec": a.codec, "ratio": a.ratio, "importance": a.method,
                   "transport": a.transport if pp > 1 else "local", "hip_graphs": not a.no_graphs},
        "scored_tokens_per_s": round(scored_per_step * a.steps / dt, 1),
        "wire_bytes_per_token": round(wire, 2),
        "wire_bits_per_element": round(8 * wire / cfg.hidden_size, 3),
        "wire_compression_vs_bf16": round(2 * cfg.hidden_size / wire, 3),
        "wire_compression_vs_fp32_reference": round(4 * cfg.hidden_size / wire, 3),
        "ppl_random_weights": ppl, "weights": prov,
    }
    if env.is_main:
        print(json.dumps(out), flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                json.dump(out, f, indent=1)
    if env.is_dist:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
