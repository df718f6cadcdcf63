#!/usr/bin/env python
"""Bit-identity of the fp32 / bf16 pipeline step under heavy contention from another process on the same GPU.

The round-5 one-off wrong PPL of the 4-rank shared-GPU rehearsal (509.05 vs 503.23) would, if it came from a kernel,
be a read that depends on timing: an LDS / register value consumed before the load or LDS DMA that produces it has
landed (a missing or miscounted ``s_waitcnt``), which an idle GPU hides because its memory latency is short.  Four
ranks sharing the GPU raise the latency a little; this check raises it a lot.  A child process ("hog") streams 2 GiB
device copies and fp16 GEMMs back to back on the same GPU (its own HIP context, as another rank's) while this
process replays the bench step (BASELINE config 3: Qwen2-0.5B, 2-stage split after layer 11, column-mean importance,
mixed int4/int8 boundary at ratio 0.5, HIP graphs) on the same windows again and again.  Every window's NLL (fp64
bits, which the boundary message and every kernel upstream feed) must equal the idle run's exactly.

Usage: ``python tools/contention_check.py [--model qwen2-0.5b] [--batch 16] [--microbatches 4] [--repeats 4]``.
Prints one JSON line (and writes it to ``--out``); exit 1 on any difference.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def hog(seconds: float) -> None:
    """Child: device copies + fp16 GEMMs back to back until ``seconds`` have passed (never outlives its deadline)."""
    import torch
    dev = torch.device("cuda", 0)
    src = torch.empty(1 << 31, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    a = torch.randn(8192, 8192, device=dev, dtype=torch.float16)
    c = torch.empty_like(a)
    torch.cuda.synchronize()
    print("hog running", flush=True)
    t_end = time.time() + seconds
    n = 0
    while time.time() < t_end:
        dst.copy_(src)
        torch.matmul(a, a, out=c)
        n += 1
        if n % 4 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    print(f"hog done {n}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen2-0.5b")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--microbatches", type=int, default=4)
    ap.add_argument("--repeats", type=int, default=4)
    ap.add_argument("--dtypes", default="fp32,bf16")
    ap.add_argument("--hog-seconds", type=float, default=90.0)
    ap.add_argument("--hog-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    if a.hog_child:
        hog(a.hog_seconds)
        return

    import torch
    from llm_inference_in_distributed_edge_networks_amd.eval.data import synthetic_stream
    from llm_inference_in_distributed_edge_networks_amd.eval.windows import batches, sliding_windows
    from llm_inference_in_distributed_edge_networks_amd.models import build_model, get_config
    from llm_inference_in_distributed_edge_networks_amd.parallel import BoundaryConfig, LocalPipeline, PipelinePlan

    dev = torch.device("cuda", 0)
    cfg = get_config(a.model)
    toks = synthetic_stream(299_078, cfg.vocab_size, 0)
    wins = [w for w in sliding_windows(toks.shape[1], 512, 32) if w.length == 512]
    pool = [b.to(dev) for b in batches(toks, wins[: a.batch * a.microbatches], a.batch)]
    split = 11 if cfg.num_layers == 24 else cfg.num_layers // 2 - 1
    plan = PipelinePlan.from_split_layers(cfg.num_layers, [split])
    bcfg = BoundaryConfig("mixed_int4_int8", 0.5, "regular_importance")

    def step(pipe) -> torch.Tensor:
        out = [pipe.run_batch(b).double() for b in pool]
        torch.cuda.synchronize()
        return torch.stack(out).cpu()

    runs = {}
    for name in a.dtypes.split(","):
        dtype = {"fp32": torch.float32, "bf16": torch.bfloat16}[name]
        model, _ = build_model(cfg, dev, dtype, seed=0, values=torch.bfloat16)
        pipe = LocalPipeline(model, plan, bcfg)
        for _ in range(2):                      # eager, then capture: every later step replays the graphs
            step(pipe)
        runs[name] = {"pipe": pipe, "ref": step(pipe), "model": model}
        runs[name]["idle_identical"] = bool(torch.equal(step(pipe), runs[name]["ref"]))

    child = subprocess.Popen([sys.executable, os.path.abspath(__file__), "--hog-child", "--hog-seconds",
                              str(a.hog_seconds)], stdout=subprocess.PIPE, text=True)
    rows = []
    try:
        line = child.stdout.readline().strip()
        if line != "hog running":
            raise RuntimeError(f"hog did not start: {line!r}")
        for k in range(a.repeats):
            for name, r in runs.items():
                t0 = time.perf_counter()
                got = step(r["pipe"])
                dt = time.perf_counter() - t0
                d = (got - r["ref"]).abs()
                rows.append({"repeat": k, "dtype": name, "identical": bool(torch.equal(got, r["ref"])),
                             "max_abs_diff": float(d.max()), "differing": (d > 0).nonzero().tolist()[:16],
                             "step_s_under_hog": round(dt, 3)})
                print(json.dumps(rows[-1]), flush=True)
            if child.poll() is not None:
                break
    finally:
        if child.poll() is None:
            child.terminate()
        try:
            child.wait(timeout=60)
        except subprocess.TimeoutExpired:
            child.kill()
            child.wait()
    out = {"what": "per-window NLL bit-identity of the bench step (config 3, HIP graphs) while another process floods "
                   "the GPU with 2 GiB copies and fp16 GEMMs",
           "model": cfg.name, "windows_per_step": a.batch * a.microbatches,
           "idle_identical": {n: r["idle_identical"] for n, r in runs.items()},
           "under_contention": len(rows), "all_identical": all(r["identical"] for r in rows) and
           all(r["idle_identical"] for r in runs.values()) and len(rows) > 0, "rows": rows}
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "rows"}))
    sys.exit(0 if out["all_identical"] else 1)


if __name__ == "__main__":
    main()
