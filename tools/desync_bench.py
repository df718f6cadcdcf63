"""Time the four-wave GEMMs of the fp32 bench step with the epilogue desync off and on, interleaved in one process
(cdna_hip_programming.md rule 24): gate/up + SwiGLU, O-projection + residual, down + residual, QKV + RoPE + planes,
LM head + LSE - at the bench shapes (one 64-window micro-batch, M = 32768; 2048 scored rows for the head).
Prints one JSON line per (op, split) with the median and min microseconds over the rounds."""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from llm_inference_in_distributed_edge_networks_amd import ops  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.ops import reference as R  # noqa: E402


def operands(M, N, K, seed, dev):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(M, K, generator=g)
    w = (torch.randn(N, K, generator=g) * 0.02).bfloat16().float()
    w3, sw = R.h3_weight(w)
    x3 = ops.split_h3(x.to(dev), 2.0 ** 10) if K <= 1024 else R.h3_act(x, 2.0 ** 10).to(dev)   # (the split kernel's row limit)
    return x3, w3.to(dev), 1.0 / (2.0 ** 10 * sw)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--splits", default="0,-1")
    ap.add_argument("--ops", default="gateup,oproj,down,qkv,lse")
    a = ap.parse_args()
    dev = "cuda"
    B, S, Hq, Hkv, H, I, V = 64, 512, 14, 2, 896, 4864, 151936
    M = B * S
    fns = {}
    sel = a.ops.split(",")
    if "gateup" in sel:
        x3, w3, al = operands(M, 2 * I, H, 1, dev)
        fns["gateup"] = lambda: ops.linear_h3(x3, w3, al, act="swiglu_il", out_scale=64.0)
    if "oproj" in sel:
        x3o, w3o, alo = operands(M, H, H, 2, dev)
        yo = torch.randn(M, H, device=dev)
        fns["oproj"] = lambda: ops.linear_h3(x3o, w3o, alo, residual=yo, out=yo)
    if "down" in sel:
        x3d, w3d, ald = operands(M, H, I, 3, dev)
        yd = torch.randn(M, H, device=dev)
        fns["down"] = lambda: ops.linear_h3(x3d, w3d, ald, residual=yd, out=yd)
    if "qkv" in sel:
        x3q, w3q, alq = operands(M, (Hq + 2 * Hkv) * 64, H, 4, dev)
        bias = torch.randn((Hq + 2 * Hkv) * 64, device=dev) * 0.02
        cos, sin = R.rope_tables(4096, 64, 1e6)
        cos, sin = cos.to(dev), sin.to(dev)
        fns["qkv"] = lambda: ops.qkv_rope_h3(x3q, w3q, alq, bias, cos, sin, B, S, Hq, Hkv, 64, 64, 0.125,
                                             kv_scales=(64.0, 64.0), need_k=False)
    if "lse" in sel:
        x3h, w3h, alh = operands(2048, V, H, 5, dev)
        tgt = torch.randint(0, V, (2048,), device=dev)
        fns["lse"] = lambda: ops.head_nll_h3(x3h, w3h, alh, tgt)
    splits = [int(s) for s in a.splits.split(",")]
    times = {(op, s): [] for op in fns for s in splits}
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for op, fn in fns.items():   # warm up every variant (workspace registration, first-launch attributes)
        for s in splits:
            ops.set_gemm_split(s)
            fn()
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for op, fn in fns.items():
            for s in splits:
                ops.set_gemm_split(s)
                fn()
                ev0.record()
                for _ in range(a.iters):
                    fn()
                ev1.record()
                ev1.synchronize()
                times[(op, s)].append(1e3 * ev0.elapsed_time(ev1) / a.iters)
    ops.set_gemm_split(0)
    for (op, s), t in times.items():
        print(json.dumps({"op": op, "split": s, "us_median": round(statistics.median(t), 1),
                          "us_min": round(min(t), 1), "rounds": a.rounds, "iters": a.iters}))


if __name__ == "__main__":
    main()
