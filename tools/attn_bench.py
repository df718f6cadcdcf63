"""Flash-attention forward (bf16 and fp32 modes) at the bench shape (B windows x 512, 14 q / 2 kv heads, d=64)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from llm_inference_in_distributed_edge_networks_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--S", type=int, default=512)
    ap.add_argument("--Hq", type=int, default=14)
    ap.add_argument("--Hkv", type=int, default=2)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--fp32", action="store_true", help="the fp32-mode kernel: bf16 x6 planes / scaled fp16 h3 planes")
    a = ap.parse_args()
    if a.fp32:
        return bench_fp32(a)
    B, S, Hq, Hkv = a.B, a.S, a.Hq, a.Hkv
    g = torch.Generator().manual_seed(0)
    q = (torch.randn(B, Hq, S, 64, generator=g) * 0.125).bfloat16().cuda()
    k = torch.randn(B, Hkv, S, 64, generator=g).bfloat16().cuda()
    vt = torch.randn(B, Hkv, 64, ops.s_pad(S), generator=g).bfloat16().cuda()
    flop = 4.0 * B * Hq * 64 * sum(i + 1 for i in range(S))   # causal QK^T + PV
    res = {}
    for r in range(a.rounds):
        for v in (3,):
            for lse in (False, True):
                ops.attention(q, k, vt, S, need_lse=lse)
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                for _ in range(a.iters):
                    ops.attention(q, k, vt, S, need_lse=lse)
                en.record()
                torch.cuda.synchronize()
                us = st.elapsed_time(en) / a.iters * 1e3
                key = f"v{v}{'_lse' if lse else ''}"
                res.setdefault(key, []).append(us)
    out = {k_: {"us": round(min(v), 2), "TFLOPs": round(flop / min(v) * 1e-6, 1)} for k_, v in res.items()}
    print(json.dumps({"shape": [B, S, Hq, Hkv], **out}))


def bench_fp32(a):
    B, S, Hq, Hkv = a.B, a.S, a.Hq, a.Hkv
    g = torch.Generator().manual_seed(0)
    q = (torch.randn(B, Hq, S, 64, generator=g) * 0.125).cuda()
    k = torch.randn(B, Hkv, S, 64, generator=g).cuda()
    vt = torch.randn(B, Hkv, 64, ops.s_pad(S), generator=g).cuda()
    flop = 4.0 * B * Hq * 64 * sum(i + 1 for i in range(S))
    res = {}
    for _ in range(a.rounds):
        for name, sc in (("x6_bf16_mfma", None), ("h3_fp16_mfma", (1024.0, 1024.0, 1024.0))):
            for h3 in (0.0, 1.0):
                ops.attention(q, k, vt, S, need_lse=True, h3=h3, in_scales=sc)
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                for _ in range(a.iters):
                    ops.attention(q, k, vt, S, need_lse=True, h3=h3, in_scales=sc)
                en.record()
                torch.cuda.synchronize()
                res.setdefault(f"{name}{'_h3out' if h3 else ''}", []).append(st.elapsed_time(en) / a.iters * 1e3)
    out = {k_: {"us": round(min(v), 2), "TFLOPs_fp32": round(flop / min(v) * 1e-6, 1)} for k_, v in res.items()}
    print(json.dumps({"shape": [B, S, Hq, Hkv], "dtype": "fp32", **out}))


if __name__ == "__main__":
    main()
