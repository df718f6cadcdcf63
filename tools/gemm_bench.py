"""Time the gfx950 GEMM kernel (all model shapes/epilogues) against torch.matmul (hipBLASLt) on random data.

Interleaved rounds in one process (guide §5.4 rule 24); prints median TFLOP/s per shape."""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_inference_in_distributed_edge_networks_amd import ops  # noqa: E402

SHAPES = {  # name: (M, N, K, act, bias, resid)
    "qkv": (8192, 1152, 896, None, True, False),
    "o_proj": (8192, 896, 896, None, False, True),
    "gate_up": (8192, 9728, 896, "swiglu_il", False, False),
    "down": (8192, 896, 4864, None, False, True),
    "lm_head": (512, 151936, 896, None, False, False),
    "down_b64": (32768, 896, 4864, None, False, True),
    "o_proj_b64": (32768, 896, 896, None, False, True),
    "gate_up_b64": (32768, 9728, 896, "swiglu_il", False, False),
    "big": (8192, 8192, 8192, None, False, False),
    "qkv_rope_b64": (32768, 1152, 896, "qkv_rope", True, False),   # fused QKV + bias + RoPE + scatter epilogue
    # fp32 execution mode (h3 split-fp16 operands, K' = 3K): TF/s below count the fp16 MFMA work (3x the fp32 FLOPs)
    "h3_gate_up_b64": (32768, 9728, 3 * 896, "h3_swiglu", False, False),
    "h3_down_b64": (32768, 896, 3 * 4864, "h3", False, True),
    "h3_o_proj_b64": (32768, 896, 3 * 896, "h3", False, True),
    "h3_big": (8192, 8192, 3 * 1024, "h3", False, False),
    "h3_qkv_rope_b64": (32768, 1152, 3 * 896, "h3_qkv_rope", True, False),
    # epilogue-cost ablation of the h3 gate/up shape: plain fp32 output
    "h3_gate_up_f32out": (32768, 9728, 3 * 896, "h3", False, False),
    # two-product h3 GEMMs (weights exact in fp16, the bench's checkpoint-valued weights): K' = 2K
    "h3_2t_gate_up_b64": (32768, 9728, 2 * 896, "h3_swiglu", False, False),
    "h3_2t_down_b64": (32768, 896, 2 * 4864, "h3", False, True),
    "h3_2t_o_proj_b64": (32768, 896, 2 * 896, "h3", False, True),
    "h3_2t_qkv_rope_b64": (32768, 1152, 2 * 896, "h3_qkv_rope", True, False),
    # the production fp32 QKV: K / V^T also emitted as the attention's h3 planes (no fp32 V^T)
    "h3_2t_qkv_rope_kvp_b64": (32768, 1152, 2 * 896, "h3_qkv_rope_kvp", True, False),
}


def timeit(fn, iters):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--m", type=int, default=0, help="override M")
    ap.add_argument("--json", default="")
    ap.add_argument("--only", default="", help="comma list of shapes")
    ap.add_argument("--tiles", default="0", help="comma list of forced tiles: 0 = automatic, 128, 192, 224, 256")
    ap.add_argument("--no-lib", action="store_true", help="skip the hipBLASLt comparison (profiling)")
    a = ap.parse_args()
    dev = "cuda"
    res = {}
    for name, (M, N, K, act, bias, resid) in SHAPES.items():
        if a.only and name not in a.only.split(","):
            continue
        M = a.m or M if name != "lm_head" else M
        h3 = act is not None and act.startswith("h3")
        # h3 shapes: K is the GEMM's K' = 3 x plane width; the activation is stored once per plane ([M, 2K'/3])
        dt = torch.float16 if h3 else torch.bfloat16
        kp = (K // 2 if "_2t_" in name else K // 3) if h3 else K   # plane width of the h3 activation
        x = (torch.rand(M, 2 * kp if h3 else K, device=dev) * 2 - 1).to(dt)
        two = h3 and "_2t_" in name   # single-plane weight [N, K'/2] (the two-product GEMM)
        w = ((torch.rand(N, K // 2 if two else K, device=dev) * 2 - 1) / K ** 0.5).to(dt)
        b = torch.randn(N, device=dev).to(torch.float32 if h3 else torch.bfloat16) if bias else None
        No = N // 2 if act in ("swiglu_il", "h3_swiglu") else N
        r = torch.randn(M, No, device=dev).to(torch.float32 if h3 else torch.bfloat16) if resid else None
        out = torch.empty(M, No, device=dev, dtype=torch.float32 if h3 else torch.bfloat16)
        tiles = a.tiles.split(",")

        def mk(spec):
            def f():
                ops.set_gemm_tile(int(spec))
                if act == "qkv_rope":
                    ops.qkv_rope(x, w, b, cos, sin, M // 512, 512, 14, 2, 64, 64, 0.125)
                elif act == "h3_qkv_rope":
                    ops.qkv_rope_h3(x, w, 1.0, b, cos, sin, M // 512, 512, 14, 2, 64, 64, 0.125)
                elif act == "h3_qkv_rope_kvp":
                    ops.qkv_rope_h3(x, w, 1.0, b, cos, sin, M // 512, 512, 14, 2, 64, 64, 0.125, kv_scales=(1.0, 1.0))
                elif act == "h3_swiglu":
                    ops.linear_h3(x, w, 1.0, act="swiglu_il")
                elif act == "h3":
                    ops.linear_h3(x, w, 1.0, bias=b, residual=r, out=out)
                else:
                    ops.linear(x, w, bias=b, residual=r, act=act, out=out)
            return f
        if act in ("qkv_rope", "h3_qkv_rope", "h3_qkv_rope_kvp"):
            cos, sin = (t.to(dev) for t in ops.rope_tables(512, 64, 1e6))
        variants = {t: mk(t) for t in tiles}
        ours = variants[tiles[0]]
        xl = torch.cat([x, x[:, :K - 2 * kp]], 1) if h3 else x   # hipBLASLt reference: the same K' GEMM, plain operands
        wl = torch.cat([w, w], 1) if two else w
        lib = lambda: torch.matmul(xl, wl.t())  # noqa: E731
        if resid and not h3:  # hipBLASLt with the residual as beta*C (what a library route for RESID GEMMs would run)
            variants["libr"] = lambda: torch.addmm(r, x, w.t())
        for _ in range(3):
            ours(); lib()
        t_o, t_l = [], []
        t_v = {t: [] for t in variants}
        for _ in range(a.rounds):
            for t, f in variants.items():
                t_v[t].append(timeit(f, a.iters))
            t_o.append(min(statistics.median(t_v[t]) for t in tiles))
            t_l.append(timeit(lib, a.iters) if not a.no_lib else 1.0)
        ops.set_gemm_tile(0)
        fl = 2.0 * M * N * K
        for t, v in t_v.items():
            print(f"   tile={t:>4s}: {statistics.median(v)*1e6:8.1f}us {fl/statistics.median(v)/1e12:7.1f} TF", flush=True)
        res[name] = {"M": M, "N": N, "K": K, "ours_us": statistics.median(t_o) * 1e6,
                     "hipblaslt_us": statistics.median(t_l) * 1e6,
                     "ours_tflops": fl / statistics.median(t_o) / 1e12,
                     "hipblaslt_tflops": fl / statistics.median(t_l) / 1e12}
        print(f"{name:8s} M={M:6d} N={N:6d} K={K:5d}  ours {res[name]['ours_us']:8.1f}us "
              f"{res[name]['ours_tflops']:7.1f} TF | hipBLASLt (plain, no epilogue) {res[name]['hipblaslt_us']:8.1f}us "
              f"{res[name]['hipblaslt_tflops']:7.1f} TF", flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
