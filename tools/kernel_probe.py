"""Run one fp32-mode kernel of the bench step at the bench shape a few times (for rocprofv3 --pmc passes and A/B).

Shapes: Qwen2-0.5B, one 64-window micro-batch of 512 tokens (M = 32768), bf16-valued weights (two-product h3 GEMMs).
  attn    fp32 flash attention, fp16 planes, h3 output (flash_attn_fwd_x6_kernel<true, 8, true>)
  qkv     h3 QKV GEMM + bias + RoPE + scatter (256x192 tiles)
  colsum  column-sum importance on the fp16 planes
  norm    fp32 RMSNorm -> h3 planes
  gateup  h3 gate/up GEMM + SwiGLU -> h3 planes (two products)
  down    h3 down GEMM + fp32 residual (two products)
  lrpattn       AttnLRP attention backward (delta + dK/dV with the GQA sum + dQ) on scaled fp16 planes (h3)
  gateupraw     the AttnLRP forward's gate/up: SwiGLU planes + the fp32 pre-activations from one GEMM
  gateup_lib / down_lib  hipBLASLt (torch.matmul) on the same fp16 operands and K' (no epilogue): the library's clock
                and MFMA rate under the same sustained load
  lrpmlp        AttnLRP MLP backward, dm GEMM with the SwiGLU rule in its epilogue (EPI_H3_LRP_SWIGLU)
  lrpmlp_split  the same as an fp32 dm GEMM + the rule's own pass (lrp_swiglu_bwd_h3_kernel), the round-4 path
Prints the mean time per call (events) as JSON."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from llm_inference_in_distributed_edge_networks_amd import ops  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.ops import reference as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", default="attn", choices=["attn", "qkv", "colsum", "norm", "gateup", "down",
                                                          "lrpmlp", "lrpmlp_split", "gateup_lib", "down_lib", "gateupraw",
                                                          "lrpattn"])
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--S", type=int, default=512)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--kv-planes", type=int, default=0,
                    help="attn: stage K / V^T h3 planes by LDS DMA; qkv: 1 emit the planes too, 2 the planes without "
                         "the fp32 K (the model's layers without importance statistics)")
    ap.add_argument("--save", default="", help="save the op's output tensors here (bit-exact A/B of two builds)")
    ap.add_argument("--compare", default="", help="compare the op's output bit for bit with a --save file")
    ap.add_argument("--tile", type=int, default=0, help="force the GEMM tile (ops.set_gemm_tile; 0 = by shape)")
    a = ap.parse_args()
    if a.tile:
        ops.set_gemm_tile(a.tile)
    B, S, Hq, Hkv, H = a.B, a.S, 14, 2, 896
    g = torch.Generator().manual_seed(0)
    dev = "cuda"
    if a.op in ("attn", "colsum"):
        q = (torch.randn(B, Hq, S, 64, generator=g) * 0.125).to(dev)
        k = torch.randn(B, Hkv, S, 64, generator=g).to(dev)
        vt = torch.randn(B, Hkv, 64, ops.s_pad(S), generator=g).to(dev)
        sc = (2.0 ** 12, 2.0 ** 12, 2.0 ** 12)
        _, lse = ops.attention(q, k, vt, S, need_lse=True, h3=2.0 ** 10, in_scales=sc)
        if a.op == "attn":
            kvp = None
            if a.kv_planes:
                kp, vp = R.kv_planes(k.cpu(), vt.cpu(), sc[1], sc[2])
                kvp = (kp.to(dev), vp.to(dev))
            fn = lambda: ops.attention(q, k, vt, S, need_lse=False, h3=2.0 ** 10, in_scales=sc,   # noqa: E731
                                       kv_planes=kvp)
        else:
            fn = lambda: ops.attn_colsum(q, k, lse, S, in_scales=sc[:2])                          # noqa: E731
    elif a.op == "qkv":
        x = torch.randn(B * S, H, generator=g)
        w = (torch.randn((Hq + 2 * Hkv) * 64, H, generator=g) * 0.02).bfloat16().float()
        w3, sw = R.h3_weight(w)
        x3 = ops.split_h3(x.to(dev), 2.0 ** 10)
        bias = (torch.randn((Hq + 2 * Hkv) * 64, generator=g) * 0.02).to(dev)
        cos, sin = R.rope_tables(4096, 64, 1e6)
        cos, sin, w3 = cos.to(dev), sin.to(dev), w3.to(dev)
        kvs = (2.0 ** 6, 2.0 ** 6) if a.kv_planes else None   # the K / V^T planes the attention stages by DMA
        # --kv-planes 2: planes only, no fp32 K (the model's layers that compute no importance statistics)
        fn = lambda: ops.qkv_rope_h3(x3, w3, 1.0 / (2.0 ** 10 * sw), bias, cos, sin, B, S, Hq, Hkv, 64, 64,  # noqa
                                     0.125, kv_scales=kvs, need_k=a.kv_planes != 2)
    elif a.op in ("gateup_lib", "down_lib"):   # the two-product K' = 2K as one plain fp16 GEMM
        K, N = (H, 9728) if a.op == "gateup_lib" else (4864, H)
        x = torch.randn(B * S, 2 * K, generator=g).half().to(dev)
        w = (torch.randn(N, 2 * K, generator=g) * 0.02).half().to(dev)
        fn = lambda: torch.matmul(x, w.t())   # noqa: E731
    elif a.op == "lrpattn":
        q = (torch.randn(B, Hq, S, 64, generator=g) * 0.125).to(dev)
        k = torch.randn(B, Hkv, S, 64, generator=g).to(dev)
        v = torch.randn(B, Hkv, S, 64, generator=g).to(dev)
        vt = torch.zeros(B, Hkv, 64, ops.s_pad(S), device=dev)
        vt[..., :S] = v.transpose(-1, -2)
        sc = (2.0 ** 12, 2.0 ** 12, 2.0 ** 12)
        o, lse = ops.attention(q, k, vt, S, need_lse=True, in_scales=sc)
        dO = torch.randn(B * S, Hq * 64, generator=g).to(dev)
        fn = lambda: ops.lrp_attn_bwd(q, k, v, o, dO, lse, gqa_sum=True, in_scales=sc)   # noqa: E731
    elif a.op == "gateupraw":
        x = torch.randn(B * S, H, generator=g)
        w = (torch.randn(9728, H, generator=g) * 0.02).bfloat16().float()
        w3, sw = R.h3_weight(w)
        x3, w3 = ops.split_h3(x.to(dev), 2.0 ** 10), w3.to(dev)
        fn = lambda: ops.linear_h3_swiglu_raw(x3, w3, 1.0 / (2.0 ** 10 * sw), 2.0 ** 6)   # noqa: E731
    elif a.op in ("gateup", "down"):   # h3 SwiGLU GEMM -> h3 planes / down GEMM + fp32 residual (two products)
        K, N = (H, 9728) if a.op == "gateup" else (4864, H)
        x = torch.randn(B * S, K, generator=g)
        w = (torch.randn(N, K, generator=g) * 0.02).bfloat16().float()
        w3, sw = R.h3_weight(w)
        x3 = ops.split_h3(x.to(dev), 2.0 ** 10) if K == H else R.h3_act(x, 2.0 ** 10).to(dev)
        w3 = w3.to(dev)
        if a.op == "gateup":
            fn = lambda: ops.linear_h3(x3, w3, 1.0 / (2.0 ** 10 * sw), act="swiglu_il", out_scale=2.0 ** 6)  # noqa
        else:
            res = torch.randn(B * S, N, generator=g).to(dev)
            fn = lambda: ops.linear_h3(x3, w3, 1.0 / (2.0 ** 10 * sw), residual=res)                      # noqa
    elif a.op.startswith("lrpmlp"):   # dx [T, H] -> d[gate|up] h3 planes [T, 4I] (I = 4864), two-product weights
        I = 4864
        wd = (torch.randn(H, I, generator=g) * 0.02).bfloat16().float()
        wgu = (torch.randn(2 * I, H, generator=g) * 0.02).bfloat16().float()
        w3, sw = R.h3_weight(wd.t().contiguous())
        w3 = w3.to(dev)
        c0 = ops.lrp_swiglu_scale(wd, wgu, torch.ones(H))
        dx3, rinv = ops.split_h3_dyn(torch.randn(B * S, H, generator=g).to(dev))
        gu = torch.randn(B * S, 2 * I, generator=g).to(dev)
        post = torch.rand(B * S, generator=g).to(dev)
        if a.op == "lrpmlp":
            fn = lambda: ops.linear_h3_lrp_swiglu(dx3, w3, 1.0 / sw, gu, c0, rinv, post=post)   # noqa: E731
        else:
            fn = lambda: ops.lrp_swiglu_bwd_h3(ops.linear_h3(dx3, w3, 1.0 / sw, rscale=rinv), gu, post=post)  # noqa
    else:
        x = torch.randn(B * S, H, generator=g).to(dev)
        w = (1 + 0.05 * torch.randn(H, generator=g)).to(dev)
        fn = lambda: ops.rmsnorm(x, w, 1e-6, h3=2.0 ** 10)                                       # noqa: E731
    out = fn()
    torch.cuda.synchronize()
    outs = [t.detach().cpu() for t in (out if isinstance(out, (tuple, list)) else (out,)) if torch.is_tensor(t)]
    if a.save:
        torch.save(outs, a.save)
    if a.compare:
        ref = torch.load(a.compare, weights_only=True)
        same = [bool(torch.equal(x, y)) for x, y in zip(outs, ref)]
        diff = [float((x.double() - y.double()).abs().max()) for x, y in zip(outs, ref)]
        print(json.dumps({"op": a.op, "bit_identical": same, "max_abs_diff": diff}))
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(a.iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    print(json.dumps({"op": a.op, "kv_planes": a.kv_planes, "tile": a.tile, "B": B, "S": S,
                      "us_per_call": round(st.elapsed_time(en) / a.iters * 1e3, 2)}))


if __name__ == "__main__":
    main()
