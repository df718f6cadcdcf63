"""Error of the fp32-mode GEMM operand schemes against fp64 (CPU study; csrc/common.h "h3").

For the model's GEMM shapes it prints the relative L2 and max errors of
  * the CPU fp32 GEMM (torch.matmul on fp32 operands, the yardstick "fp32-level"),
  * x6: three bf16 planes, six bf16 products (the previous fp32 mode),
  * h3: two fp16 planes of the power-of-two scaled operand, three fp16 products (the current fp32 mode), with the
    activation scale at the data's own maximum and 8 / 14 binades below it (the model's scales come from bounds
    that hold for any input, so they are looser than the data).
Products of 16-bit values are exact in fp32, so the plane GEMMs are emulated as fp32 GEMMs over the
K-concatenated planes, the way the MFMA accumulates them.

    python tools/h3_error.py [--out profiles/history/r02_h3_error.txt]
"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_inference_in_distributed_edge_networks_amd.ops import reference as R  # noqa: E402


def split_bf3(x):
    p0 = x.to(torch.bfloat16).float()
    r = x - p0
    p1 = r.to(torch.bfloat16).float()
    return p0, p1, (r - p1).to(torch.bfloat16).float()


def errs(y, ref):
    d = y.double() - ref
    return float(d.norm() / ref.norm()), float(d.abs().max() / ref.abs().max())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--m", type=int, default=512)
    a = ap.parse_args()
    torch.manual_seed(0)
    lines = ["shape (M x N x K), activation scale | rel L2 / rel max error vs fp64: "
             "cpu-fp32 | x6 (3 bf16 planes) | h3 | h3 (scale -8 binades) | h3 (scale -14 binades)"]
    cases = [("qkv / o_proj / gate_up K=896", 896, 896, 1.0), ("down K=4864", 896, 4864, 0.2),
             ("lm head K=896", 4096, 896, 3.0), ("outlier channels x30", 896, 896, 1.0)]
    for name, N, K, scale in cases:
        M = a.m
        x = torch.randn(M, K) * scale
        if "outlier" in name:
            x[:, :8] *= 30
        w = torch.randn(N, K) * 0.02
        ref = x.double() @ w.double().t()
        row = [errs(x @ w.t(), ref)]
        xa, wa = split_bf3(x), split_bf3(w)
        x6 = torch.cat([xa[2], xa[0], xa[1], xa[1], xa[0], xa[0]], 1) @ \
            torch.cat([wa[0], wa[2], wa[1], wa[0], wa[1], wa[0]], 1).t()
        row.append(errs(x6, ref))
        w3, sw = R.h3_weight(w)
        for slack in (0, 8, 14):
            sx = R.h3_scale(x.abs().max().item()) / 2 ** slack
            row.append(errs(R.h3_matmul(R.h3_act(x, sx), w3, 1.0 / (sx * sw)), ref))
        lines.append(f"{name:26s} {M}x{N}x{K} | " + " | ".join(f"{e2:.2e} / {em:.2e}" for e2, em in row))
    print("\n".join(lines))
    if a.out:
        with open(a.out, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
