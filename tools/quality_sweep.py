"""PPL-vs-compression sweep on a trained model and real text (the reference's experiment).

Runs the reference's 4 importance methods x boundary layers x ratios with several boundary codecs on the
held-out split of the local text corpus, using the byte-level model trained by ``tools/train_tiny_lm.py``.
LRP head weights for ``weighted_importance`` are calibrated first with the RelevanceEngine (reference C8)
on training text.  Prints one markdown table per codec and writes everything to ``--json-out``.
"""
import argparse
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from llm_inference_in_distributed_edge_networks_amd import codec as C  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.data import local_text_bytes  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.sweep import SweepConfig, SweepEngine, run_sweep  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.windows import batches, sliding_windows  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.models import DecoderLM, get_config  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.relevance.attnlrp import normalize_per_layer  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.relevance.engine import RelevanceEngine  # noqa: E402

METHODS = ["regular_importance", "weighted_importance", "last_row", "aggregate_till"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="byte-qwen2")
    ap.add_argument("--weights", default="/tmp/byte_qwen2.safetensors")
    ap.add_argument("--windows", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--layers", default="1,3,5,6")
    ap.add_argument("--ratios", default="0,0.25,0.5,0.75,1")
    ap.add_argument("--codecs", default="ref_int4_global,int4_token,mixed_int4_int8,mixed_int2_int8")
    ap.add_argument("--relevance-windows", type=int, default=256)
    ap.add_argument("--json-out", default="gpurun_out/quality_sweep.json")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"],
                    help="execution mode of the sweep (fp32 = the reference's precision)")
    a = ap.parse_args()
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    dtype = torch.bfloat16 if (dev == "cuda" and a.dtype == "bf16") else torch.float32
    cfg = get_config(a.model)
    m = DecoderLM.load_native(cfg, a.weights, dev, dtype)
    layers = [int(x) for x in a.layers.split(",")]
    ratios = [float(x) for x in a.ratios.split(",")]

    # LRP head weights (reference C8) on training text, 512-byte windows
    t0 = time.time()
    tr = local_text_bytes("train")
    wins = sliding_windows(tr.shape[1], 512, 512)[: a.relevance_windows]
    # LRP calibration at the sweep's precision: the fp32 engine (h3 GEMMs, fp32 attention rule) in fp32 mode on a GPU,
    # the bf16 engine in bf16 mode, the autograd rules on the CPU
    if dev == "cuda" and dtype == torch.float32:
        from llm_inference_in_distributed_edge_networks_amd.relevance.engine_f32 import RelevanceEngineH3
        eng = RelevanceEngineH3(m)
    else:
        eng = RelevanceEngine(m)
    acc = torch.zeros(cfg.num_layers, cfg.num_heads, dtype=torch.float64, device=dev)
    cacc = torch.zeros(cfg.num_layers, cfg.hidden_size // 64, dtype=torch.float64, device=dev)
    for b in batches(tr, wins, a.batch):
        rel, _, _, chan = eng.head_relevance(b.ids, want_channels=True)
        acc += rel.double().sum(0)
        cacc += chan.double().sum(0)
    hw = normalize_per_layer(acc).float().cpu()
    grel = normalize_per_layer(cacc).float().cpu()     # channel-group relevance: the head-group codecs' bit plans
    print(f"relevance: {len(wins)} windows in {time.time() - t0:.1f}s", flush=True)

    ev = local_text_bytes("eval")
    wins = sliding_windows(ev.shape[1], 512, 32)[: a.windows]
    out = {"model": cfg.name, "weights": a.weights, "dtype": a.dtype if dev == "cuda" else "fp32", "data": f"python-stdlib-bytes/eval, {len(wins)} windows "
           "(max_length 512, stride 32)", "methods": METHODS, "layers": layers, "ratios": ratios,
           "head_weights": hw.tolist(), "channel_group_relevance": grel.tolist(), "codecs": {}}
    # outlier structure of the boundary tensors: what a one-global-scale quantizer (ref_int4_global) is sensitive to.
    # peak/rms = max |x| over the batch / rms of x; token_peak = median over tokens of max_c |x_tc| / rms_t
    with torch.no_grad():
        b0 = next(iter(batches(ev, wins, a.batch)))
        x = m.embed(b0.ids)
        outl = {}
        for i in range(cfg.num_layers):
            x, _ = m.layer(i, x, b0.B, b0.S)
            if i in layers:
                xf = x.float()
                rms_t = xf.pow(2).mean(1).sqrt()
                xw = xf.view(b0.B, b0.S, -1)   # Q1 scales per window: |x| < max / 14 rounds to 0
                outl[i] = {"peak_over_rms": float(xf.abs().max() / xf.pow(2).mean().sqrt()),
                           "token_peak_over_rms_median": float((xf.abs().amax(1) / rms_t).median()),
                           "int4_global_zero_fraction": float((xw.abs() < xw.abs().amax((1, 2), keepdim=True) / 14)
                                                              .float().mean())}
    out["boundary_outliers"] = outl
    print("boundary outliers (peak/rms, median token peak/rms, fraction rounding to 0 under one global int4 scale): "
          + "; ".join(f"L{L}: {v['peak_over_rms']:.1f}, {v['token_peak_over_rms_median']:.1f}, "
                      f"{v['int4_global_zero_fraction']:.2f}" for L, v in sorted(outl.items())), flush=True)
    for codec in a.codecs.split(","):
        t0 = time.time()
        # head-group codecs: "name@bits" = relevance-allocated plans of that average width, "name@bitsu" = the
        # same width in every group (uniform plan, the ablation)
        base, _, bits = codec.partition("@")
        uniform = bits.endswith("u")
        avg = float(bits.rstrip("u") or 4.0)
        sc = SweepConfig(METHODS, layers, ratios, codec=base, head_weights=hw,
                         group_relevance=None if uniform else grel, group_avg_bits=avg)
        res = run_sweep(SweepEngine(m, sc), batches(ev, wins, a.batch))
        out["codecs"][codec] = {"avg_ppl_results": res["avg_ppl_results"],
                                "wire_bytes_per_token": res["wire_bytes_per_token"], "seconds": res["seconds"]}
        print(f"\n### {codec}  ({time.time() - t0:.1f}s)\n", flush=True)
        print("| method | layer | " + " | ".join(f"{r:g}" for r in ratios) + " |")
        print("|---|---|" + "---|" * len(ratios))
        for mi, meth in enumerate(METHODS):
            for li, L in enumerate(layers):
                row = res["avg_ppl_results"][mi][li]
                print(f"| {meth} | {L} | " + " | ".join(f"{v:.4f}" if v < 1e4 else f"{v:.3g}" for v in row) + " |")
        bpt = res["wire_bytes_per_token"][0][0]
        print("wire B/token per ratio: " + ", ".join(f"{b:.1f}" for b in bpt), flush=True)
        if C.wire.needs_plan(C.get_codec(base)):
            eng_ = SweepEngine(m, sc)
            plans = {L: list(eng_._spec_at(base, L).plan) for L in layers}
            out["codecs"][codec]["group_plans"] = plans
            print("group plans: " + "; ".join(f"layer {L}: {''.join(str(b) for b in p)}" for L, p in plans.items()))

    os.makedirs(os.path.dirname(os.path.abspath(a.json_out)), exist_ok=True)
    with open(a.json_out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
