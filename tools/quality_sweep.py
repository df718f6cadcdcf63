"""PPL-vs-compression sweep on a trained model and real text (the reference's experiment).

Runs the reference's 4 importance methods x boundary layers x ratios with several boundary codecs on the
held-out split of the local text corpus, using the byte-level model trained by ``tools/train_tiny_lm.py``.
LRP head weights for ``weighted_importance`` are calibrated first with the RelevanceEngine (reference C8)
on training text.  Prints one markdown table per codec and writes everything to ``--json-out``.

Statistics (``eval.stats``): every window's NLL is kept, and each cell's damage against the unquantized ratio 0 gets
a paired window-bootstrap 95 % interval; ``findings`` tests the reference's three depth findings
(``Notebooks/qwen2-0.5B_experiment.ipynb`` JSON lines 557-588) on the Q1 quantizer with intervals:
(1) late boundaries hurt more (log PPL at the latest layer minus the others, per ratio), (2) last_row beats
column-mean importance at the late boundaries, (3) the one-global-scale collapse at ratio 1.
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
from llm_inference_in_distributed_edge_networks_amd.eval import stats  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.data import local_text_bytes  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.sweep import SweepConfig, SweepEngine, run_sweep  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.windows import batches, sliding_windows  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.models import DecoderLM, get_config  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.relevance.attnlrp import normalize_per_layer  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.relevance.engine import RelevanceEngine  # noqa: E402

METHODS = ["regular_importance", "weighted_importance", "last_row", "aggregate_till"]


def findings(flat, wts, layers, ratios, reps):
    """The reference's three depth findings on Q1 (``flat`` [N, methods x layers x ratios] per-window NLL), each a
    paired window-bootstrap interval of a log-PPL difference (positive = the first cell is worse)."""
    L_, R_ = len(layers), len(ratios)
    cell = lambda mi, li, ri: (mi * L_ + li) * R_ + ri                     # noqa: E731
    mi_reg, mi_last = METHODS.index("regular_importance"), METHODS.index("last_row")
    late = max(range(L_), key=lambda li: layers[li])
    out = {"late_boundaries_hurt_more": [], "last_row_beats_column_mean": [], "one_scale_collapse_at_ratio_1": []}
    for ri, r in enumerate(ratios):
        if r == 0:
            continue
        for li in range(L_):                                               # (1) latest layer vs each other layer
            if li != late:
                d = stats.paired_diff(flat, wts, cell(mi_last, late, ri), cell(mi_last, li, ri), reps, seed=ri)
                out["late_boundaries_hurt_more"].append(dict(d, method="last_row", late=layers[late],
                                                             other=layers[li], ratio=r))
        if r < 1:
            for li in sorted(range(L_), key=lambda i: -layers[i])[:2]:      # (2) at the two latest boundaries
                d = stats.paired_diff(flat, wts, cell(mi_reg, li, ri), cell(mi_last, li, ri), reps, seed=10 + ri)
                out["last_row_beats_column_mean"].append(dict(d, layer=layers[li], ratio=r))
    ri1 = ratios.index(1.0) if 1.0 in ratios else R_ - 1
    for li in range(L_):                                                   # (3) ratio 1 vs ratio 0
        d = stats.paired_diff(flat, wts, cell(mi_last, li, ri1), cell(mi_last, li, 0), reps, seed=20 + li)
        out["one_scale_collapse_at_ratio_1"].append(dict(d, layer=layers[li], rel=float(torch.tensor(d["diff"]).expm1())))
    return out


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
    ap.add_argument("--bos", type=int, default=-1,
                    help="start-of-window token put at position 0 of every window (as the model was trained with "
                         "tools/train_tiny_lm.py --bos); -1: none")
    ap.add_argument("--json-out", default="gpurun_out/quality_sweep.json")
    ap.add_argument("--boot", type=int, default=1000, help="window-bootstrap replicates of the intervals")
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
    sacc = torch.zeros_like(cacc)
    for b in batches(tr, wins, a.batch, bos=a.bos if a.bos >= 0 else None):
        rel, _, _, chan, sens = eng.head_relevance(b.ids, want_channels=True, want_sens=True)
        acc += rel.double().sum(0)
        cacc += chan.double().sum(0)
        sacc += sens.double().sum(0)
    hw = normalize_per_layer(acc).float().cpu()
    grel = normalize_per_layer(cacc).float().cpu()     # channel-group relevance and sensitivity: the head-group
    gsens = (sacc / sacc.mean(-1, keepdim=True).clamp_min(1e-300)).float().cpu()   # codecs' bit plans
    print(f"relevance: {len(wins)} windows in {time.time() - t0:.1f}s", flush=True)

    ev = local_text_bytes("eval")
    wins = sliding_windows(ev.shape[1], 512, 32)[: a.windows]
    out = {"model": cfg.name, "weights": a.weights, "dtype": a.dtype if dev == "cuda" else "fp32", "data": f"python-stdlib-bytes/eval, {len(wins)} windows "
           "(max_length 512, stride 32)", "methods": METHODS, "layers": layers, "ratios": ratios,
           "head_weights": hw.tolist(), "channel_group_relevance": grel.tolist(),
           "channel_group_sensitivity": gsens.tolist(), "codecs": {}}
    # outlier structure of the boundary tensors: what a one-global-scale quantizer (ref_int4_global) is sensitive to.
    # peak/rms = max |x| over the batch / rms of x; token_peak = median over tokens of max_c |x_tc| / rms_t
    with torch.no_grad():
        b0 = next(iter(batches(ev, wins, a.batch, bos=a.bos if a.bos >= 0 else None)))
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
        # head-group codecs: "name@bits" = plans of that average width allocated over the groups' sensitivity (MSE),
        # "name@bitsr" = over the LRP relevance (round 3's first-order allocator), "name@bitsu" = the same width in
        # every group (uniform plan, the ablation)
        base, _, bits = codec.partition("@")
        kind = bits[-1] if bits[-1:] in ("u", "r") else "s"
        avg = float(bits.rstrip("ur") or 4.0)
        table = {"u": None, "r": grel, "s": {"relevance": grel, "sensitivity": gsens}}[kind]
        sc = SweepConfig(METHODS, layers, ratios, codec=base, head_weights=hw, group_relevance=table,
                         group_avg_bits=avg)
        eng_s = SweepEngine(m, sc, keep_windows=True)
        res = run_sweep(eng_s, batches(ev, wins, a.batch, bos=a.bos if a.bos >= 0 else None))
        nll, wts = eng_s.window_results()            # [N, methods, layers, ratios], [N]
        flat = nll.reshape(nll.shape[0], -1)
        dmg = stats.damage_table(flat, wts, base=0, reps=a.boot, seed=1)   # cell 0 = (method 0, layer 0, ratio 0)
        R_ = len(ratios)
        cells = [[[dmg[(mi * len(layers) + li) * R_ + ri] for ri in range(R_)] for li in range(len(layers))]
                 for mi in range(len(METHODS))]
        out["codecs"][codec] = {"avg_ppl_results": res["avg_ppl_results"], "damage_ci": cells,
                                "wire_bytes_per_token": res["wire_bytes_per_token"], "seconds": res["seconds"],
                                "windows": int(nll.shape[0])}
        if base == "ref_int4_global":
            out["findings"] = findings(flat, wts, layers, ratios, a.boot)
        print(f"\n### {codec}  ({time.time() - t0:.1f}s)\n", flush=True)
        print("| method | layer | " + " | ".join(f"{r:g}" for r in ratios) + " |")
        print("|---|---|" + "---|" * len(ratios))
        for mi, meth in enumerate(METHODS):
            for li, L in enumerate(layers):
                row = res["avg_ppl_results"][mi][li]
                print(f"| {meth} | {L} | " + " | ".join(f"{v:.4f}" if v < 1e4 else f"{v:.3g}" for v in row) + " |")
        print("\ndamage vs ratio 0 (PPL / PPL_0 - 1, paired window-bootstrap 95 % interval):\n")
        print("| method | layer | " + " | ".join(f"{r:g}" for r in ratios) + " |")
        print("|---|---|" + "---|" * len(ratios))
        for mi, meth in enumerate(METHODS):
            for li, L in enumerate(layers):
                print(f"| {meth} | {L} | " + " | ".join(
                    f"{100 * c['rel']:+.2f}% [{100 * c['ci'][0]:+.2f}, {100 * c['ci'][1]:+.2f}]"
                    for c in cells[mi][li]) + " |")
        bpt = res["wire_bytes_per_token"][0][0]
        print("wire B/token per ratio: " + ", ".join(f"{b:.1f}" for b in bpt), flush=True)
        if C.wire.needs_plan(C.get_codec(base)):
            eng_ = SweepEngine(m, sc)
            plans = {L: list(eng_._spec_at(base, L).plan) for L in layers}
            out["codecs"][codec]["group_plans"] = plans
            print("group plans: " + "; ".join(f"layer {L}: {''.join(str(b) for b in p)}" for L, p in plans.items()))

    if "findings" in out:
        f = out["findings"]
        fmt = lambda d: f"{d['diff']:+.2e} [{d['ci'][0]:+.1e}, {d['ci'][1]:+.1e}] {d['verdict']}"   # noqa: E731
        print("\nfindings (Q1, paired window-bootstrap 95 % intervals of log-PPL differences):", flush=True)
        for d in f["late_boundaries_hurt_more"]:
            print(f"  late hurts more: last_row L{d['late']} - L{d['other']} at r={d['ratio']:g}: {fmt(d)}")
        for d in f["last_row_beats_column_mean"]:
            print(f"  column-mean - last_row at L{d['layer']} r={d['ratio']:g}: {fmt(d)}")
        for d in f["one_scale_collapse_at_ratio_1"]:
            print(f"  ratio 1 - ratio 0 at L{d['layer']} (last_row): {100 * d['rel']:+.2f}% {fmt(d)}")
    os.makedirs(os.path.dirname(os.path.abspath(a.json_out)), exist_ok=True)
    with open(a.json_out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
