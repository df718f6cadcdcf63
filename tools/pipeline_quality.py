"""PPL vs wire bytes through the real multi-boundary pipeline (BASELINE configs 3-5) on a trained model.

The reference quantizes ONE boundary (``Experiments/Qwen2-0.5B/qwen_layer_wise.py:54-70``).  BASELINE configs 4
and 5 quantize at every boundary of a 4- and an 8-stage split, so the quantization error compounds over 3 and 7
boundaries - something random weights cannot show (their PPL is ~|V| whatever happens).  This runs the
``LocalPipeline`` (every stage encodes its outgoing boundary with the codec and the next one decodes it, exactly the
message the RCCL transport carries) on the byte-level Qwen2 trained by ``tools/train_tiny_lm.py``, at fp32:

* pp in {2, 4, 8} (cost-balanced stages; pp 8 = one layer per stage), importance method per config
  (config 3: column-mean ``regular_importance``; config 4: ``last_row``; config 5: ``weighted_importance`` from
  the LRP head table), plus ``last_row`` at every depth so the compounding is visible on one method;
* codecs: the config's codec, the reference Q1 (``ref_int4_global``) at every boundary, and for config 5 the
  head-group codec with allocated plans against the same codec with uniform plans (same bits): "sens" = the MSE
  allocation over the groups' quantization sensitivity on the widths 2-8 (``codec.wire.allocate_group_bits``), "rel"
  = round 3's first-order allocation over the LRP relevance on 2 / 4 / 8 bits;
* ratios {0, .25, .5, .75, 1}; PPL on held-out text and the measured wire bytes per token per boundary; for every
  allocated plan, the paired window-bootstrap 95 % interval of log PPL(plan) - log PPL(uniform) at each ratio
  (``eval.stats``).

The LRP tables (head weights for ``weighted_importance``, channel-group relevance and sensitivity for the head-group
plans) are calibrated first on training text with the fp32 relevance engine.  Output: JSON + markdown tables.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from llm_inference_in_distributed_edge_networks_amd.eval import stats  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.data import local_text_bytes  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.windows import batches, sliding_windows  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.models import DecoderLM, get_config  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.parallel import (BoundaryConfig, LocalPipeline,  # noqa: E402
                                                                      PipelinePlan)
from llm_inference_in_distributed_edge_networks_amd.relevance.attnlrp import (head_relevance_batched,  # noqa: E402
                                                                              normalize_per_layer)

# (pp, method, codec, plan) rows; plan: "rel" = relevance-allocated head-group widths, "uniform" = the same average
# width in every group, "-" = not a head-group codec
GRID = [
    # config 3: 2-stage, column-mean importance, mixed int4/int8 per token
    (2, "regular_importance", "mixed_int4_int8", "-"), (2, "regular_importance", "ref_int4_global", "-"),
    # the compounding of last_row + mixed int4/int8 over 1, 3 and 7 boundaries (config 4 is the pp 4 row)
    (2, "last_row", "mixed_int4_int8", "-"), (4, "last_row", "mixed_int4_int8", "-"),
    (4, "last_row", "ref_int4_global", "-"), (8, "last_row", "mixed_int4_int8", "-"),
    (8, "last_row", "ref_int4_global", "-"),
    # config 5: 8-stage, LRP-weighted importance, allocated head-group quantization ("@bits" = average width of the
    # group-quantized rows)
    (8, "weighted_importance", "mixed_rgroup_int8", "sens"), (8, "weighted_importance", "mixed_rgroup_int8", "rel"),
    (8, "weighted_importance", "mixed_rgroup_int8", "uniform"),
    (8, "weighted_importance", "mixed_rgroup_int8@3", "sens"), (8, "weighted_importance", "mixed_rgroup_int8@3", "rel"),
    (8, "weighted_importance", "mixed_rgroup_int8@3", "uniform"),
    (8, "weighted_importance", "mixed_int4_int8", "-"), (8, "weighted_importance", "ref_int4_global", "-"),
    (8, "last_row", "mixed_rgroup_int8@3", "rel"), (8, "last_row", "mixed_rgroup_int8@3", "uniform"),
    (8, "weighted_importance", "rgroup@3", "rel"), (8, "weighted_importance", "rgroup@3", "uniform"),
]


def stage_plan(cfg, pp: int, splits: str) -> PipelinePlan:
    if splits == "bench":
        from llm_inference_in_distributed_edge_networks_amd.models import QWEN2_0_5B
        if cfg.num_layers != QWEN2_0_5B.num_layers:
            raise ValueError("--splits bench needs a model with Qwen2-0.5B's 24 layers")
        if pp == 2:   # bench.py --split 11 (the reference notebook's middle layer)
            return PipelinePlan.from_split_layers(cfg.num_layers, [11])
        return PipelinePlan(cfg.num_layers, PipelinePlan.balanced(QWEN2_0_5B, pp, 512, 32 / 512).bounds)
    return PipelinePlan.balanced(cfg, pp, 512)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="byte-qwen2")
    ap.add_argument("--weights", default="/tmp/byte_qwen2.safetensors")
    ap.add_argument("--windows", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--ratios", default="0,0.25,0.5,0.75,1")
    ap.add_argument("--group-bits", type=float, default=4.0, help="average bits of the head-group codecs")
    ap.add_argument("--relevance-windows", type=int, default=256)
    ap.add_argument("--bos", type=int, default=-1,
                    help="start-of-window token put at position 0 of every window (as the model was trained with "
                         "tools/train_tiny_lm.py --bos); -1: none")
    ap.add_argument("--json-out", default="gpurun_out/pipeline_quality.json")
    ap.add_argument("--splits", default="balanced", choices=["balanced", "bench"],
                    help="stage boundaries: cost-balanced for this model, or the bench's splits for Qwen2-0.5B "
                         "(pp 2: after layer 11; pp 4 / 8: balanced with the 151936-row LM head) - the same layer "
                         "indices on a 24-layer model")
    a = ap.parse_args()
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    cfg = get_config(a.model)
    m = DecoderLM.load_native(cfg, a.weights, dev, torch.float32)
    ratios = [float(x) for x in a.ratios.split(",")]

    t0 = time.time()
    tr = local_text_bytes("train")
    wins = sliding_windows(tr.shape[1], 512, 512)[: a.relevance_windows]
    acc = torch.zeros(cfg.num_layers, cfg.num_heads, dtype=torch.float64, device=dev)
    cacc = torch.zeros(cfg.num_layers, cfg.hidden_size // 64, dtype=torch.float64, device=dev)
    sacc = torch.zeros_like(cacc)
    if dev == "cuda":
        from llm_inference_in_distributed_edge_networks_amd.relevance.engine_f32 import RelevanceEngineH3
        eng = RelevanceEngineH3(m)
        run = lambda ids: eng.head_relevance(ids, want_channels=True, want_sens=True)   # noqa: E731
    else:
        run = lambda ids: head_relevance_batched(m, ids, want_sens=True)                 # noqa: E731
    for b in batches(tr, wins, 16, bos=a.bos if a.bos >= 0 else None):
        rel, _, _, chan, sens = run(b.ids.to(dev))
        acc += rel.double().sum(0)
        cacc += chan.double().sum(0)
        sacc += sens.double().sum(0)
    hw = normalize_per_layer(acc).float().cpu()
    grel = normalize_per_layer(cacc).float().cpu()
    gsens = (sacc / sacc.mean(-1, keepdim=True).clamp_min(1e-300)).float().cpu()
    tables = {"sens": {"relevance": grel, "sensitivity": gsens}, "rel": grel, "uniform": None, "-": None}
    print(f"relevance (fp32 engine): {len(wins)} windows in {time.time() - t0:.1f}s", flush=True)

    ev = local_text_bytes("eval")
    wins = sliding_windows(ev.shape[1], 512, 32)[: a.windows]
    bl = [b.to(dev) for b in batches(ev, wins, a.batch, bos=a.bos if a.bos >= 0 else None)]
    out = {"model": cfg.name, "weights": a.weights, "dtype": "fp32", "device": dev,
           "data": f"python-stdlib-bytes/eval, {len(wins)} windows (max_length 512, stride 32)",
           "ratios": ratios, "group_avg_bits": a.group_bits, "head_weights": hw.tolist(),
           "channel_group_relevance": grel.tolist(), "channel_group_sensitivity": gsens.tolist(), "rows": []}
    win_nll = {}   # row index -> per ratio: per-window NLL [N] (for the paired intervals)
    weights = None
    for pp, meth, codec_spec, plan in GRID:
        t0 = time.time()
        codec, _, bits = codec_spec.partition("@")
        gbits = float(bits) if bits else a.group_bits
        pplan = stage_plan(cfg, pp, a.splits)
        row = {"pp": pp, "boundaries": pplan.boundary_layers(), "method": meth, "codec": codec_spec, "plan": plan,
               "group_avg_bits": gbits, "ppl": [], "wire_bytes_per_token": []}
        pipe = None
        per_ratio = []
        for r in ratios:
            bc = BoundaryConfig(codec, r, meth, hw, group_relevance=tables[plan], group_avg_bits=gbits)
            if pipe is None:
                pipe = LocalPipeline(m, pplan, bc)
            else:
                pipe.set_boundary(bc)     # one pipeline per row: its graphs are dropped, not left to the collector
            wn = []
            row["ppl"].append(pipe.evaluate(bl, on_batch=lambda b, x: wn.append(x.detach().float().cpu())).ppl())
            per_ratio.append(torch.cat(wn))
            if weights is None:
                weights = torch.cat([b.weights.float().cpu() for b in bl])
            wb = pipe.wire_bytes_per_token()
            row["wire_bytes_per_token"].append(sum(wb) / len(wb))
            if plan != "-" and r == 0.5:
                row["group_plans"] = {str(s.boundary): list(s.spec_out.plan) for s in pipe.stages[:-1]}
        pipe.graphs.clear()
        row["seconds"] = round(time.time() - t0, 2)
        win_nll[len(out["rows"])] = per_ratio
        out["rows"].append(row)
        print(f"pp{pp} {meth:20s} {codec_spec:20s} {plan:8s} " +
              "  ".join(f"{p:.4f}@{w:.0f}B" for p, w in zip(row["ppl"], row["wire_bytes_per_token"])), flush=True)

    lines = [f"# Multi-boundary pipeline quality: {cfg.name} (trained), fp32, {out['data']}", "",
             "PPL at each ratio (fraction of tokens in the low class), with the measured wire bytes per token per "
             "boundary (mean over boundaries) in parentheses.  fp32 activations = 2048 B/token.", "",
             "| stages | boundaries | method | codec | plan | " + " | ".join(f"r={r:g}" for r in ratios) + " |",
             "|---|---|---|---|---|" + "---|" * len(ratios)]
    for row in out["rows"]:
        cells = [f"{p:.4f} ({w:.0f})" if p < 1e4 else f"{p:.3g} ({w:.0f})"
                 for p, w in zip(row["ppl"], row["wire_bytes_per_token"])]
        lines.append(f"| {row['pp']} | {len(row['boundaries'])} | {row['method']} | {row['codec']} | {row['plan']} | "
                     + " | ".join(cells) + " |")
    # allocated plan vs the uniform plan of the same codec / bits / method / depth, paired over windows
    comps = []
    for ia, ra in enumerate(out["rows"]):
        if ra["plan"] not in ("sens", "rel"):
            continue
        for ib, rb in enumerate(out["rows"]):
            if (rb["plan"] == "uniform" and rb["codec"] == ra["codec"] and rb["method"] == ra["method"]
                    and rb["pp"] == ra["pp"]):
                cells = []
                for ri, r in enumerate(ratios):
                    nll = torch.stack([win_nll[ia][ri], win_nll[ib][ri]], 1)
                    cells.append(dict(stats.paired_diff(nll, weights, 0, 1, reps=1000, seed=ri), ratio=r))
                comps.append({"codec": ra["codec"], "method": ra["method"], "pp": ra["pp"], "plan": ra["plan"],
                              "vs": "uniform", "cells": cells})
    out["plan_vs_uniform"] = comps
    if comps:
        lines += ["", "Allocated plan vs the uniform plan (same bits): log PPL(plan) - log PPL(uniform), paired "
                  "window-bootstrap 95 % interval; negative = the allocated plan is better:", "",
                  "| method | codec | plan | " + " | ".join(f"r={r:g}" for r in ratios) + " | better at |",
                  "|---|---|---|" + "---|" * len(ratios) + "---|"]
        for c in comps:
            cells = [f"{x['diff']:+.2e} [{x['ci'][0]:+.1e}, {x['ci'][1]:+.1e}]" for x in c["cells"]]
            better = sum(1 for x in c["cells"] if x["ci"][1] < 0)
            lines.append(f"| {c['method']} | {c['codec']} | {c['plan']} | " + " | ".join(cells) +
                         f" | {better} of {len(ratios)} ratios |")
    plans = [r for r in out["rows"] if r.get("group_plans")]
    if plans:
        lines += ["", "Head-group bit plans per boundary (one digit per 64-channel group, ratio 0.5):", ""]
        for r in plans:
            lines.append(f"- {r['method']} / {r['codec']} / {r['plan']}: " +
                         "; ".join(f"after layer {b}: {''.join(str(x) for x in p)}" for b, p in r["group_plans"].items()))
    out["markdown"] = "\n".join(lines)
    print("\n" + out["markdown"], flush=True)
    os.makedirs(os.path.dirname(os.path.abspath(a.json_out)), exist_ok=True)
    with open(a.json_out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
