#!/usr/bin/env python
"""Markdown summary of a sink-surrogate run (``scripts/gpu_r06d_sink.sh`` output directory).

Reads ``train.log`` (per-evaluation held-out loss and boundary outlier probes from ``tools/train_tiny_lm.py``),
``quality_sweep.json`` (``tools/quality_sweep.py``: the notebook sweep, three findings, codec tables) and, when present,
``pipeline_quality.json`` (``tools/pipeline_quality.py``: configs 3-5 and the head-group plans), and prints:

1. the training curve: held-out nats/byte and peak / RMS of the boundary tensors after the notebook layers, with the
   position-0 (start-of-window) token's share;
2. the reference's Q1 (one global int4 scale) at ratio 1 against per-token int4 and mixed int4/int8 at the same or
   fewer wire bytes, per boundary, with paired window-bootstrap 95 % intervals;
3. the three notebook findings;
4. (pipeline) the MSE-allocated head-group plans against the uniform plan.
"""
from __future__ import annotations

import argparse
import json
import math
import os


def training_curve(path):
    rows, cur = [], None
    with open(path) as f:
        for line in f:
            if line.startswith("step "):
                parts = line.split()
                cur = {"step": int(parts[1]), "held": float(line.split("held-out ")[1].split()[0])}
            elif line.startswith('{"probe_step"') and cur is not None:
                d = json.loads(line)
                if d["probe_step"] == cur["step"]:
                    cur["probe"] = {k: v for k, v in d.items() if k != "probe_step"}
                    rows.append(cur)
                    cur = None
            elif line.startswith('{"best_step"'):
                summ = json.loads(line)
                rows.append({"final": summ})
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--every", type=int, default=3, help="print every n-th evaluation of the training curve")
    a = ap.parse_args()
    for d in a.dirs:
        print(f"## {d}\n")
        tl = os.path.join(d, "train.log")
        if os.path.exists(tl):
            rows = training_curve(tl)
            curve = [r for r in rows if "probe" in r]
            final = next((r["final"] for r in rows if "final" in r), None)
            layers = sorted(curve[0]["probe"], key=int) if curve else []
            print("Training curve (held-out nats/byte; boundary peak / RMS over 8 held-out windows, position-0 token's "
                  "peak / RMS in brackets = the sink):\n")
            print("| step | held-out | " + " | ".join(f"L{L}" for L in layers) + " |")
            print("|---|---|" + "---|" * len(layers))
            for i, r in enumerate(curve):
                if i % a.every and i != len(curve) - 1:
                    continue
                p = r["probe"]
                print(f"| {r['step']} | {r['held']:.3f} | " + " | ".join(
                    f"{p[L]['peak_over_rms']:.1f} ({p[L]['pos0_peak_over_rms']:.1f} / rest {p[L]['rest_peak_over_rms']:.1f})"
                    for L in layers) + " |")
            if final:
                fp = final.get("final_probe", {})
                print(f"\nKept checkpoint: step {final['best_step']} of {final['steps']}, held-out "
                      f"{final['held_out_nats_per_byte']} nats/byte, train sample {final['train_sample_nats_per_byte']}, "
                      f"bos {final.get('bos')}, {final.get('excluded_eval_copies')} package files dropped as copies of "
                      f"held-out files.  Max boundary peak / RMS: "
                      + ", ".join(f"L{k} {v['peak_over_rms']}" for k, v in fp.items() if k != "probe_step") + "\n")
        qs = os.path.join(d, "quality_sweep.json")
        if os.path.exists(qs):
            q = json.load(open(qs))
            L, R, M = q["layers"], q["ratios"], q["methods"]
            ri1, ri0 = R.index(1.0), R.index(0.0)
            mi = M.index("last_row")
            out = q.get("boundary_outliers", {})
            print("Ratio 1 (every token quantized), `last_row` rows, PPL and damage vs ratio 0 (paired window-bootstrap "
                  "95 % interval), wire bytes per token:\n")
            codecs = list(q["codecs"])
            print("| layer | peak / RMS | " + " | ".join(codecs) + " |")
            print("|---|---|" + "---|" * len(codecs))
            for li, Lr in enumerate(L):
                cells = []
                for c in codecs:
                    cc = q["codecs"][c]
                    ppl = cc["avg_ppl_results"][mi][li][ri1]
                    dm = cc["damage_ci"][mi][li][ri1]
                    wb = cc["wire_bytes_per_token"][mi][li][ri1]
                    cells.append(f"{ppl:.4g} ({100 * dm['rel']:+.3g} % [{100 * dm['ci'][0]:+.3g}, "
                                 f"{100 * dm['ci'][1]:+.3g}]; {wb:.0f} B)")
                po = out.get(str(Lr), {}).get("peak_over_rms", float("nan"))
                print(f"| {Lr} | {po:.1f} | " + " | ".join(cells) + " |")
            base = q["codecs"][codecs[0]]["avg_ppl_results"][mi][0][ri0]
            print(f"\nUnquantized PPL {base:.4f} ({math.log(base):.4f} nats/byte).\n")
            f = q.get("findings")
            if f:
                fmt = lambda x: f"{x['diff']:+.2e} [{x['ci'][0]:+.1e}, {x['ci'][1]:+.1e}] {x['verdict']}"  # noqa: E731
                print("Findings (Q1; log-PPL differences, paired window-bootstrap 95 % intervals; 'a worse' = the first "
                      "cell is worse):\n")
                print("- late boundaries hurt more (`last_row` at L23 minus the other layers):")
                for x in f["late_boundaries_hurt_more"]:
                    print(f"  - r={x['ratio']:g} L{x['late']} - L{x['other']}: {fmt(x)}")
                print("- `last_row` beats the column mean at the late boundaries (column mean minus last_row):")
                for x in f["last_row_beats_column_mean"]:
                    print(f"  - L{x['layer']} r={x['ratio']:g}: {fmt(x)}")
                print("- the one-scale collapse at ratio 1 (ratio 1 minus ratio 0, `last_row`):")
                for x in f["one_scale_collapse_at_ratio_1"]:
                    print(f"  - L{x['layer']}: x{math.exp(x['diff']):.1f} PPL, {fmt(x)}")
                print()
        pq = os.path.join(d, "pipeline_quality.json")
        if os.path.exists(pq):
            p = json.load(open(pq))
            print("Pipeline (BASELINE configs 3-5: 1 / 3 / 7 quantized boundaries), the tool's own tables:\n")
            print(p.get("markdown", ""))
            print()


if __name__ == "__main__":
    main()
