"""Summarise the quality campaign over seeds (scripts/gpu_r05c_quality.sh outputs) as markdown.

Usage: python tools/quality_seeds.py <seed dir> [<seed dir> ...] > summary.md

Each seed dir holds train.log (last line: the trainer's JSON summary), quality_sweep.json (the notebook sweep with
per-cell window-bootstrap intervals and the three findings) and pipeline_quality.json (configs 3-5 with the head-group
plans against the uniform plan).  Per finding and seed: the paired log-PPL difference, its 95 % interval and whether
the interval excludes 0; a finding counts as reproduced on a seed when its interval excludes 0 in the reference's
direction (reference: ``Notebooks/qwen2-0.5B_experiment.ipynb``)."""
import json
import os
import sys


def load(d):
    tr = None
    with open(os.path.join(d, "train.log")) as f:
        for line in f:
            if line.startswith("{"):
                tr = json.loads(line)
    sw = json.load(open(os.path.join(d, "quality_sweep.json")))
    pq = json.load(open(os.path.join(d, "pipeline_quality.json")))
    return tr, sw, pq


def ci(x):
    return f"{x['diff']:+.1e} [{x['ci'][0]:+.1e}, {x['ci'][1]:+.1e}]"


def main():
    dirs = sys.argv[1:]
    runs = [(os.path.basename(d.rstrip("/")), *load(d)) for d in dirs]
    out = ["# Quality surrogate over seeds", ""]
    out += ["## Training (held-out-driven stop)", "",
            "| seed | best step / steps | held-out nats/byte | stdlib-train sample | gap | seen vs fresh (memorisation) "
            "| epochs |", "|---|---|---|---|---|---|---|"]
    for name, tr, _, _ in runs:
        if tr is None:
            continue
        mem = tr.get("memorisation_gap")
        out.append(f"| {tr['seed']} | {tr['best_step']} / {tr['steps']} | {tr['held_out_nats_per_byte']:.4f} | "
                   f"{tr['train_sample_nats_per_byte']:.4f} | {100 * tr['gap']:+.1f} % | "
                   f"{'n/a' if mem is None else f'{100 * mem:+.1f} %'} | {tr.get('epochs', 'n/a')} |")

    # findings
    def table(key, label, cols, reproduced):
        rows = {}
        for name, _, sw, _ in runs:
            for x in sw["findings"][key]:
                k = tuple(x.get(c) for c in cols)
                rows.setdefault(k, {})[name] = x
        lines = [f"### {label}", "", "| " + " | ".join(cols) + " | " + " | ".join(n for n, *_ in runs) +
                 " | reproduced on |", "|" + "---|" * (len(cols) + len(runs) + 1)]
        for k, per in rows.items():
            cells = [ci(per[n]) + f" {per[n]['verdict']}" if n in per else "-" for n, *_ in runs]
            rep = sum(1 for n, *_ in runs if n in per and reproduced(per[n]))
            lines.append("| " + " | ".join(str(v) for v in k) + " | " + " | ".join(cells) +
                         f" | {rep} of {len(runs)} |")
        return lines + [""]

    out += ["", "## The reference's three findings, per seed (paired window-bootstrap 95 % intervals of log-PPL "
            "differences)", ""]
    out += table("late_boundaries_hurt_more", "Late boundaries hurt more: log PPL(L23) - log PPL(other), last_row, Q1",
                 ["other", "ratio"], lambda x: x["verdict"] == "a worse")
    out += table("last_row_beats_column_mean", "last_row beats the column mean: log PPL(column-mean) - log PPL(last_row),"
                 " Q1", ["layer", "ratio"], lambda x: x["verdict"] == "a worse")
    out += table("one_scale_collapse_at_ratio_1", "One-scale collapse at ratio 1: log PPL(r=1) - log PPL(r=0), last_row,"
                 " Q1 (reference, BASELINE.md: 13.3 -> 382 at L22, 8.7e6 at L3)", ["layer"], lambda x: x["verdict"] == "a worse" and x["rel"] > 1.0)

    # mechanism: the one-scale damage against the boundary's outlier statistics, every (seed, layer)
    pts = []
    for name, _, sw, _ in runs:
        dmg = {x["layer"]: x["rel"] for x in sw["findings"]["one_scale_collapse_at_ratio_1"]}
        for L, b in sorted(sw.get("boundary_outliers", {}).items(), key=lambda kv: int(kv[0])):
            if int(L) in dmg:
                pts.append((name, int(L), b["peak_over_rms"], b["int4_global_zero_fraction"], dmg[int(L)]))
    if len(pts) >= 3:
        from scipy.stats import spearmanr
        out += ["### What the one-scale damage follows", "",
                "| seed | layer | boundary peak / RMS | values one global int4 scale rounds to 0 | ratio-1 damage |",
                "|---|---|---|---|---|"]
        out += [f"| {n} | {L} | {pk:.1f} | {z:.3f} | {100 * d:+.2f} % |" for n, L, pk, z, d in pts]
        rz = spearmanr([p[3] for p in pts], [p[4] for p in pts])
        rp = spearmanr([p[2] for p in pts], [p[4] for p in pts])
        rl = spearmanr([p[1] for p in pts], [p[4] for p in pts])
        out += ["", f"Spearman over the {len(pts)} (seed, layer) points: zeroed fraction vs damage "
                f"{rz.statistic:.2f} (p = {rz.pvalue:.1e}); peak / RMS vs damage {rp.statistic:.2f} "
                f"(p = {rp.pvalue:.1e}); depth vs damage {rl.statistic:.2f} (p = {rl.pvalue:.1e}).", ""]

    # config 5: allocated head-group plans against the uniform plan
    out += ["## Head-group plans against the uniform plan (pipeline, 7 boundaries)", "",
            "Ratios at which the allocated plan is better (interval below 0) / worse (interval above 0), of the 4 "
            "nonzero ratios:", "",
            "| method | codec | plan | " + " | ".join(n for n, *_ in runs) + " |", "|---|---|---|" + "---|" * len(runs)]
    comps = {}
    for name, _, _, pq in runs:
        for c in pq["plan_vs_uniform"]:
            comps.setdefault((c["method"], c["codec"], c["plan"]), {})[name] = c
    for (meth, codec, plan), per in comps.items():
        cells = []
        for n, *_ in runs:
            c = per.get(n)
            if c is None:
                cells.append("-")
                continue
            nz = [x for x in c["cells"] if x["ratio"] > 0]
            b = sum(1 for x in nz if x["ci"][1] < 0)
            w = sum(1 for x in nz if x["ci"][0] > 0)
            same = all(x["diff"] == 0 and x["ci"] == [0, 0] for x in nz)
            cells.append("identical plan" if same else f"better {b} / worse {w}")
        out.append(f"| {meth} | {codec} | {plan} | " + " | ".join(cells) + " |")
    print("\n".join(out))


if __name__ == "__main__":
    main()
