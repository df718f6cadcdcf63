"""Experiment drivers behind ``Experiments/{Pythia-70M,Qwen2-0.5B,Relevance}/main.py``.

Reference dispatch:

* Pythia ``main.py:23-32``: ``params["experiment"]`` in {"last_row", "initial"} else ``ValueError``;
* Qwen2 ``main.py:108-119``: channel sweep if the first method names a channel quantizer, otherwise
  the 4-method importance sweep (the reference's ``str.contains`` / module-call bugs B2/B3 fixed);
* Relevance ``main.py``: LRP head-relevance calibration (its params-path bug B13 fixed);
* ``experiment: "pipeline"`` / ``num_stages`` > 1 / ``split_layers`` (new): the real N-stage split
  with a quantized boundary message per stage hand-off (``pipeline_experiment``).

All drivers run single-process or data-parallel under ``torchrun`` (windows sharded by batch,
sums all-reduced), write JSON results in the reference's nested-list layouts, checkpoint every
``checkpoint_every`` windows and resume from the checkpoint of an identical configuration.
"""
from __future__ import annotations

import json
import math
import os
import time

import torch

from ..config import Params, dump_json, resolve_device, resolve_dtype
from ..importance import canonical, load_head_weights
from ..models import build_model, get_config
from ..parallel.dist import all_reduce_sum, get_env, init_distributed
from ..utils.checkpoint import SweepState
from ..utils.logging import log, progress_bar
from .data import token_stream
from .sweep import SweepConfig, SweepEngine, run_sweep
from .windows import batches, sliding_windows

CHANNEL_METHODS = ("channel_8", "channel_4", "channel_1_mean", "channel_1_max")


def _setup(p: Params, default_model: str):
    env = init_distributed(p.device)
    device = str(env.device) if env.device.type == "cuda" else resolve_device(p)
    dtype = resolve_dtype(p, device)
    cfg = get_config(p.model or default_model)
    model, prov = build_model(cfg, device, dtype, weights=p.weights, seed=p.seed)
    ids, data_prov = token_stream(p.dataset, cfg.hf_id, cfg.vocab_size, p.synthetic_tokens, p.seed)
    max_len = p.max_length or cfg.max_position
    wins = sliding_windows(ids.shape[1], max_len, p.stride)
    if p.max_windows:
        wins = wins[: p.max_windows]
    log(f"model={cfg.name} weights={prov} data={data_prov} tokens={ids.shape[1]} windows={len(wins)} "
        f"max_length={max_len} stride={p.stride} device={device} dtype={dtype} world={env.world_size}")
    return env, cfg, model, ids, wins, {"weights": prov, "data": data_prov, "device": device,
                                        "dtype": str(dtype), "max_length": max_len}


def _shard(batch_iter, env):
    for i, b in enumerate(batch_iter):
        if i % env.world_size == env.rank:
            yield b


def _reduce(engine: SweepEngine):
    env = get_env()
    if not env.is_dist:
        return
    dev = env.device if env.backend == "nccl" else torch.device("cpu")
    t = torch.cat([engine.total_nll.reshape(-1), engine.wire_bytes.reshape(-1),
                   torch.tensor([engine.n_tokens, engine.windows_done, engine.tokens_done, engine.forward_tokens],
                                dtype=torch.float64)]).to(dev)
    all_reduce_sum(t)
    t = t.cpu()
    n = engine.total_nll.numel()
    engine.total_nll = t[:n].reshape(engine.total_nll.shape)
    engine.wire_bytes = t[n:2 * n].reshape(engine.wire_bytes.shape)
    engine.n_tokens, engine.windows_done, engine.tokens_done, engine.forward_tokens = \
        float(t[2 * n]), int(t[2 * n + 1]), int(t[2 * n + 2]), int(t[2 * n + 3])


def importance_sweep(p: Params, default_model: str, out_name: str) -> dict:
    env, cfg, model, ids, wins, meta = _setup(p, default_model)
    methods = [canonical(m) for m in p.methods]
    hw = None
    if "weighted_importance" in methods:
        path = p.head_weights or _default_head_weights()
        hw = load_head_weights(path) if path and os.path.exists(path) else None
        if hw is None:
            raise FileNotFoundError("weighted_importance needs attention_head_weights.json "
                                    "(run Experiments/Relevance/main.py or set params['head_weights'])")
    sc = SweepConfig(methods, p.layers_of_interest, p.ratios, p.codec, hw)
    eng = SweepEngine(model, sc)
    state = SweepState(os.path.join(p.output_dir, f"{out_name}.rank{env.rank}.ckpt.json"), p.config_hash(),
                       enabled=p.resume)
    pb = progress_bar(len(wins), env.is_main)
    res = run_sweep(eng, _shard(batches(ids, wins, p.window_batch), env), state, p.checkpoint_every,
                    progress=pb.update, reduce_fn=_reduce)
    pb.close()
    res.update(meta)
    res["params"] = p.to_dict()
    res["throughput_forward_tokens_per_s"] = res["forward_tokens"] / max(res["seconds"], 1e-9)
    if env.is_main:
        os.makedirs(p.output_dir, exist_ok=True)
        dump_json(res, os.path.join(p.output_dir, f"{out_name}.json"))
        _print_table(res)
    return res


def channel_sweep(p: Params, default_model: str) -> dict:
    """Reference ``channel_wise.py``: per-channel quantization of the whole boundary tensor."""
    env, cfg, model, ids, wins, meta = _setup(p, default_model)
    out = {"layers_of_interest": p.layers_of_interest, "methods": list(p.methods), "avg_ppl_results": []}
    engines = {}
    for meth in p.methods:
        if meth not in CHANNEL_METHODS:
            raise ValueError(f"channel sweep got non-channel method {meth!r}")
        engines[meth] = SweepEngine(model, SweepConfig(["regular_importance"], p.layers_of_interest, [1], meth))
    t0 = time.perf_counter()
    for b in _shard(batches(ids, wins, p.window_batch), env):
        b = b.to(model.device)
        for e in engines.values():
            e.run_batch(b)
    for e in engines.values():
        _reduce(e)
    res_l = []
    for li, L in enumerate(p.layers_of_interest):
        res_l.append([float(engines[m].ppl()[0, li, 0]) for m in p.methods])
    out["avg_ppl_results"] = res_l           # [layer][method] (reference layout)
    out["wire_bytes_per_token"] = [[float(engines[m].wire_bytes[0, li, 0]) / max(1, engines[m].tokens_done)
                                    for m in p.methods] for li in range(len(p.layers_of_interest))]
    out["seconds"] = time.perf_counter() - t0
    out.update(meta)
    if env.is_main:
        os.makedirs(p.output_dir, exist_ok=True)
        dump_json(out, os.path.join(p.output_dir, "avg_ppl_results_channel.json"))
        for li, L in enumerate(p.layers_of_interest):
            log(f"layer {L}: " + "  ".join(f"{m}={v:.4f}" for m, v in zip(p.methods, res_l[li])))
    return out


def initial_experiment(p: Params) -> dict:
    """Pythia ``initial_exp.py``: quantize at layer 2 with orderings from special 'layers'.

    ``layers_of_interest`` entries: int l (order by layer-l column mean), 'aggregate upto 2',
    'maximum aggregation', 'upto ratio' (top-rho on the layer-2 distribution).  Ratios are ints
    0..10 meaning 0.1*ratio of the tokens (Q4, ``pythia_model.py:142``).  Quantizer: per-token int8
    on the selected tokens (intended semantics of Q2, B9-B11 fixed).  Output ``exp_1.json`` =
    ``{layer: {ratio: mean_nll}}`` (unweighted mean over windows, ``initial_exp.py:130-134``).
    """
    from .. import codec as C
    from ..importance import ImportanceTracker
    from .windows import window_nll
    env, cfg, model, ids, wins, meta = _setup(p, "pythia-70m")
    QL = 2
    spec = C.get_codec("int8_token_keep")
    sums: dict = {}
    counts = 0
    for b in _shard(batches(ids, wins, p.window_batch), env):
        b = b.to(model.device)
        B, S = b.B, b.S
        tr = ImportanceTracker("aggregate_till", [0, 1, 2], cfg.num_heads)
        trm = ImportanceTracker("maximum_aggregation", [2], cfg.num_heads)
        x = model.embed(b.ids)
        regs = {}
        h2 = None
        for i in range(cfg.num_layers):
            need = "colsum" if i <= max(2, max([l for l in p.layers_of_interest if isinstance(l, int)] or [0])) \
                else None
            x, st = model.layer(i, x, B, S, stats=need)
            if need:
                tr.observe(i, st, S) if i <= 2 else None
                trm.observe(i, st, S) if i <= 2 else None
                from .. import ops
                regs[i] = ops.head_combine(st.colsum, None, 1.0 / (cfg.num_heads * S))
            if i == QL:
                h2 = x
        for l in p.layers_of_interest:
            if l == "aggregate upto 2":
                imp = tr.importance(2)
            elif l == "maximum aggregation":
                imp = trm.importance(2)
            elif l == "upto ratio":
                imp = regs[2]
            else:
                imp = regs[int(l)]
            for r in p.ratios:
                if l == "upto ratio":
                    # top-rho: keep the smallest prefix (by descending importance) reaching 1 - 0.1*r mass
                    srt = torch.sort(imp.float(), dim=1, descending=True).values
                    cum = srt.cumsum(1)
                    keep = (cum < (1 - 0.1 * float(r))).sum(1) + 1
                    ks = (S - keep.clamp(max=S)).tolist()
                else:
                    ks = [int(0.1 * float(r) * S)] * B
                wn = []
                for bi in range(B):
                    xb = h2.view(B, S, -1)[bi].contiguous()
                    xq, _ = C.fake_quant(xb, spec, 1, S, importance=imp[bi:bi + 1], k=ks[bi])
                    xs = xq
                    for i in range(QL + 1, cfg.num_layers):
                        xs, _ = model.layer(i, xs, 1, S)
                    sel = b.row_window == bi
                    rows = b.rows[sel] - bi * S
                    nll = model.row_nll(xs, rows, b.targets[sel])
                    wn.append(float(nll.mean()))
                key = (str(l), r)
                sums[key] = sums.get(key, 0.0) + sum(wn)
        counts += B
    if env.is_dist:
        keys = sorted(sums, key=str)
        t = torch.tensor([sums[k] for k in keys] + [counts], dtype=torch.float64)
        all_reduce_sum(t)
        sums = dict(zip(keys, t[:-1].tolist()))
        counts = int(t[-1])
    res = {}
    for (l, r), s in sums.items():
        res.setdefault(l, {})[str(r)] = s / counts
    out = {"exp_1": res, "ppl": {l: {r: math.exp(v) for r, v in d.items()} for l, d in res.items()}, **meta}
    if env.is_main:
        os.makedirs(p.output_dir, exist_ok=True)
        dump_json(out, os.path.join(p.output_dir, "exp_1.json"))
    return out


def _default_head_weights() -> str | None:
    for c in ("attention_head_weights.json", "../Relevance/attention_head_weights.json",
              "../../attention_head_weights.json"):
        if os.path.exists(c):
            return c
    return None


def _print_table(res: dict) -> None:
    ratios = res["ratios"]
    log("method               layer | " + " ".join(f"{r:>10}" for r in ratios))
    for mi, m in enumerate(res["methods"]):
        for li, L in enumerate(res["layers_of_interest"]):
            log(f"{m:20s} {L:5d} | " + " ".join(f"{v:10.4f}" for v in res["avg_ppl_results"][mi][li]))


def pipeline_experiment(p: Params, default_model: str) -> dict:
    """Real N-stage split inference (BASELINE.json configs 1-5), one result per (method, ratio).

    The reference only simulates the device boundary (``qwen_layer_wise.py:54-70``).  Here
    ``num_stages`` > 1 (or ``split_layers``) partitions the layers; under ``torchrun`` with
    ``world = num_stages * dp`` every rank runs one stage and the boundary message goes over
    RCCL (gloo on CPU); a single process runs all stages locally with the same codec.  Every
    boundary uses ``codec`` with importance ``method`` scored at that boundary layer.  Output
    ``pipeline_results.json``: ``{method: {ratio: {ppl, wire_bytes_per_token, tokens_per_s}}}``.
    """
    from ..parallel import BoundaryConfig, DistributedPipeline, Grid, LocalPipeline, PipelinePlan
    env = init_distributed(p.device)
    device = str(env.device) if env.device.type == "cuda" else resolve_device(p)
    dtype = resolve_dtype(p, device)
    cfg = get_config(p.model or default_model)
    max_len = p.max_length or cfg.max_position
    pp = len(p.split_layers) + 1 if p.split_layers else p.num_stages
    plan = PipelinePlan.from_split_layers(cfg.num_layers, p.split_layers) if p.split_layers \
        else PipelinePlan.balanced(cfg, pp, max_len)
    distributed = env.world_size > 1
    if distributed:
        if env.world_size % pp:
            raise ValueError(f"world size {env.world_size} is not a multiple of num_stages {pp}")
        grid = Grid(env.world_size, pp)
        dp_idx, stage = grid.coords(env.rank)
        model, prov = build_model(cfg, device, dtype, weights=p.weights, seed=p.seed,
                                  layers=plan.stage_layers(stage), with_embed=stage == 0, with_head=stage == pp - 1)
    else:
        model, prov = build_model(cfg, device, dtype, weights=p.weights, seed=p.seed)
    ids, data_prov = token_stream(p.dataset, cfg.hf_id, cfg.vocab_size, p.synthetic_tokens, p.seed)
    wins = sliding_windows(ids.shape[1], max_len, p.stride)
    if p.max_windows:
        wins = wins[: p.max_windows]
    methods = [canonical(m) for m in p.methods]
    hw = None
    if "weighted_importance" in methods:
        path = p.head_weights or _default_head_weights()
        if not (path and os.path.exists(path)):
            raise FileNotFoundError("weighted_importance needs attention_head_weights.json "
                                    "(run Experiments/Relevance/main.py or set params['head_weights'])")
        hw = load_head_weights(path)
    log(f"pipeline: model={cfg.name} weights={prov} data={data_prov} stages={plan.num_stages} "
        f"boundaries={plan.boundary_layers()} world={env.world_size} codec={p.codec} windows={len(wins)}")
    results: dict = {}
    for m in methods:
        for r in p.ratios:
            bcfg = BoundaryConfig(p.codec, float(r), m, hw)
            bl = list(batches(ids, wins, p.window_batch))
            t0 = time.perf_counter()
            if distributed:
                runner = DistributedPipeline(model, plan, bcfg, grid, env.rank)
                acc, info = runner.evaluate(bl)
                wire = torch.tensor([info["wire_bytes_per_token"] if stage < pp - 1 else 0.0], dtype=torch.float64,
                                    device=env.device if env.backend == "nccl" else "cpu")
                all_reduce_sum(wire)
                wire_pt = float(wire) / (grid.dp * max(1, pp - 1))
            else:
                runner = LocalPipeline(model, plan, bcfg)
                acc = runner.evaluate(bl)
                wb = runner.wire_bytes_per_token()
                wire_pt = sum(wb) / len(wb) if wb else 0.0
            if device.startswith("cuda"):
                torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            toks = sum(w.end - w.begin for w in wins)
            results.setdefault(m, {})[str(r)] = {"ppl": acc.ppl(), "total_nll": acc.total_nll,
                                                 "n_tokens": acc.n_tokens, "wire_bytes_per_token": wire_pt,
                                                 "tokens_per_s": toks / max(dt, 1e-9), "seconds": dt}
            if env.is_main:
                log(f"{m:20s} ratio={r:<5} ppl={acc.ppl():.4f} wire={wire_pt:.1f} B/token "
                    f"({toks / max(dt, 1e-9):,.0f} tok/s)")
    out = {"results": results, "stages": plan.num_stages, "boundaries": plan.boundary_layers(),
           "stage_layers": [list(plan.stage_layers(s)) for s in range(plan.num_stages)], "codec": p.codec,
           "world_size": env.world_size, "weights": prov, "data": data_prov, "device": device, "dtype": str(dtype),
           "max_length": max_len, "params": p.to_dict()}
    if env.is_main:
        os.makedirs(p.output_dir, exist_ok=True)
        dump_json(out, os.path.join(p.output_dir, "pipeline_results.json"))
    return out


# ------------------------------------------------------------------------------------------
def wants_pipeline(p: Params) -> bool:
    return p.experiment == "pipeline" or p.num_stages > 1 or bool(p.split_layers)


def pythia_main(p: Params) -> dict:
    if wants_pipeline(p):
        return pipeline_experiment(p, "pythia-70m")
    if p.experiment == "last_row":
        return importance_sweep(p, "pythia-70m", "avg_ppl_results_pythia_70m")
    if p.experiment == "initial":
        return initial_experiment(p)
    raise ValueError(f"Unknown experiment: {p.experiment}")


def qwen2_main(p: Params) -> dict:
    if wants_pipeline(p):
        return pipeline_experiment(p, "qwen2-0.5b")
    if p.methods and "channel" in str(p.methods[0]):
        return channel_sweep(p, "qwen2-0.5b")
    return importance_sweep(p, "qwen2-0.5b", "avg_ppl_results")
