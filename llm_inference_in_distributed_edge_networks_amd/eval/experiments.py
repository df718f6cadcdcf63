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

from .. import codec as C
from ..config import Params, dump_json, resolve_device, resolve_dtype, resolve_window_batch
from ..importance import canonical, load_head_weights
from ..models import build_model, get_config
from ..parallel.dist import all_reduce_sum, broadcast_object, get_env, init_distributed
from ..utils.checkpoint import SweepState
from ..utils.logging import log, progress_bar
from .data import token_stream
from .sweep import SweepConfig, SweepEngine, SweepMethod, run_sweep
from .windows import batches, sliding_windows

CHANNEL_METHODS = ("channel_8", "channel_4", "channel_1_mean", "channel_1_max")


def _setup(p: Params, default_model: str):
    env = init_distributed(p.device)
    device = str(env.device) if env.device.type == "cuda" else resolve_device(p)
    dtype = resolve_dtype(p, device)
    resolve_window_batch(p, device)
    cfg = get_config(p.model or default_model)
    model, prov = build_model(cfg, device, dtype, weights=p.weights, seed=p.seed)
    ids, data_prov = token_stream(p.dataset, cfg.hf_id, cfg.vocab_size, p.synthetic_tokens, p.seed,
                                  strict=p.strict_data)
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
    engine._flush()
    if not env.is_dist:
        return
    dev = env.device if env.backend == "nccl" else torch.device("cpu")
    t = torch.cat([engine.total_nll.reshape(-1), engine.wire_bytes.reshape(-1), engine.sum_window_nll.reshape(-1),
                   torch.tensor([engine.n_tokens, engine.windows_done, engine.tokens_done, engine.forward_tokens],
                                dtype=torch.float64)]).to(dev)
    all_reduce_sum(t)
    t = t.cpu()
    n = engine.total_nll.numel()
    engine.total_nll = t[:n].reshape(engine.total_nll.shape)
    engine.wire_bytes = t[n:2 * n].reshape(engine.wire_bytes.shape)
    engine.sum_window_nll = t[2 * n:3 * n].reshape(engine.sum_window_nll.shape)
    engine.n_tokens, engine.windows_done, engine.tokens_done, engine.forward_tokens = \
        float(t[3 * n]), int(t[3 * n + 1]), int(t[3 * n + 2]), int(t[3 * n + 3])


def importance_sweep(p: Params, default_model: str, out_name: str) -> dict:
    env, cfg, model, ids, wins, meta = _setup(p, default_model)
    methods = [canonical(m) for m in p.methods]
    hw = None
    if "weighted_importance" in methods:
        path = p.head_weights or _default_head_weights()
        hw = load_head_weights(path) if path and os.path.exists(path) else None
        if hw is None:
            raise FileNotFoundError("weighted_importance needs attention_head_weights.json / .pkl "
                                    "(run Experiments/Relevance/main.py or set params['head_weights'])")
    rows = [SweepMethod(m, m, selection=p.selection) for m in methods]
    sc = SweepConfig(rows, p.layers_of_interest, p.ratios, p.codec, hw, group_relevance=_group_relevance(p),
                     group_avg_bits=p.group_avg_bits)
    eng = SweepEngine(model, sc)
    state = _state(p, env, out_name)
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


def _state(p: Params, env, name: str) -> SweepState:
    return SweepState(os.path.join(p.output_dir, f"{name}.rank{env.rank}.ckpt.json"), p.config_hash(),
                      enabled=p.resume, shard=(env.rank, env.world_size, f"batch-mod/{p.window_batch}"))


def channel_sweep(p: Params, default_model: str) -> dict:
    """Reference ``channel_wise.py``: per-channel quantization of the whole boundary tensor.

    One unquantized prefix forward per window batch; the 4 channel codecs (and every boundary layer) fork
    from it in one stacked suffix forward (the reference re-runs the whole model per (method, layer))."""
    env, cfg, model, ids, wins, meta = _setup(p, default_model)
    for meth in p.methods:
        if meth not in CHANNEL_METHODS:
            raise ValueError(f"channel sweep got non-channel method {meth!r}")
    rows = [SweepMethod(m, None, codec=m) for m in p.methods]
    eng = SweepEngine(model, SweepConfig(rows, p.layers_of_interest, [1], p.methods[0]))
    pb = progress_bar(len(wins), env.is_main)
    res = run_sweep(eng, _shard(batches(ids, wins, p.window_batch), env), _state(p, env, "channel"),
                    p.checkpoint_every, progress=pb.update, reduce_fn=_reduce)
    pb.close()
    ppl = eng.ppl()
    out = {"layers_of_interest": p.layers_of_interest, "methods": list(p.methods)}
    out["avg_ppl_results"] = [[float(ppl[mi, li, 0]) for mi in range(len(p.methods))]
                              for li in range(len(p.layers_of_interest))]          # [layer][method] (reference)
    out["wire_bytes_per_token"] = [[float(eng.wire_bytes[mi, li, 0]) / max(1, eng.tokens_done)
                                    for mi in range(len(p.methods))] for li in range(len(p.layers_of_interest))]
    out["seconds"] = res["seconds"]
    out["windows"] = res["windows"]
    out["windows_per_s"] = res["windows"] / max(res["seconds"], 1e-9)
    out.update(meta)
    if env.is_main:
        os.makedirs(p.output_dir, exist_ok=True)
        dump_json(out, os.path.join(p.output_dir, "avg_ppl_results_channel.json"))
        for li, L in enumerate(p.layers_of_interest):
            log(f"layer {L}: " + "  ".join(f"{m}={v:.4f}" for m, v in zip(p.methods, out["avg_ppl_results"][li])))
    return out


INITIAL_QUANT_LAYER = 2   # initial_exp.py:118/:122


def initial_rows(layers_of_interest) -> list:
    """Pythia ``initial`` orderings (``initial_exp.py:27-72``) as sweep rows at the fixed boundary layer 2."""
    rows = []
    for l in layers_of_interest:
        if l == "aggregate upto 2":
            rows.append(SweepMethod(str(l), "aggregate_till"))
        elif l == "maximum aggregation":
            rows.append(SweepMethod(str(l), "maximum_aggregation"))
        elif l == "upto ratio":
            rows.append(SweepMethod(str(l), "regular_importance", selection="top_rho"))
        else:
            rows.append(SweepMethod(str(l), "regular_importance", source_layer=int(l)))
    return rows


def initial_experiment(p: Params) -> dict:
    """Pythia ``initial_exp.py``: quantize at layer 2 with orderings from special 'layers'.

    ``layers_of_interest`` entries: int l (order by layer-l column mean), 'aggregate upto 2',
    'maximum aggregation', 'upto ratio' (top-rho on the layer-2 distribution, k per window).  Ratios are
    ints 0..10 meaning 0.1*ratio of the tokens (Q4, ``pythia_model.py:142``; top-rho mass 1 - 0.1*ratio).
    Quantizer: per-token int8 on the selected tokens (intended semantics of Q2, B9-B11 fixed).  Like the
    reference (``initial_exp.py:113-122``: one batch row per ratio) every (ordering, ratio) variant of a window
    batch runs in ONE stacked suffix forward after a single shared prefix; no host sync per window.  Output
    ``exp_1.json`` = ``{layer: {ratio: mean_nll}}`` (unweighted mean over windows, ``initial_exp.py:130-134``).
    """
    env, cfg, model, ids, wins, meta = _setup(p, "pythia-70m")
    sc = SweepConfig(initial_rows(p.layers_of_interest), [INITIAL_QUANT_LAYER], p.ratios, codec="int8_token_keep",
                     ratio_scale=0.1)
    eng = SweepEngine(model, sc)
    pb = progress_bar(len(wins), env.is_main)
    res = run_sweep(eng, _shard(batches(ids, wins, p.window_batch), env), _state(p, env, "exp_1"),
                    p.checkpoint_every, progress=pb.update, reduce_fn=_reduce)
    pb.close()
    mw = res["mean_window_nll"]
    exp1 = {name: {str(r): mw[mi][0][ri] for ri, r in enumerate(p.ratios)} for mi, name in enumerate(eng.methods)}
    out = {"exp_1": exp1, "ppl": {l: {r: math.exp(v) for r, v in d.items()} for l, d in exp1.items()},
           "wire_bytes_per_token": {name: {str(r): res["wire_bytes_per_token"][mi][0][ri]
                                           for ri, r in enumerate(p.ratios)} for mi, name in enumerate(eng.methods)},
           "windows": res["windows"], "seconds": res["seconds"],
           "windows_per_s": res["windows"] / max(res["seconds"], 1e-9), **meta}
    if env.is_main:
        os.makedirs(p.output_dir, exist_ok=True)
        dump_json(out, os.path.join(p.output_dir, "exp_1.json"))
    return out


def _group_relevance(p: Params):
    """Channel-group relevance table [layers][H / 64] for the head-group codecs (None: uniform plans), loaded the
    same way by the sweep and the pipeline drivers so both quantize a boundary identically."""
    if not C.wire.needs_plan(C.get_codec(p.codec)):
        return None
    path = p.group_relevance or _default_group_relevance()
    if p.group_relevance and not os.path.exists(path):
        raise FileNotFoundError(f"group_relevance {path} not found (run Experiments/Relevance/main.py)")
    if path and os.path.exists(path):
        return C.wire.load_group_tables(path)   # + channel_group_sensitivity.json when the pass wrote it
    log("head-group codec without channel_group_relevance.json: every group gets the same width")
    return None


def _default_group_relevance() -> str | None:
    for c in ("channel_group_relevance.json", "../Relevance/channel_group_relevance.json",
              os.path.join(os.path.dirname(__file__), "..", "..", "Experiments", "Relevance",
                           "channel_group_relevance.json")):
        if os.path.exists(c):
            return c
    return None


def _default_head_weights() -> str | None:
    """The LRP head-weight table: ours (JSON, Experiments/Relevance) or the reference's pickle at the place its
    Qwen2 sweep reads it (``../../attention_head_weights.pkl``, Experiments/Qwen2-0.5B/main.py:129-130)."""
    for c in ("attention_head_weights.json", "attention_head_weights.pkl", "../Relevance/attention_head_weights.json",
              "../Relevance/attention_head_weights.pkl", "../../attention_head_weights.json",
              "../../attention_head_weights.pkl"):
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
    resolve_window_batch(p, device)
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
    ids, data_prov = token_stream(p.dataset, cfg.hf_id, cfg.vocab_size, p.synthetic_tokens, p.seed,
                                  strict=p.strict_data)
    wins = sliding_windows(ids.shape[1], max_len, p.stride)
    if p.max_windows:
        wins = wins[: p.max_windows]
    methods = [canonical(m) for m in p.methods]
    hw = None
    if "weighted_importance" in methods:
        path = p.head_weights or _default_head_weights()
        if not (path and os.path.exists(path)):
            raise FileNotFoundError("weighted_importance needs attention_head_weights.json / .pkl "
                                    "(run Experiments/Relevance/main.py or set params['head_weights'])")
        hw = load_head_weights(path)
    grel = _group_relevance(p)
    log(f"pipeline: model={cfg.name} weights={prov} data={data_prov} stages={plan.num_stages} "
        f"boundaries={plan.boundary_layers()} world={env.world_size} codec={p.codec} windows={len(wins)}")
    results: dict = {}
    state = SweepState(os.path.join(p.output_dir, f"pipeline_results.rank{env.rank}.ckpt.json"), p.config_hash(),
                       enabled=p.resume, shard=(env.rank, env.world_size, f"pipeline/{p.window_batch}"))
    saved = state.load() or {}
    if distributed:
        # pipeline stages exchange boundary messages batch by batch, so every rank must resume at the same point:
        # rank 0's checkpoint is the one (its sums are the all-reduced totals, like every rank's); a rank whose own
        # file is one chunk ahead or behind (a job killed between two ranks' saves) follows it
        saved = broadcast_object(saved, src=0)
    results.update(saved.get("results", {}))
    bl = list(batches(ids, wins, p.window_batch))
    toks = sum(w.end - w.begin for w in wins)
    runner = None
    # windows per resumable chunk (the reference dumps its running sums every 1000 windows, main.py:184-192)
    chunk = max(1, p.checkpoint_every // max(1, p.window_batch))
    for m in methods:
        for r in p.ratios:
            if str(r) in results.get(m, {}):
                log(f"{m} ratio={r}: resumed from checkpoint")
                continue
            bcfg = BoundaryConfig(p.codec, float(r), m, hw, selection=p.selection, group_relevance=grel,
                                  group_avg_bits=p.group_avg_bits)
            # one runtime for the whole sweep: the transport (RCCL channels / IPC slot rings) is set up once, only
            # the boundary codec changes between (method, ratio)
            if runner is None:
                runner = (DistributedPipeline(model, plan, bcfg, grid, env.rank) if distributed
                          else LocalPipeline(model, plan, bcfg))
            else:
                runner.set_boundary(bcfg)
            part = saved.get("partial") if saved.get("partial", {}).get("key") == [m, str(r)] else None
            if part is not None and not {"total_nll", "n_tokens", "seconds", "wire_bytes", "wire_tokens",
                                         "next_batch"} <= set(part):
                # a checkpoint of an older format (e.g. round 3's wire_sum / wire_n): redo this (method, ratio)
                log(f"{m} ratio={r}: partial checkpoint of an older format, restarting it from batch 0")
                part = None
            tot, ntok, sec = (part["total_nll"], part["n_tokens"], part["seconds"]) if part else (0.0, 0.0, 0.0)
            # wire bytes and the tokens they carried, summed over the boundaries (and replicas) and over the chunks,
            # so a resumed run reports the uninterrupted run's bytes per token (variable-k codecs included)
            wbytes, wtoks = (part["wire_bytes"], part["wire_tokens"]) if part else (0.0, 0.0)
            prev_b = prev_t = 0.0            # the runner's counters restart at set_boundary / construction
            start = part["next_batch"] if part else 0
            for c0 in range(start, len(bl), chunk):
                t0 = time.perf_counter()
                piece = bl[c0:c0 + chunk]
                if distributed:
                    acc, info = runner.evaluate(piece)
                    wire = torch.tensor([info["wire_bytes"], info["wire_tokens"]], dtype=torch.float64,
                                        device=env.device if env.backend == "nccl" else "cpu")
                    all_reduce_sum(wire)
                    cb, ct = float(wire[0]), float(wire[1])
                else:
                    acc = runner.evaluate(piece)
                    cb, ct = runner.wire_totals()
                if device.startswith("cuda"):
                    torch.cuda.synchronize()
                sec += time.perf_counter() - t0
                tot += acc.total_nll
                ntok += acc.n_tokens
                wbytes += cb - prev_b
                wtoks += ct - prev_t
                prev_b, prev_t = cb, ct
                if c0 + chunk < len(bl):
                    state.save({"results": results, "partial": {
                        "key": [m, str(r)], "next_batch": c0 + chunk, "total_nll": tot, "n_tokens": ntok,
                        "seconds": sec, "wire_bytes": wbytes, "wire_tokens": wtoks}})
            ppl = math.exp(tot / ntok) if ntok else float("nan")
            wire_pt = wbytes / wtoks if wtoks else 0.0
            results.setdefault(m, {})[str(r)] = {"ppl": ppl, "total_nll": tot, "n_tokens": ntok,
                                                 "wire_bytes_per_token": wire_pt,
                                                 "tokens_per_s": toks / max(sec, 1e-9), "seconds": sec}
            state.save({"results": results})
            if env.is_main:
                log(f"{m:20s} ratio={r:<5} ppl={ppl:.4f} wire={wire_pt:.1f} B/token "
                    f"({toks / max(sec, 1e-9):,.0f} tok/s)")
    if runner is not None and distributed:
        runner.close()
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
