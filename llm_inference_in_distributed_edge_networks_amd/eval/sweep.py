"""Importance x boundary-layer x ratio perplexity sweeps (the reference experiments).

Reference drivers: ``Experiments/Qwen2-0.5B/main.py:100-207`` (4 methods x layers x ratios),
``Experiments/Pythia-70M/last_row_exp.py:47-143`` and ``Experiments/Qwen2-0.5B/channel_wise.py:10-78``.
Per window the reference runs one eager forward for attention maps and then one full split
forward per (method, layer, ratio) - 101 forwards of 512 tokens per Qwen2 window.

Here, per window batch:

1. ONE unquantized forward: it yields the ratio-0 NLL, the hidden state after every boundary layer
   of interest (kept on device) and every method's importance at the layers it is needed (fused
   attention statistics, no S x S maps);
2. per boundary layer L, the (method, ratio) variants are de-duplicated (ratio 0 and "all tokens
   quantized" do not depend on the method), their fake-quantized copies of h_L are stacked along the
   batch dimension and ONLY layers L+1.. are run, once, on the stacked batch (shared-prefix fork).

A sweep row is a ``SweepMethod``: an importance method (or none, for importance-free codecs), the
layer its importance is read at (default: the boundary layer), the selection rule ("ratio" or
"top_rho") and the codec.  That covers all three reference drivers with one engine:
``Experiments/Qwen2-0.5B/main.py`` (4 methods x layers x ratios), the Pythia ``initial`` sweep
(``initial_exp.py:113-122``: orderings from other layers, top-rho, boundary fixed at layer 2, all
ratios of a window in ONE stacked suffix forward) and the channel sweep (``channel_wise.py:35-68``:
4 importance-free codecs forked from one prefix).

Results keep the reference layouts: ``total_nll[method][layer][ratio]`` and
``avg_ppl_results[method][layer][ratio]`` (ordered as in params.json), channel sweeps
``[layer][method]``, plus the unweighted mean per-window NLL of the ``initial`` experiment.
Progress is checkpointed every ``checkpoint_every`` windows and resumed.
"""
from __future__ import annotations

import json
import os
import time
from dataclasses import dataclass

import torch

from .. import codec as C
from ..importance import ImportanceTracker, canonical
from ..models.model import DecoderLM
from ..utils import trace
from ..utils.checkpoint import SweepState
from ..utils.graphs import GraphCache
from .windows import WindowBatch, segment_mean, window_nll


@dataclass(frozen=True)
class SweepMethod:
    """One row of a sweep."""
    name: str                          # result key
    method: str | None                 # importance method, None for importance-free codecs
    codec: str | None = None           # None -> SweepConfig.codec
    source_layer: int | None = None    # importance read at this layer instead of the boundary layer
    selection: str = "ratio"           # "ratio" | "top_rho" (codec.wire)


@dataclass
class SweepConfig:
    methods: list                      # method names (str) or SweepMethod
    layers: list
    ratios: list
    codec: str = "ref_int4_global"
    head_weights: torch.Tensor | None = None
    max_fork_tokens: int = 1 << 17     # cap on tokens per stacked suffix forward
    ratio_scale: float = 1.0           # Pythia 'initial' uses ratio in 0..10 meaning 0.1*ratio
    group_relevance: object = None     # head-group codecs: channel-group tables (plan source, PipelineConfig)
    group_avg_bits: float = 4.0

    def rows(self) -> list:
        out = []
        for m in self.methods:
            out.append(m if isinstance(m, SweepMethod) else SweepMethod(str(m), canonical(m)))
        return out


class SweepEngine:
    def __init__(self, model: DecoderLM, sc: SweepConfig, use_graphs: bool = True, keep_windows: bool = False):
        """``keep_windows``: also keep every window's NLL and loss weight (``window_results``: the input of the
        bootstrap intervals in ``eval.stats``)."""
        self.m, self.sc = model, sc
        self._kept = [] if keep_windows else None
        self.spec = C.get_codec(sc.codec)
        self.rows = sc.rows()
        self.methods = [r.name for r in self.rows]
        self.layers = [int(l) for l in sc.layers]
        self.ratios = list(sc.ratios)
        shape = (len(self.methods), len(self.layers), len(self.ratios))
        self.total_nll = torch.zeros(shape, dtype=torch.float64)
        self.sum_window_nll = torch.zeros(shape, dtype=torch.float64)   # unweighted (initial experiment)
        self.n_tokens = 0.0
        self.windows_done = 0
        self.forward_tokens = 0
        self.wire_bytes = torch.zeros(shape, dtype=torch.float64)
        self.tokens_done = 0
        # the model's last layer only at the scored rows (see DecoderLM.layer_rows)
        self.rows_only = os.environ.get("EDGE_LAST_LAYER_ALL_ROWS", "0") in ("", "0")
        self._dev = None               # [total_nll, sum_window_nll] increments on the model's device
        # the unquantized prefix forward has a fixed launch sequence per batch signature: one HIP graph replay
        need = self._needed()
        self._imp_keys = [(meth, L) for meth in sorted(need) for L in sorted(need[meth])]
        self._graphs = GraphCache(self._prefix_flat, enabled=use_graphs and model.device.type == "cuda")
        hw = sc.head_weights  # LRP head table on the model's device once
        self.head_weights = None if hw is None else torch.as_tensor(hw).to(self.m.device, torch.float32).contiguous()

    # -------------------------------------------------------------- one batch
    def _needed(self) -> dict:
        """importance method -> layers its importance is read at."""
        need: dict = {}
        for r in self.rows:
            if r.method is None:
                continue
            src = [r.source_layer] if r.source_layer is not None else self.layers
            need.setdefault(canonical(r.method), set()).update(int(x) for x in src)
        return need

    def _imp_key(self, r: SweepMethod, L: int):
        return (canonical(r.method), r.source_layer if r.source_layer is not None else L)

    def _prefix_flat(self, ids, rows, targets, row_window, n_rows):
        """Graph-capturable prefix on tensors only: (base NLL, h_L for every boundary layer in order, importance for
        every (method, layer) of ``_imp_keys``)."""
        b = WindowBatch(ids, None, rows, targets, row_window, n_rows, None)
        base, saved, imp = self._prefix_eager(b)
        return (base, *[saved[L] for L in self.layers], *[imp[k] for k in self._imp_keys])

    def _prefix(self, batch: WindowBatch):
        """Unquantized forward: base per-window NLL, h_L per boundary layer, importance per (method, layer)."""
        out = self._graphs(batch.ids, batch.rows, batch.targets, batch.row_window, batch.n_rows)
        self.forward_tokens += batch.B * batch.S
        nl = len(self.layers)
        saved = dict(zip(self.layers, out[1:1 + nl]))
        imp = dict(zip(self._imp_keys, out[1 + nl:]))
        return out[0], saved, imp

    def _prefix_eager(self, batch: WindowBatch):
        m, B, S = self.m, batch.B, batch.S
        need = self._needed()
        trackers = {meth: ImportanceTracker(meth, sorted(ls), m.cfg.num_heads, self.head_weights)
                    for meth, ls in need.items()}
        x = m.embed(batch.ids)
        saved = {}
        last = m.cfg.num_layers - 1
        rows = batch.rows
        for i in range(m.cfg.num_layers):
            kinds = set()
            for tr in trackers.values():
                k = tr.stats_for(i)
                if k:
                    kinds.add(k)
            if i == last and not kinds and i not in self.layers and self.rows_only:
                x = m.layer_rows(i, x, B, S, batch.rows, batch.n_rows)    # only the scored rows reach the head
                rows = torch.arange(x.shape[0], device=x.device)
                continue
            x, st = m.layer(i, x, B, S, stats=tuple(sorted(kinds)) or None)
            for tr in trackers.values():
                if tr.stats_for(i):
                    tr.observe(i, st, S)
            if i in self.layers:
                saved[i] = x
        base = window_nll(m.row_nll(x, rows, batch.targets), batch)
        imp = {(meth, L): trackers[meth].importance(L) for meth, ls in need.items() for L in ls}
        return base, saved, imp

    def _spec_at(self, name: str, L: int) -> C.CodecSpec:
        """Codec ``name`` at the boundary after layer L (relevance-allocated group plan for head-group codecs)."""
        spec = C.get_codec(name)
        if not C.wire.needs_plan(spec):
            return spec
        G = self.m.cfg.hidden_size // C.wire.GROUP
        return C.wire.with_plan(spec, C.wire.boundary_group_plan(self.sc.group_relevance, L, G,
                                                                 self.sc.group_avg_bits))

    def _k(self, ratio, S, spec=None):
        return C.wire.num_lo(spec or self.spec, float(ratio) * self.sc.ratio_scale, S)

    def run_batch(self, batch: WindowBatch) -> torch.Tensor:
        """Returns per-window NLL [M, Lc, R, B] for this batch (also accumulated)."""
        m, B, S = self.m, batch.B, batch.S
        with trace.range("sweep/prefix"):
            base, saved, imp = self._prefix(batch)
        M, Lc, R = len(self.methods), len(self.layers), len(self.ratios)
        out = torch.empty(M, Lc, R, B, dtype=torch.float32, device=base.device)
        for li, L in enumerate(self.layers):
            # de-duplicate variants: key -> list of (mi, ri)
            variants: dict = {}
            for mi, row in enumerate(self.rows):
                spec = C.get_codec(row.codec) if row.codec else self.spec
                for ri, r in enumerate(self.ratios):
                    reff = float(r) * self.sc.ratio_scale
                    if C.wire.uses_kvar(spec, row.selection):
                        key = (self._imp_key(row, L), "top_rho", reff, spec.name)
                        variants.setdefault(key, []).append((mi, ri))
                        continue
                    k = self._k(r, S, spec)
                    # no lo tokens and an exact hi class (reference Q1 "ratio 0"): the unquantized base
                    if k == 0 and spec.uses_ratio and spec.hi_fmt == C.wire.NATIVE:
                        out[mi, li, ri] = base
                        self.wire_bytes[mi, li, ri] += C.message_bytes(C.get_codec("passthrough"), B, S,
                                                                       m.cfg.hidden_size, 0.0, m.dtype)
                        continue
                    method_free = k >= S or k == 0 or not spec.needs_importance or row.method is None
                    key = ("all", k, spec.name) if method_free else (self._imp_key(row, L), k, spec.name)
                    variants.setdefault(key, []).append((mi, ri))
            keys = list(variants)
            per_fork = max(1, self.sc.max_fork_tokens // (B * S))
            for c0 in range(0, len(keys), per_fork):
                chunk = keys[c0:c0 + per_fork]
                xs = []
                for key in chunk:
                    src, kk, cname = key[0], key[1], key[-1]
                    spec = self._spec_at(cname, L)
                    im = None if src == "all" else imp[src]
                    if kk == "top_rho":
                        xq, nbytes = C.fake_quant(saved[L], spec, B, S, key[2], importance=im, selection="top_rho")
                    else:
                        xq, nbytes = C.fake_quant(saved[L], spec, B, S, importance=im, k=kk)
                    xs.append(xq)
                    for (mi, ri) in variants[key]:
                        self.wire_bytes[mi, li, ri] += nbytes
                V = len(chunk)
                x = torch.cat(xs, 0)
                off = (torch.arange(V, device=batch.rows.device) * (B * S)).repeat_interleave(batch.rows.numel())
                rows = batch.rows.repeat(V) + off
                for i in range(L + 1, m.cfg.num_layers):
                    if i == m.cfg.num_layers - 1 and self.rows_only:
                        x = m.layer_rows(i, x, V * B, S, rows, batch.n_rows.repeat(V))
                        rows = torch.arange(x.shape[0], device=x.device)
                    else:
                        x, _ = m.layer(i, x, V * B, S)
                # layer-token work in units of full-model forward tokens
                self.forward_tokens += V * B * S * (m.cfg.num_layers - L - 1) / m.cfg.num_layers
                nll = m.row_nll(x, rows, batch.targets.repeat(V))
                wn = segment_mean(nll, batch.n_rows.to(nll.device).repeat(V)).view(V, B)
                for vi, key in enumerate(chunk):
                    for (mi, ri) in variants[key]:
                        out[mi, li, ri] = wn[vi]
        w = batch.weights.to(out.device, non_blocking=True)
        if self._kept is not None:
            self._kept.append((out.detach().clone(), w.detach().clone()))
        od = out.double()
        if self._dev is None:          # device-side running sums: no host sync per batch (flushed by _flush)
            self._dev = [torch.zeros_like(self.total_nll, device=out.device) for _ in range(2)]
        self._dev[0] += (od * w).sum(-1)
        self._dev[1] += od.sum(-1)
        self.n_tokens += float(batch.weights.sum())
        self.windows_done += B
        self.tokens_done += B * S
        return out

    # -------------------------------------------------------------- results
    def window_results(self) -> tuple[torch.Tensor, torch.Tensor]:
        """(per-window NLL [N, methods, layers, ratios], loss weights [N]) of every window run since construction
        (``keep_windows``)."""
        if not self._kept:
            raise RuntimeError("no windows kept (SweepEngine(..., keep_windows=True))")
        nll = torch.cat([o.permute(3, 0, 1, 2).float().cpu() for o, _ in self._kept], 0)
        w = torch.cat([w.float().cpu() for _, w in self._kept], 0)
        return nll, w

    def _flush(self) -> None:
        """Move the device-side NLL sums into the host accumulators (one sync)."""
        if self._dev is not None:
            self.total_nll += self._dev[0].cpu()
            self.sum_window_nll += self._dev[1].cpu()
            self._dev = None

    def ppl(self) -> torch.Tensor:
        self._flush()
        return torch.exp(self.total_nll / self.n_tokens)

    def results(self) -> dict:
        self._flush()
        p = self.ppl()
        return {
            "methods": self.methods, "layers_of_interest": self.layers, "ratios": self.ratios, "codec": self.sc.codec,
            "avg_ppl_results": [[[float(p[mi, li, ri]) for ri in range(len(self.ratios))]
                                 for li in range(len(self.layers))] for mi in range(len(self.methods))],
            "total_nll": self.total_nll.tolist(), "n_tokens": self.n_tokens, "windows": self.windows_done,
            "wire_bytes_per_token": (self.wire_bytes / max(1, self.tokens_done)).tolist(),
            "mean_window_nll": (self.sum_window_nll / max(1, self.windows_done)).tolist(),
        }

    def state(self) -> dict:
        self._flush()
        return {"total_nll": self.total_nll.tolist(), "n_tokens": self.n_tokens, "windows_done": self.windows_done,
                "wire_bytes": self.wire_bytes.tolist(), "tokens_done": self.tokens_done,
                "sum_window_nll": self.sum_window_nll.tolist()}

    def load_state(self, st: dict) -> None:
        self._dev = None
        self.total_nll = torch.tensor(st["total_nll"], dtype=torch.float64)
        self.sum_window_nll = torch.tensor(st["sum_window_nll"], dtype=torch.float64)
        self.n_tokens = float(st["n_tokens"])
        self.windows_done = int(st["windows_done"])
        self.wire_bytes = torch.tensor(st["wire_bytes"], dtype=torch.float64)
        self.tokens_done = int(st.get("tokens_done", 0))


def run_sweep(engine: SweepEngine, batch_iter, state: SweepState | None = None, log_every: int = 1000,
              progress=None, reduce_fn=None) -> dict:
    """Drive ``engine`` over batches with periodic checkpoint/resume."""
    start_windows = 0
    if state is not None:
        saved = state.load()
        if saved is not None:
            engine.load_state(saved["engine"])
            start_windows = saved["windows_done"]
    t0 = time.perf_counter()
    seen = 0
    next_log = (engine.windows_done // log_every + 1) * log_every
    for b in batch_iter:
        if seen + b.B <= start_windows:   # already accounted for in the checkpoint
            seen += b.B
            continue
        seen += b.B
        b = b.to(engine.m.device)
        engine.run_batch(b)
        if progress:
            progress(b.B)
        if engine.windows_done >= next_log:
            next_log += log_every
            if state is not None:
                state.save({"engine": engine.state(), "windows_done": seen})
    if reduce_fn is not None:
        reduce_fn(engine)
    res = engine.results()
    res["seconds"] = time.perf_counter() - t0
    res["forward_tokens"] = engine.forward_tokens
    return res
