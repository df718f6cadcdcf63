"""Token-importance scorers.

Reference: ``get_importance_order`` in ``Experiments/Qwen2-0.5B/main.py:21-98`` and
``Experiments/Pythia-70M/last_row_exp.py:9-45``, ``extract_attentions`` in
``Experiments/Pythia-70M/initial_exp.py:27-72``.  The reference computes every
score from a second, eager copy of the model that returns all S x S attention
maps.  Here the model emits only the per-head statistics a scorer needs at the
layers it needs them (``DecoderLM.layer(..., stats=...)``): last-row
probabilities or column sums of P recomputed from the row LSE.

Method                  importance of token j for boundary layer L
----------------------  -------------------------------------------------------
regular_importance      mean_h mean_i A_L[h, i, j]            (colsum / (Hq*S))
last_row                mean_h A_L[h, S-1, j]
aggregate_till          mean_{l<=L} regular_importance_l
weighted_importance     mean_i sum_h w[L][h] A_L[h, i, j]     (LRP head weights, signed)
maximum_aggregation     max_{l<=L} regular_importance_l       (Pythia "initial" extra)
"""
from __future__ import annotations

import json

import torch

from .. import ops
from ..models.model import AttnStats

METHODS = ("regular_importance", "last_row", "aggregate_till", "weighted_importance", "maximum_aggregation")
ALIASES = {"aggregate upto 2": "aggregate_till", "maximum aggregation": "maximum_aggregation",
           "column_mean": "regular_importance", "colmean": "regular_importance", "lastrow": "last_row"}


def canonical(method: str) -> str:
    m = ALIASES.get(method, method)
    if m not in METHODS:
        raise KeyError(f"unknown importance method {method!r}; known: {METHODS}")
    return m


def stats_kind(method: str) -> str:
    return "lastrow" if canonical(method) == "last_row" else "colsum"


def needs_all_layers(method: str) -> bool:
    return canonical(method) in ("aggregate_till", "maximum_aggregation")


def load_head_weights(path: str) -> torch.Tensor:
    """``attention_head_weights.json`` ([layers][heads], Relevance/main.py:127-128) -> fp32 tensor."""
    with open(path) as f:
        w = json.load(f)
    return torch.tensor(w, dtype=torch.float32)


class ImportanceTracker:
    """Computes one method's importance at a set of boundary layers during a forward pass.

    Usage per micro-batch: ``need = tr.stats_for(layer)`` before running a layer, then
    ``tr.observe(layer, stats)``; ``tr.importance(L)`` -> ``[B, S]`` fp32 after layer L ran.
    ``carry``/``load_carry`` move the running aggregate across pipeline stages.
    """

    def __init__(self, method: str, boundaries, num_heads: int, head_weights: torch.Tensor | None = None):
        self.method = canonical(method)
        self.boundaries = sorted(set(int(b) for b in boundaries))
        self.Hq = num_heads
        self.head_weights = head_weights
        if self.method == "weighted_importance" and head_weights is None:
            raise ValueError("weighted_importance needs head weights (attention_head_weights.json)")
        self.reset()

    def reset(self):
        self.run_sum = None      # aggregate_till: sum of regular importances of layers seen so far
        self.run_max = None
        self.n_seen = 0
        self.scores: dict[int, torch.Tensor] = {}

    def stats_for(self, layer: int) -> str | None:
        if needs_all_layers(self.method):
            return "colsum" if layer <= max(self.boundaries, default=-1) else None
        return stats_kind(self.method) if layer in self.boundaries else None

    def observe(self, layer: int, st: AttnStats, S: int) -> None:
        m = self.method
        if m == "last_row":
            if layer in self.boundaries:
                self.scores[layer] = ops.head_combine(st.lastrow, None, 1.0 / self.Hq)
            return
        if m == "weighted_importance":
            if layer in self.boundaries:
                w = self.head_weights[layer]
                self.scores[layer] = ops.head_combine(st.colsum, w, 1.0 / S)
            return
        reg = ops.head_combine(st.colsum, None, 1.0 / (self.Hq * S))
        if m == "regular_importance":
            if layer in self.boundaries:
                self.scores[layer] = reg
            return
        self.n_seen += 1
        if m == "aggregate_till":
            self.run_sum = reg.clone() if self.run_sum is None else self.run_sum.add_(reg)
            if layer in self.boundaries:
                self.scores[layer] = self.run_sum / float(layer + 1)
        else:
            self.run_max = reg.clone() if self.run_max is None else torch.maximum(self.run_max, reg)
            if layer in self.boundaries:
                self.scores[layer] = self.run_max.clone()

    def importance(self, layer: int) -> torch.Tensor:
        return self.scores[layer]

    # running state across pipeline stages
    def carry(self) -> torch.Tensor | None:
        if self.method == "aggregate_till":
            return self.run_sum
        if self.method == "maximum_aggregation":
            return self.run_max
        return None

    def load_carry(self, t: torch.Tensor | None, layers_seen: int) -> None:
        if self.method == "aggregate_till":
            self.run_sum = t
        elif self.method == "maximum_aggregation":
            self.run_max = t
        self.n_seen = layers_seen


def reference_importance(method: str, attn_maps: list, layer: int, head_weights=None) -> torch.Tensor:
    """Oracle straight from the reference formulas on full attention maps ``[B, Hq, S, S]`` per layer."""
    m = canonical(method)
    A = attn_maps[layer].float()
    if m == "regular_importance":
        return A.mean(1).mean(1)
    if m == "last_row":
        return A[:, :, -1, :].mean(1)
    if m == "weighted_importance":
        w = head_weights[layer].float().view(1, -1, 1, 1)
        return (A * w).sum(1).mean(1)
    regs = torch.stack([attn_maps[l].float().mean(1).mean(1) for l in range(layer + 1)])
    if m == "aggregate_till":
        return regs.mean(0)
    return regs.max(0).values
