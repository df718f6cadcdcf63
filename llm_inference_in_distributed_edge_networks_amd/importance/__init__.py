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
    """LRP head weights ``[layers][heads]`` -> fp32 tensor, from ``attention_head_weights.json`` (what
    ``Experiments/Relevance/main.py:127-128`` writes) or ``attention_head_weights.pkl`` (what the reference's Qwen2
    sweep reads, ``Experiments/Qwen2-0.5B/main.py:129-130``, written by ``pickle.dump`` in
    ``Notebooks/attention_head_weights_via_relevance.ipynb``).  A pickle is never unpickled by ``pickle``: see
    :func:`_load_table_pickle`."""
    if path.endswith(".pkl") or path.endswith(".pickle"):
        w = _load_table_pickle(path)
    else:
        with open(path) as f:
            w = json.load(f)
    return _validated_table(w, path)


def _validated_table(w, path: str) -> torch.Tensor:
    if isinstance(w, torch.Tensor):
        w = w.tolist()
    ok = isinstance(w, (list, tuple)) and len(w) > 0 and all(isinstance(r, (list, tuple)) and len(r) > 0 for r in w)
    ok = ok and all(isinstance(v, (int, float)) and not isinstance(v, bool) for r in w for v in r)
    if not ok or len({len(r) for r in w}) != 1:
        raise ValueError(f"{path}: head weights must be a [layers][heads] table of numbers")
    return torch.tensor([[float(v) for v in r] for r in w], dtype=torch.float32)


# pickle opcodes a list / tuple of lists / tuples of numbers is made of (any protocol); everything that could name,
# build or call an object (GLOBAL, STACK_GLOBAL, REDUCE, BUILD, INST, OBJ, NEWOBJ, PERSID, EXT*, ...) is refused
_TABLE_OPS = {"PROTO", "FRAME", "STOP", "MARK", "EMPTY_LIST", "LIST", "APPEND", "APPENDS", "EMPTY_TUPLE", "TUPLE",
              "TUPLE1", "TUPLE2", "TUPLE3", "BINFLOAT", "FLOAT", "BININT", "BININT1", "BININT2", "INT", "LONG",
              "LONG1", "MEMOIZE", "PUT", "BINPUT", "LONG_BINPUT", "GET", "BINGET", "LONG_BINGET"}


def _load_table_pickle(path: str):
    """A numbers table from a pickle file, executing nothing from it.

    First ``torch.load(path, weights_only=True)`` (torch's restricted unpickler; it reads protocol <= 2 and
    ``torch.save`` files).  It refuses protocol-4 framing (``pickle.dump``'s default, opcode FRAME), which is what the
    reference notebook writes, so a refused file is then decoded by walking its opcode stream with
    ``pickletools.genops`` (a decoder: it constructs nothing) and rebuilding the value from a whitelist of list /
    tuple / number / memo opcodes.  Any other opcode - a class, a callable, a persistent id - is refused."""
    import pickle
    import pickletools
    import warnings
    try:
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")   # (its note on protocols it was not written for)
            return torch.load(path, weights_only=True)
    except (pickle.UnpicklingError, RuntimeError, EOFError, AttributeError, ValueError):
        pass
    with open(path, "rb") as f:
        data = f.read()
    stack: list = []
    marks: list[int] = []
    memo: dict[int, object] = {}
    result = None
    for op, arg, _pos in pickletools.genops(data):
        n = op.name
        if n not in _TABLE_OPS:
            raise ValueError(f"{path}: refusing pickle opcode {n} (only lists / tuples of numbers are accepted)")
        if n in ("PROTO", "FRAME"):
            continue
        if n == "MARK":
            marks.append(len(stack))
        elif n == "EMPTY_LIST":
            stack.append([])
        elif n == "EMPTY_TUPLE":
            stack.append(())
        elif n in ("LIST", "TUPLE"):
            k = marks.pop()
            items = stack[k:]
            del stack[k:]
            stack.append(list(items) if n == "LIST" else tuple(items))
        elif n in ("TUPLE1", "TUPLE2", "TUPLE3"):
            k = int(n[-1])
            items = tuple(stack[-k:])
            del stack[-k:]
            stack.append(items)
        elif n == "APPEND":
            v = stack.pop()
            if not isinstance(stack[-1], list):
                raise ValueError(f"{path}: APPEND to a non-list")
            stack[-1].append(v)
        elif n == "APPENDS":
            k = marks.pop()
            items = stack[k:]
            del stack[k:]
            if not isinstance(stack[-1], list):
                raise ValueError(f"{path}: APPENDS to a non-list")
            stack[-1].extend(items)
        elif n in ("BINFLOAT", "FLOAT", "BININT", "BININT1", "BININT2", "INT", "LONG", "LONG1"):
            if isinstance(arg, bool) or not isinstance(arg, (int, float)):
                raise ValueError(f"{path}: non-numeric scalar {arg!r}")
            stack.append(arg)
        elif n == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif n in ("PUT", "BINPUT", "LONG_BINPUT"):
            memo[int(arg)] = stack[-1]
        elif n in ("GET", "BINGET", "LONG_BINGET"):
            stack.append(memo[int(arg)])
        elif n == "STOP":
            if len(stack) != 1 or marks:
                raise ValueError(f"{path}: malformed pickle")
            result = stack.pop()
            break
    if result is None:
        raise ValueError(f"{path}: no value in pickle")
    return result


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
