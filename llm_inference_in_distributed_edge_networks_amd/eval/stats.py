"""Window-bootstrap confidence intervals for token-weighted perplexities (the quality experiments' statistics).

A sweep cell's PPL is ``exp(sum_i w_i nll_i / sum_i w_i)`` over windows i (``w_i`` = the window's scored tokens, the
reference's ``num_loss_tokens``, ``Experiments/Qwen2-0.5B/main.py:166-178``).  Windows are the resampling unit: every
bootstrap replicate draws N windows with replacement, and ALL cells are evaluated on the same replicate, so
differences between cells (a method against another, a boundary against another, a cell against the unquantized
ratio 0) are paired and their intervals do not double count the windows' own spread.

``nll`` is [N, cells] per-window mean NLL, ``w`` [N]; intervals are percentile intervals of the replicate
distribution (95 % by default).
"""
from __future__ import annotations

import math

import torch


def _counts(n: int, reps: int, seed: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    idx = torch.randint(0, n, (reps, n), generator=g)
    c = torch.zeros(reps, n, dtype=torch.float64)
    c.scatter_add_(1, idx, torch.ones_like(idx, dtype=torch.float64))
    return c


def bootstrap_log_ppl(nll: torch.Tensor, w: torch.Tensor, reps: int = 1000, seed: int = 0) -> torch.Tensor:
    """[reps, cells] log-PPL of every cell on every window-bootstrap replicate (the same replicates for all cells)."""
    nll = nll.double().reshape(nll.shape[0], -1)
    w = w.double().reshape(-1)
    c = _counts(nll.shape[0], reps, seed)
    return (c @ (w[:, None] * nll)) / (c @ w)[:, None]


def interval(samples: torch.Tensor, level: float = 0.95) -> tuple[float, float]:
    lo = (1 - level) / 2
    q = torch.quantile(samples.double(), torch.tensor([lo, 1 - lo], dtype=torch.float64))
    return float(q[0]), float(q[1])


def log_ppl(nll: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """[cells] point estimates."""
    nll = nll.double().reshape(nll.shape[0], -1)
    w = w.double().reshape(-1)
    return (w[:, None] * nll).sum(0) / w.sum()


def damage_table(nll: torch.Tensor, w: torch.Tensor, base: int, reps: int = 1000, seed: int = 0,
                 level: float = 0.95) -> list[dict]:
    """Per cell: PPL, and its relative change against cell ``base`` (PPL_c / PPL_base - 1) with the paired
    bootstrap interval."""
    pt = log_ppl(nll, w)
    bs = bootstrap_log_ppl(nll, w, reps, seed)
    out = []
    for c in range(pt.numel()):
        d = torch.expm1(bs[:, c] - bs[:, base])
        lo, hi = interval(d, level)
        out.append({"ppl": math.exp(float(pt[c])), "rel": math.expm1(float(pt[c] - pt[base])), "ci": [lo, hi]})
    return out


def paired_diff(nll: torch.Tensor, w: torch.Tensor, a: int, b: int, reps: int = 1000, seed: int = 0,
                level: float = 0.95) -> dict:
    """log PPL_a - log PPL_b (a positive value: cell a is worse) with its paired bootstrap interval, and whether the
    interval excludes 0 ("a worse" / "b worse" / "not resolved")."""
    pt = log_ppl(nll, w)
    bs = bootstrap_log_ppl(nll, w, reps, seed)
    d = bs[:, a] - bs[:, b]
    lo, hi = interval(d, level)
    verdict = "a worse" if lo > 0 else ("b worse" if hi < 0 else "not resolved")
    return {"diff": float(pt[a] - pt[b]), "ci": [lo, hi], "verdict": verdict}
