"""Layer-divergence analysis of importance distributions (reference C16,
``Notebooks/distributions_distance_across_layers.ipynb`` cells 10-18).

For every text line with at least 125 characters (JSON line 4800), compute each layer's column-mean
attention importance (a distribution over the line's tokens, sums to 1 under the causal mask), then
the pairwise Jensen-Shannon divergence between layers with log2 KL (JSON lines 4860-4874), averaged
over lines.  Published Pythia-70M values are in BASELINE.md (e.g. JS(0,4) = 0.395).
"""
from __future__ import annotations


import torch

from .. import ops


def js_divergence(p: torch.Tensor, q: torch.Tensor, eps: float = 1e-12) -> float:
    p = p.double().clamp_min(0)
    q = q.double().clamp_min(0)
    p = p / p.sum()
    q = q / q.sum()
    m = 0.5 * (p + q)

    def kl(a, b):
        mask = a > eps
        return float((a[mask] * (a[mask] / b[mask]).log2()).sum())
    return 0.5 * kl(p, m) + 0.5 * kl(q, m)


def layer_importances(model, ids: torch.Tensor) -> torch.Tensor:
    """Column-mean importance of every layer for one sequence: [layers, S]."""
    B, S = ids.shape
    x = model.embed(ids)
    out = []
    for i in range(model.cfg.num_layers):
        x, st = model.layer(i, x, B, S, stats="colsum")
        out.append(ops.head_combine(st.colsum, None, 1.0 / (model.cfg.num_heads * S))[0].float().cpu())
    return torch.stack(out)


def js_matrix(model, sequences, min_chars: int = 125, texts=None) -> torch.Tensor:
    """Average pairwise JS divergence between layers over ``sequences`` (list of [1, S] id tensors)."""
    n = model.cfg.num_layers
    acc = torch.zeros(n, n, dtype=torch.float64)
    cnt = 0
    for si, ids in enumerate(sequences):
        if texts is not None and len(texts[si]) < min_chars:
            continue
        if ids.shape[1] < 2:
            continue
        imp = layer_importances(model, ids.to(model.device))
        for a in range(n):
            for b in range(a + 1, n):
                d = js_divergence(imp[a], imp[b])
                acc[a, b] += d
                acc[b, a] += d
        cnt += 1
    return acc / max(cnt, 1)
