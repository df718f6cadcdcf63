"""HF sliding-window perplexity recipe, batched.

Reference loop (``Experiments/Qwen2-0.5B/main.py:151-180``, ``last_row_exp.py:85-113``)::

    prev_end = 0
    for begin in range(0, N, stride):
        end = min(begin + max_length, N); trg_len = end - prev_end
        target = ids[begin:end].clone(); target[:-trg_len] = -100
        nll = CE(logits[:, :-1], target[:, 1:])            # mean over valid targets
        total_nll += nll * (num_valid - batch)              # num_valid = trg_len, batch = 1
        prev_end = end; if end == N: break
    PPL = exp(total_nll / total_tokens)

Windows are independent, so they are grouped into batches of equal length (all but
the last window have ``S = max_length``).  For every window only the rows whose
logits are scored are listed (``rows``/``targets``): the LM head runs on those
rows only (a ~16x cut at stride 32 / length 512).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch


@dataclass(frozen=True)
class Window:
    idx: int
    begin: int
    end: int
    trg_len: int

    @property
    def length(self) -> int:
        return self.end - self.begin

    @property
    def weight(self) -> int:
        # num_loss_tokens = num_valid_tokens - batch_size (batch_size = 1 in the reference).  With stride >
        # max_length, trg_len exceeds the window and the reference's target[:, :-trg_len] = -100 masks nothing:
        # all length tokens are valid.
        return min(self.trg_len, self.length) - 1

    @property
    def first_scored(self) -> int:
        return max(0, self.length - self.trg_len - 1)


def sliding_windows(N: int, max_length: int, stride: int) -> list[Window]:
    out, prev_end = [], 0
    for i, begin in enumerate(range(0, N, stride)):
        end = min(begin + max_length, N)
        out.append(Window(i, begin, end, end - prev_end))
        prev_end = end
        if end == N:
            break
    return out


@dataclass
class WindowBatch:
    ids: torch.Tensor          # [B, S] int64 (CPU)
    windows: list
    rows: torch.Tensor         # [R] flat row index b*S + p of every scored logit row
    targets: torch.Tensor      # [R] target token ids
    row_window: torch.Tensor   # [R] window slot (0..B-1) of each row
    n_rows: torch.Tensor       # [B] number of CE terms per window
    weights: torch.Tensor      # [B] float64 num_loss_tokens per window

    @property
    def B(self) -> int:
        return self.ids.shape[0]

    @property
    def S(self) -> int:
        return self.ids.shape[1]

    @property
    def tokens(self) -> int:
        return self.ids.numel()

    def to(self, device) -> "WindowBatch":
        return WindowBatch(self.ids.to(device, non_blocking=True), self.windows, self.rows.to(device),
                           self.targets.to(device), self.row_window.to(device), self.n_rows.to(device),
                           self.weights)


def make_batch(tokens: torch.Tensor, wins: list) -> WindowBatch:
    ids = tokens.view(-1)
    S = wins[0].length
    assert all(w.length == S for w in wins)
    rows, tgts, rw, nr = [], [], [], []
    for b, w in enumerate(wins):
        p = torch.arange(w.first_scored, S - 1)
        rows.append(b * S + p)
        tgts.append(ids[w.begin + p + 1])
        rw.append(torch.full_like(p, b))
        nr.append(p.numel())
    return WindowBatch(
        ids=torch.stack([ids[w.begin:w.end] for w in wins]).contiguous(),
        windows=list(wins), rows=torch.cat(rows), targets=torch.cat(tgts), row_window=torch.cat(rw),
        n_rows=torch.tensor(nr, dtype=torch.float32),
        weights=torch.tensor([w.weight for w in wins], dtype=torch.float64))


def with_bos(batch: WindowBatch, bos: int) -> WindowBatch:
    """The batch with every window's first input token replaced by ``bos`` (a fixed sink / start-of-window token, as
    the byte surrogate is trained with: ``tools/train_tiny_lm.py --bos``).  Position 0 is never a target, so the
    scored rows and their targets are unchanged."""
    ids = batch.ids.clone()
    ids[:, 0] = bos
    return WindowBatch(ids, batch.windows, batch.rows, batch.targets, batch.row_window, batch.n_rows, batch.weights)


def batches(tokens: torch.Tensor, wins: list, batch_size: int, bos: int | None = None):
    """Group consecutive equal-length windows into batches of at most ``batch_size`` (``bos``: see ``with_bos``)."""
    cur = []
    for w in wins:
        if cur and (len(cur) == batch_size or w.length != cur[0].length):
            b = make_batch(tokens, cur)
            yield b if bos is None else with_bos(b, bos)
            cur = []
        cur.append(w)
    if cur:
        b = make_batch(tokens, cur)
        yield b if bos is None else with_bos(b, bos)


def segment_mean(values: torch.Tensor, counts: torch.Tensor) -> torch.Tensor:
    """Mean of consecutive segments of ``values`` (lengths ``counts``), bitwise deterministic on GPU:
    an fp64 prefix sum instead of float atomics (``index_add_``)."""
    cs = torch.cumsum(values.double(), 0)
    ends = torch.cumsum(counts.to(torch.int64), 0) - 1
    tot = cs.index_select(0, ends)
    prev = torch.cat([tot.new_zeros(1), tot[:-1]])
    return ((tot - prev) / counts.double()).float()


def window_nll(row_nll: torch.Tensor, batch: WindowBatch) -> torch.Tensor:
    """Per-window mean CE over its scored rows (rows are grouped by window): [B] fp32."""
    return segment_mean(row_nll, batch.n_rows.to(row_nll.device))


class PPLAccumulator:
    """Token-weighted NLL accumulation, exactly the reference's ``total_nll``/``n_tokens``.

    ``add`` keeps the running NLL sum on the device of the per-window NLLs (fp64, no host sync per batch); reading
    ``total_nll`` synchronises once."""

    def __init__(self):
        self._host_nll = 0.0
        self._dev_nll = None
        self.n_tokens = 0.0

    def add(self, wnll: torch.Tensor, batch: WindowBatch) -> None:
        w = batch.weights
        contrib = (wnll.double() * w.to(wnll.device, non_blocking=True)).sum()
        self._dev_nll = contrib if self._dev_nll is None else self._dev_nll + contrib
        self.n_tokens += float(w.sum())

    @property
    def total_nll(self) -> float:
        if self._dev_nll is not None:
            self._host_nll += float(self._dev_nll)
            self._dev_nll = None
        return self._host_nll

    @total_nll.setter
    def total_nll(self, v: float) -> None:
        self._dev_nll = None
        self._host_nll = float(v)

    def ppl(self) -> float:
        return math.exp(self.total_nll / self.n_tokens) if self.n_tokens else float("nan")
