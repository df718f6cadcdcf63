"""Rank-aware logging and progress (reference: tqdm over windows + periodic prints)."""
from __future__ import annotations

import os
import sys
import time


def _rank() -> int:
    return int(os.environ.get("RANK", "0"))


def log(msg: str, all_ranks: bool = False) -> None:
    if all_ranks or _rank() == 0:
        print(f"[{time.strftime('%H:%M:%S')}][r{_rank()}] {msg}", file=sys.stderr, flush=True)


class _NullBar:
    def update(self, n=1):
        pass

    def close(self):
        pass


def progress_bar(total: int, enabled: bool = True, desc: str = "windows"):
    if not enabled or os.environ.get("EDGE_NO_PROGRESS"):
        return _NullBar()
    try:
        from tqdm import tqdm
        return tqdm(total=total, desc=desc, file=sys.stderr, mininterval=5.0)
    except ImportError:
        return _NullBar()
