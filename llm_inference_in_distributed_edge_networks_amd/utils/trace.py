"""Tracing / profiling hooks (the reference has only tqdm rates).

* ``trace.range(name)`` - a roctx range (``libroctx64``, shown by ``rocprofv3 --marker-trace``) plus a
  host-side timer, around pipeline phases: ``stage{s}/recv_wait``, ``stage{s}/compute``,
  ``stage{s}/send``, ``sweep/prefix``, ``sweep/fork``...  Enabled with ``EDGE_TRACE=1``; zero cost
  otherwise.
* ``trace.counter(name, value)`` - accumulates counters (wire bytes, windows, tokens).
* ``trace.summary()`` - {name: {"count", "total_s", "mean_ms"}} + counters, JSON-serialisable.
"""
from __future__ import annotations

import contextlib
import ctypes
import glob
import os
import time
from collections import defaultdict

_ENABLED = os.environ.get("EDGE_TRACE", "0") not in ("0", "")
_roctx = None
_times: dict = defaultdict(lambda: [0, 0.0])
_counters: dict = defaultdict(float)


def _load_roctx():
    global _roctx
    if _roctx is not None:
        return _roctx or None
    cands = glob.glob("/opt/rocm/lib/libroctx64.so*") + glob.glob("/opt/rocm*/lib/libroctx64.so*")
    for c in cands:
        try:
            L = ctypes.CDLL(c)
            L.roctxRangePushA.argtypes = [ctypes.c_char_p]
            L.roctxRangePop.argtypes = []
            L.roctxMarkA.argtypes = [ctypes.c_char_p]
            _roctx = L
            return L
        except OSError:
            continue
    _roctx = False
    return None


def enable(flag: bool = True) -> None:
    global _ENABLED
    _ENABLED = flag


def enabled() -> bool:
    return _ENABLED


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors roctx naming
    if not _ENABLED:
        yield
        return
    L = _load_roctx()
    if L:
        L.roctxRangePushA(name.encode())
    t0 = time.perf_counter()
    try:
        yield
    finally:
        dt = time.perf_counter() - t0
        if L:
            L.roctxRangePop()
        rec = _times[name]
        rec[0] += 1
        rec[1] += dt


def mark(name: str) -> None:
    if _ENABLED:
        L = _load_roctx()
        if L:
            L.roctxMarkA(name.encode())


def counter(name: str, value: float) -> None:
    if _ENABLED:
        _counters[name] += value


def summary() -> dict:
    out = {k: {"count": c, "total_s": t, "mean_ms": 1000 * t / max(c, 1)} for k, (c, t) in _times.items()}
    out["counters"] = dict(_counters)
    return out


def reset() -> None:
    _times.clear()
    _counters.clear()
