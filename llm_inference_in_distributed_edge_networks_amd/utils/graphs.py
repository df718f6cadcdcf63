"""HIP-graph capture of launch-bound stage compute (MI355X replacement for a tracing compiler).

A pipeline stage's forward for a fixed micro-batch signature (B, S, number of scored rows) is a fixed
sequence of ~170 kernel launches (7 per Qwen2 layer + boundary codec + head).  ``GraphCache`` captures
it once per signature into a ``torch.cuda.CUDAGraph`` (hipGraph on ROCm) with static input/output
buffers and replays it: one launch instead of hundreds, no Python or ctypes overhead per kernel.
Kernels launched through the ctypes library go to the current (capturing) stream, so they are
captured like any torch op.  Batches with a new signature (first / last window of a corpus) run
eagerly the first time they are seen and are captured on the second sighting.

Outputs of a replay are the graph's STATIC buffers: the next replay of the same graph overwrites them.  A caller
that hands an output to asynchronous work (an RCCL send of the boundary message) uses ``slot``: each slot is an
independent capture with its own buffers, so with two slots replay i+1 writes other memory than the send of
replay i reads; before replaying a slot again the caller makes the stream wait for that slot's send.
"""
from __future__ import annotations

import gc
from typing import Callable

import torch


_PRERUN = False


def prerun_active() -> bool:
    """True during the extra eager run that precedes a capture: side-effect counters (e.g. wire-byte accumulators)
    skip it so every micro-batch is counted once."""
    return _PRERUN


class GraphCache:
    def __init__(self, fn: Callable, enabled: bool = True, warmup: int = 1):
        """``fn(*tensors) -> tensor or tuple of tensors``; every input must be a tensor."""
        self.fn = fn
        self.enabled = enabled and torch.cuda.is_available()
        self.warmup = warmup
        self.seen: dict = {}
        self.graphs: dict = {}

    @staticmethod
    def _sig(args):
        return tuple((tuple(a.shape), a.dtype, a.device) for a in args)

    def __call__(self, *args, slot: int = 0):
        if not self.enabled or not all(torch.is_tensor(a) and a.is_cuda for a in args):
            return self.fn(*args)
        key = (self._sig(args), slot)
        g = self.graphs.get(key)
        if g is None:
            n = self.seen.get(key, 0)
            self.seen[key] = n + 1
            if n < self.warmup:
                return self.fn(*args)      # also warms allocator / lazy kernel attributes
            g = self._capture(args)
            self.graphs[key] = g
        graph, static_in, static_out = g
        for s, a in zip(static_in, args):
            s.copy_(a, non_blocking=True)
        graph.replay()
        return static_out

    def _capture(self, args):
        static_in = [a.clone() for a in args]
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        global _PRERUN
        with torch.cuda.stream(s):
            _PRERUN = True
            try:
                self.fn(*static_in)  # one more eager run on the capture stream
            finally:
                _PRERUN = False
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        # thread_local: only this thread's stream-unsafe calls invalidate the capture.  Under RCCL the process
        # group's watchdog thread keeps querying its events while a stage captures; in the default "global" mode such
        # a query from another thread aborts the capture.
        # No garbage collection while capturing: a cycle collected mid-capture can hold a dropped CUDAGraph (e.g. of
        # a pipeline rebuilt for another codec), and its destructor is not permitted while a stream captures.  (No
        # collection forced before it either: 2.2 % of the fp32 bench and 3.8 % of the bf16 one, same-box, round 4,
        # profiles/history/r04h/gc_ab_and_lrp.txt.)
        was = gc.isenabled()
        gc.disable()
        try:
            with torch.cuda.graph(graph, capture_error_mode="thread_local"):
                static_out = self.fn(*static_in)
        finally:
            if was:
                gc.enable()
        torch.cuda.synchronize()
        return graph, static_in, static_out

    def clear(self):
        self.graphs.clear()
        self.seen.clear()
