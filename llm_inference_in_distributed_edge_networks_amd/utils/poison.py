"""Poison-fill debug mode (SURVEY §5.2 race / uninitialised-read detection).

``EDGE_POISON=1`` makes every buffer the framework gets from ``torch.empty`` / ``empty_like`` / ``new_empty`` (receive
and message buffers, ``GraphCache`` static buffers, codec / GEMM / attention workspaces, kernel outputs) start as
NaN (floating point) or all-ones bits (integers, 0xFF bytes) instead of whatever the caching allocator last left
there.  A kernel or a transport that reads memory nobody wrote for this step then gives a NaN or a wildly wrong
answer EVERY time, not an intermittent small error that depends on which block the allocator happened to reuse.
Inside a captured HIP graph the fill is captured too, so each replay re-poisons the step's intermediates.

``EDGE_POISON=2`` additionally launches ``csrc/debug.hip``'s ``lds_poison_kernel`` on the current stream before every
framework kernel (``ops._native.call``): it fills the LDS of every CU and the register file of every SIMD with
all-ones bits, so a kernel reading LDS / a VGPR / an AGPR it never wrote sees NaN every time.  Neither is cleared
between workgroups by the hardware: without it such a read returns what an earlier workgroup left, which changes
when other processes share the GPU (the 4-rank rehearsal's setting).

Mechanism (level 1): PyTorch's own ``torch.utils.deterministic.fill_uninitialized_memory`` (active only while deterministic
algorithms are on; ``warn_only`` so ops without a deterministic variant still run).  Set in the environment, the mode
is inherited by every rank a launcher starts; ``enable()`` is called on package import.
"""
from __future__ import annotations

import os

_ON = False


def level() -> int:
    """0 off, 1 poisoned torch.empty, 2 also poisoned LDS / registers before every kernel (``EDGE_POISON``)."""
    v = os.environ.get("EDGE_POISON", "0").strip()
    return int(v) if v.isdigit() else (1 if v else 0)


def requested() -> bool:
    return level() > 0


def active() -> bool:
    return _ON


def enable() -> None:
    global _ON
    import torch
    import torch.utils.deterministic
    torch.use_deterministic_algorithms(True, warn_only=True)
    torch.utils.deterministic.fill_uninitialized_memory = True
    _ON = True


def from_env() -> bool:
    if requested() and not _ON:
        enable()
    return _ON
