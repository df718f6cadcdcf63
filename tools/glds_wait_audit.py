#!/usr/bin/env python
"""Audit of the hand-counted ``s_waitcnt vmcnt(N)`` in the four-wave GEMM prologue (csrc/gemm.hip, ``gemm_4w_kernel``:
``stage_all`` of K-tile 0, ``stage_all`` of K-tile 1, then ``vmcnt(8 | 14 | 15 | 16)`` and the barrier before the first
fragment reads of buffer 0) against the EMITTED gfx950 ISA.

``tools/isa_check.py`` tracks loads into registers; an LDS-DMA load (``global_load_lds_*``) has no destination register
- it writes LDS - so its consumer (a ``ds_read`` of that buffer after the barrier) is invisible to that check.  Here
the rule is checked directly, on the straight-line prologue of every instantiation: vmcnt(N) retires every vector-memory
op except the N most recent, so K-tile 0's LDS DMA (the first NR = 8 + NB ``global_load_lds`` of the kernel, NB = 6 / 7
/ 8 for BN = 192 / 224 / 256) has landed iff at least N vector-memory ops (of any kind: stores and scratch count too)
were issued after the last of them.  Prints one line per instantiation; exit 1 if any prologue violates the rule.

Usage: ``hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S csrc/gemm.hip -o gemm.s``, then
``python tools/glds_wait_audit.py gemm.s``.
"""
from __future__ import annotations

import re
import sys

FUNC = re.compile(r"^(_Z14gemm_4w_kernelILi(\d+)ELi(\d+)ELi(\d+)ELb([01])E(?:L[bi](\d)E)?Ev8GemmArgs):")
VM = re.compile(r"^\s*(global|buffer|scratch|flat)_\w+")
WAIT = re.compile(r"^\s*s_waitcnt\s+.*vmcnt\((\d+)\)")


def audit(path: str) -> int:
    lines = open(path).read().splitlines()
    bad = 0
    i = 0
    while i < len(lines):
        m = FUNC.match(lines[i])
        if not m:
            i += 1
            continue
        name, epi, rh, bn, pb = m.group(1), int(m.group(2)), int(m.group(3)), int(m.group(4)), m.group(5) == "1"
        nr = 8 + {192: 6, 224: 7, 256: 8}[bn]
        vm_ops, glds_pos, verdict = 0, [], None
        j = i + 1
        while j < len(lines) and not lines[j].startswith(".Lfunc_end"):
            s = lines[j].split(";")[0]
            if VM.match(s):
                vm_ops += 1
                if "global_load_lds" in s:
                    glds_pos.append(vm_ops)
            w = WAIT.match(s)
            if w and int(w.group(1)) > 0 and len(glds_pos) >= nr:
                n = int(w.group(1))
                after = vm_ops - glds_pos[nr - 1]
                ok = after >= n
                verdict = (n, len(glds_pos), after, ok)
                break
            if "s_barrier" in s and len(glds_pos) >= nr:
                break
            j += 1
        if verdict is None:
            print(f"{name}: EPI {epi} RH {rh} BN {bn} PB {int(pb)}: no counted prologue wait found")
        else:
            n, g, after, ok = verdict
            bad += not ok
            print(f"{name}: EPI {epi} BN {bn} PB {int(pb)}: K-tile 0 = first {nr} LDS-DMA ops; vmcnt({n}) reached after "
                  f"{g} LDS-DMA ops, {after} vector-memory ops issued after K-tile 0's last -> "
                  f"{'OK (K-tile 0 landed)' if ok else 'HAZARD'}")
        i = j
    return bad


if __name__ == "__main__":
    nbad = sum(audit(p) for p in sys.argv[1:])
    print(f"{nbad} hazard(s)")
    sys.exit(1 if nbad else 0)
