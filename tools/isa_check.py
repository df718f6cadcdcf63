#!/usr/bin/env python
"""Static check of the emitted gfx950 ISA for memory-return hazards the compiler cannot see.

Several kernels issue instructions from inline asm (``DS_READ_B128`` in ``csrc/gemm.hip``, hand-counted
``s_waitcnt vmcnt(N)`` in the GEMM prologue and the attention K/V ring).  The compiler's waitcnt pass does not
track an asm instruction's result, so it will happily copy, spill or overwrite a VGPR whose LDS / memory return
is still outstanding - a read of stale data whose likelihood grows with memory latency (i.e. under load from
other processes on the same GPU).  This tool walks every kernel's basic blocks (a forward dataflow over the
control-flow graph, loops iterated to a fixed point) and reports any instruction that touches a VGPR / AGPR
while a load into it is still pending:

* LDS returns (``ds_read*``) retire at ``s_waitcnt lgkmcnt(n)``: LDS ops return in order among themselves, so
  ``lgkmcnt(n)`` retires all but the ``n`` most recent lgkm ops (scalar memory ops are counted too, which makes
  the check conservative).
* Vector memory returns (``global_/buffer_/scratch_/flat_load*`` into registers) retire at ``vmcnt(n)``: every
  vector-memory op, stores and ``global_load_lds`` included, is counted in issue order.

Usage: ``python tools/isa_check.py file.s [--kernel REGEX]`` where ``file.s`` comes from
``hipcc --offload-arch=gfx950 -O3 --cuda-device-only -S csrc/X.hip``.  Exit status 1 if a hazard is found.
"""
from __future__ import annotations

import argparse
import re
import sys

REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)\b)")
WAIT = re.compile(r"^s_waitcnt\b(.*)")
BR = re.compile(r"^s_(c?branch\w*)\s+(\S+)")
LDS_LOAD = re.compile(r"^ds_(read|load)\w*")
LDS_OTHER = re.compile(r"^ds_\w+")
VM_LOAD_REG = re.compile(r"^(global|buffer|scratch|flat)_load\w*")
VM_ANY = re.compile(r"^(global|buffer|scratch|flat)_\w+")
SMEM = re.compile(r"^s_(load|buffer_load)\w*")


def regs(text: str) -> set:
    out = set()
    for m in REG.finditer(text):
        k = m.group(1)
        if m.group(4) is not None:
            out.add((k, int(m.group(4))))
        else:
            for r in range(int(m.group(2)), int(m.group(3)) + 1):
                out.add((k, r))
    return out


def parse_functions(path: str, kernel_re: str | None):
    """{name: [(lineno, label|None, instr|None)]} for every function in the file."""
    funcs, cur, name = {}, None, None
    kre = re.compile(kernel_re) if kernel_re else None
    with open(path) as f:
        for no, raw in enumerate(f, 1):
            line = raw.split(";")[0].rstrip()
            if not line.strip():
                continue
            m = re.match(r"^([A-Za-z_.$][\w.$]*):", line)
            if m and not line.startswith("\t") and not line.startswith(" "):
                lab = m.group(1)
                if lab.startswith("_Z") or (not lab.startswith(".") and "$" not in lab):
                    name = lab
                    cur = [] if (kre is None or kre.search(lab)) else None
                    if cur is not None:
                        funcs[name] = cur
                    continue
                if cur is not None:
                    cur.append((no, lab, None))
                continue
            if cur is None:
                continue
            s = line.strip()
            if s.startswith(".") or s.startswith("//"):
                if s.startswith(".Lfunc_end"):
                    cur = None
                continue
            cur.append((no, None, s))
    return funcs


def blocks(items):
    """Split into basic blocks: [(label, [(no, instr)], succ_labels, falls_through)]."""
    out = []
    label, body = "__entry__", []

    def close(fall):
        nonlocal label, body
        out.append([label, body, [], fall])
        body = []

    for no, lab, ins in items:
        if lab is not None:
            if body or label == "__entry__":
                close(True)
            label = lab
            continue
        body.append((no, ins))
        op = ins.split()[0]
        m = BR.match(ins)
        if m:
            tgt = m.group(2)
            cond = m.group(1).startswith("cbranch")
            out.append([label, body, [tgt], cond])
            body = []
            label = f"__after_{no}"
        elif op in ("s_endpgm", "s_setpc_b64"):
            out.append([label, body, [], False])
            body = []
            label = f"__after_{no}"
    if body:
        close(False)
    # successors: explicit targets + fallthrough to the next block
    for i, b in enumerate(out):
        if b[3] and i + 1 < len(out):
            b[2].append(out[i + 1][0])
    return out


def wait_counts(arg: str):
    vm = re.search(r"vmcnt\((\d+)\)", arg)
    lg = re.search(r"lgkmcnt\((\d+)\)", arg)
    if not vm and not lg and arg.strip() and re.fullmatch(r"\s*(0x[0-9a-fA-F]+|\d+)\s*", arg):
        v = int(arg.strip(), 0)   # raw encoding (gfx9): vmcnt lo[3:0] hi[15:14], lgkmcnt[11:8]
        return (v & 0xF) | (((v >> 14) & 3) << 4), (v >> 8) & 0xF
    return (int(vm.group(1)) if vm else None), (int(lg.group(1)) if lg else None)


SREG = re.compile(r"\bs(?:\[(\d+):(\d+)\]|(\d+)\b)")


def sregs(text: str) -> tuple:
    m = SREG.match(text.strip())
    if not m:
        return ()
    if m.group(3) is not None:
        return (int(m.group(3)),)
    return tuple(range(int(m.group(1)), int(m.group(2)) + 1))


def step(state, no, ins, report):
    """state = (lgkm queue, vm queue, scalar constants): the queues are tuples of (issue line, kind, frozenset(regs));
    the constants (frozenset of (sgpr, value) and ("vcc", nonzero?)) make the check path-sensitive for the
    ``s_mov_b64 s[x], -1 / 0 ... s_andn2_b64 vcc, exec, s[x] ; s_cbranch_vccnz`` diamonds the compiler emits for
    if/else around asm.  Returns the new state."""
    lg, vm, cs = list(state[0]), list(state[1]), dict(state[2])
    op = ins.split()[0]
    m = WAIT.match(ins)
    if m:
        v, l = wait_counts(m.group(1))
        if l is not None:
            lg = lg[len(lg) - l:] if l < len(lg) else lg
            if l == 0:
                lg = []
        if v is not None:
            vm = vm[len(vm) - v:] if v < len(vm) else vm
            if v == 0:
                vm = []
        return tuple(lg), tuple(vm), frozenset(cs.items())
    args = ins.split(None, 1)[1] if " " in ins else ""
    if op.startswith("s_"):
        parts = [x.strip() for x in args.split(",")]
        if op in ("s_mov_b64", "s_mov_b32") and len(parts) == 2 and re.fullmatch(r"-?\d+", parts[1]):
            for r in sregs(parts[0]):
                cs[r] = int(parts[1])
        elif op == "s_andn2_b64" and parts[:2] == ["vcc", "exec"]:
            rs = sregs(parts[2])
            vals = {cs.get(r) for r in rs}
            cs["vcc"] = None if None in vals or len(vals) != 1 else (vals.pop() == 0)   # exec & ~s: nonzero iff s == 0
        elif parts and parts[0] and not op.startswith(("s_cbranch", "s_branch", "s_cmp", "s_wait", "s_barrier", "s_nop",
                                                        "s_setprio", "s_sched", "s_endpgm")):
            for r in sregs(parts[0]):
                cs.pop(r, None)
            if parts[0].startswith("vcc"):
                cs.pop("vcc", None)
    elif op.startswith("v_cmp") or "vcc" in args.split(",")[0]:
        cs.pop("vcc", None)
    is_lds_load = bool(LDS_LOAD.match(op))
    is_vm_load = bool(VM_LOAD_REG.match(op)) and "_lds" not in op and not ins.rstrip().endswith(" lds")
    if is_lds_load or is_vm_load:
        # a load's destination may be re-targeted by a later load of the same queue (returns are in order: the later
        # one lands last); its other operands are reads
        dst_w, touched = regs(args.split(",")[0]), regs(args.split(",", 1)[1]) if "," in args else set()
    else:
        dst_w, touched = set(), regs(args)
    for q, same in ((lg, is_lds_load), (vm, is_vm_load)):
        for (src, kind, rs) in q:
            hit = (rs & touched) | (set() if same else (rs & dst_w))
            if hit and kind.endswith("load"):
                report.add((no, ins, src, tuple(sorted(hit))[:4]))
    if is_lds_load:
        lg.append((no, "lds_load", frozenset(dst_w)))
    elif LDS_OTHER.match(op):
        lg.append((no, "lds", frozenset()))
    elif SMEM.match(op):
        lg.append((no, "smem", frozenset()))
    elif is_vm_load:
        vm.append((no, "vm_load", frozenset(dst_w)))
    elif VM_ANY.match(op):
        vm.append((no, "vm", frozenset()))
    return tuple(lg[-64:]), tuple(vm[-64:]), frozenset(cs.items())


def successors(block, state):
    """The successor labels a block can reach in ``state`` (a vcc branch on a known vcc goes one way)."""
    label, body, succ, fall = block
    if not body:
        return succ
    last = body[-1][1]
    m = BR.match(last)
    if m and m.group(1) in ("cbranch_vccnz", "cbranch_vccz"):
        v = dict(state[2]).get("vcc")
        if v is not None:
            taken = v if m.group(1) == "cbranch_vccnz" else not v
            tgt = succ[0]
            rest = succ[1:]
            return [tgt] if taken else rest
    return succ


def merge(a, b):
    """Path-insensitive join of two states: the union of the pending loads (issue order), the common constants."""
    if a is None:
        return b
    if b is None:
        return a

    def mq(x, y):
        out = sorted(set(x) | set(y), key=lambda e: e[0])
        return tuple(out[-64:])
    return mq(a[0], b[0]), mq(a[1], b[1]), frozenset(set(a[2]) & set(b[2]))


MAX_STATES = 8


def check_function(items):
    """Forward dataflow over the blocks.  States at a block are kept apart only by their tracked scalar constants
    (the registers some ``s_andn2_b64 vcc, exec, s[..]`` reads); states with the same constants are joined."""
    bl = blocks(items)
    if not bl:
        return []
    tracked = set()
    for _, lab, ins in items:
        if ins and ins.startswith("s_andn2_b64 vcc, exec,"):
            tracked.update(sregs(ins.split(",")[2]))
    index = {b[0]: i for i, b in enumerate(bl)}
    entry = {0: {frozenset(): ((), (), frozenset())}}
    report = set()
    work = [0]
    iters = 0
    while work and iters < 200000:
        iters += 1
        i = work.pop(0)
        for st0 in list(entry[i].values()):
            st = st0
            for no, ins in bl[i][1]:
                st = step(st, no, ins, report)
            st = (st[0], st[1], frozenset((k, v) for k, v in st[2] if k in tracked or k == "vcc"))
            for s in successors(bl[i], st):
                j = index.get(s)
                if j is None:
                    continue
                cur = entry.setdefault(j, {})
                key = st[2]
                new = merge(cur.get(key), st)
                new = (new[0], new[1], key)
                if cur.get(key) == new:
                    continue
                cur[key] = new
                if j not in work:
                    work.append(j)
    return sorted(report)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm", nargs="+")
    ap.add_argument("--kernel", default=None, help="regex on the mangled kernel name")
    ap.add_argument("--max", type=int, default=20)
    a = ap.parse_args()
    bad = 0
    nk = 0
    for path in a.asm:
        for name, items in parse_functions(path, a.kernel).items():
            nk += 1
            rep = check_function(items)
            if rep:
                bad += 1
                print(f"{path}: {name}: {len(rep)} instruction(s) touch a register with a pending load")
                for no, ins, src, hit in rep[: a.max]:
                    print(f"  line {no}: {ins}    <- pending load from line {src}, regs {hit}")
    print(f"checked {nk} function(s): {bad} with hazards")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
