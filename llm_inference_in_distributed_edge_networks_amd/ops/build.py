"""Build the gfx950 kernel library in-tree: ``hipcc --offload-arch=gfx950 -O3`` over ``csrc/*.hip``.

No torch headers are involved (plain C ABI, loaded with ctypes), so the resulting ``.so`` travels with the
source tree to the GPU machines.  Each ``.hip`` translation unit compiles to its own object (in parallel), and
everything is keyed on CONTENT, not mtimes: an object is named by the hash of its source, the shared headers and
the compiler flags, and the library carries a ``.hash`` stamp of all of them.  A library copied next to sources it
was not built from (a stale ``.so`` newer than edited sources, as on a pushed snapshot) is therefore rebuilt.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import os
import shutil
import subprocess

from ._native import LIB_PATH

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "csrc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0] or "gfx950"
OBJ_DIR = os.path.join(os.path.dirname(LIB_PATH), "obj")
COMM_LIB = os.path.join(os.path.dirname(LIB_PATH), "libedge_comm.so")
COMM_SRC = os.path.join(CSRC, "comm", "rccl_comm.cpp")
CFLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-variable", "-Wno-unused-function"]


def _hipcc() -> str:
    for c in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def sources() -> list[str]:
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def headers() -> list[str]:
    return sorted(glob.glob(os.path.join(CSRC, "*.h")))


def _digest(paths, extra=()) -> str:
    h = hashlib.sha256()
    for p in paths:
        h.update(os.path.basename(p).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    for e in extra:
        h.update(str(e).encode())
    return h.hexdigest()[:20]


def _flags(extra_flags=()) -> list[str]:
    return [f"--offload-arch={ARCH}", *CFLAGS, *extra_flags]


def _obj_path(src: str, flags) -> str:
    return os.path.join(OBJ_DIR, f"{os.path.basename(src)}.{_digest([src, *headers()], flags)}.o")


def library_hash(extra_flags=()) -> str:
    flags = _flags(extra_flags)
    return _digest(sources() + headers(), flags)


def _read(p):
    try:
        with open(p) as f:
            return f.read().strip()
    except OSError:
        return ""


def up_to_date(extra_flags=()) -> bool:
    return os.path.exists(LIB_PATH) and _read(LIB_PATH + ".hash") == library_hash(extra_flags)


def _compile(src, flags, verbose):
    obj = _obj_path(src, flags)
    if os.path.exists(obj):
        return obj
    tmp = obj + f".tmp{os.getpid()}"
    cmd = [_hipcc(), *flags, "-c", src, "-o", tmp]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, obj)
    return obj


def build_comm(force: bool = False, verbose: bool = False) -> str:
    """The native RCCL transport (links librccl; kept out of the kernel library)."""
    h = _digest([COMM_SRC], ["comm", ARCH])
    if not force and os.path.exists(COMM_LIB) and _read(COMM_LIB + ".hash") == h:
        return COMM_LIB
    os.makedirs(os.path.dirname(COMM_LIB), exist_ok=True)
    tmp = COMM_LIB + ".tmp"
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O2", "-std=c++17", "-shared", "-fPIC", "-Wall", "-o", tmp, COMM_SRC,
           f"-L{rocm}/lib", "-lrccl", f"-Wl,-rpath,{rocm}/lib"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, COMM_LIB)
    with open(COMM_LIB + ".hash", "w") as f:
        f.write(h)
    return COMM_LIB


def build_native(force: bool = False, verbose: bool = False, extra_flags=(), out: str | None = None,
                 jobs: int | None = None) -> str:
    """Compile (changed) translation units in parallel and link ``libedge_kernels.so`` (or ``out``)."""
    build_comm(force and out is None, verbose)
    target = out or LIB_PATH
    lib_hash = library_hash(extra_flags)
    if not force and os.path.exists(target) and _read(target + ".hash") == lib_hash:
        return target
    os.makedirs(OBJ_DIR, exist_ok=True)
    flags = _flags(extra_flags)
    if force:
        for s in sources():
            p = _obj_path(s, flags)
            if os.path.exists(p):
                os.remove(p)
    jobs = jobs or min(len(sources()), max(1, min(8, os.cpu_count() or 1)))
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, flags, verbose), sources()))
    tmp = target + ".tmp"
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, target)
    with open(target + ".hash", "w") as f:
        f.write(lib_hash)
    # drop objects of older source versions
    keep = set(objs)
    for o in glob.glob(os.path.join(OBJ_DIR, "*.o")):
        if o not in keep and (out is None):
            try:
                os.remove(o)
            except OSError:
                pass
    return target


if __name__ == "__main__":
    print(build_native(force=False, verbose=True))
