"""Build the gfx950 kernel library in-tree: ``hipcc --offload-arch=gfx950 -O3 -shared`` over ``csrc/*.hip``.

No torch headers are involved (plain C ABI, loaded with ctypes), so a rebuild takes seconds and the
resulting ``.so`` travels with the source tree to the GPU machines."""
from __future__ import annotations

import glob
import os
import shutil
import subprocess

from ._native import LIB_PATH

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "csrc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0] or "gfx950"


def _hipcc() -> str:
    for c in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def sources() -> list[str]:
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def up_to_date() -> bool:
    if not os.path.exists(LIB_PATH):
        return False
    t = os.path.getmtime(LIB_PATH)
    deps = sources() + glob.glob(os.path.join(CSRC, "*.h"))
    return all(os.path.getmtime(d) <= t for d in deps)


COMM_LIB = os.path.join(os.path.dirname(LIB_PATH), "libedge_comm.so")
COMM_SRC = os.path.join(CSRC, "comm", "rccl_comm.cpp")


def build_comm(force: bool = False, verbose: bool = False) -> str:
    """The native RCCL transport (links librccl; kept out of the kernel library)."""
    if not force and os.path.exists(COMM_LIB) and os.path.getmtime(COMM_LIB) >= os.path.getmtime(COMM_SRC):
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
    return COMM_LIB


def build_native(force: bool = False, verbose: bool = False, extra_flags=()) -> str:
    build_comm(force, verbose)
    if not force and up_to_date():
        return LIB_PATH
    os.makedirs(os.path.dirname(LIB_PATH), exist_ok=True)
    tmp = LIB_PATH + ".tmp"
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC", "-Wall",
           "-Wno-unused-variable", "-Wno-unused-function", *extra_flags, "-o", tmp, *sources()]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build_native(force=True, verbose=True))
