"""Native RCCL transport (csrc/comm/rccl_comm.cpp) on one GPU: self-loopback send/recv + all-reduce.

Runs in a subprocess so a failure inside RCCL cannot take down the test session."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rccl_self_loopback_and_allreduce():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rccl_selftest.py")], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and "RCCL_SELFTEST_OK" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
