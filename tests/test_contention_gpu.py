"""Bit-identity of the pipeline step under contention (tools/contention_check.py; docs/RESULTS.md section 2): the
2-stage split on HIP graphs, fp32 and bf16, replayed while another process floods the same GPU with copies and GEMMs,
gives every window's NLL bit for bit as on the idle GPU.  A kernel that consumes a load before it has landed (a
missing or miscounted s_waitcnt) passes on an idle GPU and fails here."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_pipeline_step_bit_identical_under_contention(tmp_path):
    out = tmp_path / "c.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "contention_check.py"), "--model", "tiny-qwen2",
                        "--batch", "8", "--microbatches", "3", "--repeats", "3", "--hog-seconds", "60", "--out",
                        str(out)], cwd=ROOT, capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    d = json.loads(out.read_text())
    assert d["all_identical"] and d["under_contention"] == 6 and all(d["idle_identical"].values())
