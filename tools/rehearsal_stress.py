#!/usr/bin/env python
"""Instrumented repeat of the 4-rank shared-GPU pp4 rehearsal (tests/test_rehearsal_gpu.py
``test_four_stage_pipeline_one_gpu_equals_local``), for the round-5 one-off 509.05-vs-503.23 PPL.

One single-process run (``--pp 4``, the reference) and ``--runs`` 4-rank runs of the same bench step, every one with
``EDGE_DUMP_NLL`` (the last stage saves each micro-batch's per-window NLL) and ``EDGE_P2P_CHECK=1`` (every boundary
message is fingerprinted with a sequence number and checked on arrival, with the HIP graphs on).  Each multi-rank
run's per-window NLLs are compared bit for bit with the reference's: a wrong PPL is then traced to the micro-batches /
windows that differ, and a transport corruption raises in the checked transport.  Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["bench.py", "--model", "tiny-qwen2", "--batch", "4", "--microbatches", "2", "--steps", "3", "--warmup", "1",
        "--max-length", "256", "--split", "1", "--pp", "4", "--no-bf16", "--no-fp32-weights", "--no-hf-compare",
        "--no-transports", "--no-sweep", "--no-hf-compare"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run(n, prefix, extra_env=None, timeout=240):
    env = dict(os.environ, EDGE_SHARED_GPU="1", EDGE_DUMP_NLL=prefix, **(extra_env or {}))
    if n == 1:
        cmd = [sys.executable] + ARGS
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", "--master-addr",
               "127.0.0.1", "--master-port", str(_port())] + ARGS + ["--gpus", str(n)]
    t0 = time.time()
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    if r.returncode != 0:
        return {"rc": r.returncode, "stderr": r.stderr[-2000:], "s": round(time.time() - t0, 1)}
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    return {"rc": 0, "ppl": d["ppl_random_weights"], "s": round(time.time() - t0, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=8)
    ap.add_argument("--out", default="gpurun_out/rehearsal_stress")
    ap.add_argument("--hog-seconds", type=float, default=0.0,
                    help="> 0: the 4-rank runs share the GPU with tools/contention_check.py's hog (2 GiB copies + fp16 "
                         "GEMMs back to back in a fifth process) for at most this long")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    tmp = tempfile.mkdtemp(prefix="stress_")
    ref = run(1, os.path.join(tmp, "ref"))
    ref_nll = torch.load(os.path.join(tmp, "ref.local.1.pt"))
    rows = []
    child = None
    if a.hog_seconds > 0:
        child = subprocess.Popen([sys.executable, os.path.join(ROOT, "tools", "contention_check.py"), "--hog-child",
                                  "--hog-seconds", str(a.hog_seconds)], stdout=subprocess.PIPE, text=True)
        assert child.stdout.readline().strip() == "hog running"
    for k in range(a.runs):
        pre = os.path.join(tmp, f"r{k}")
        r = run(4, pre, {"EDGE_P2P_CHECK": "1"})
        if r["rc"] == 0:
            got = torch.load(f"{pre}.rank3.1.pt")
            diff = (got - ref_nll).abs()
            r["bit_identical"] = bool(torch.equal(got, ref_nll))
            r["max_abs_diff"] = float(diff.max())
            bad = (diff > 0).nonzero().tolist()
            r["differing_microbatch_window"] = bad[:32]
            r["ppl_equal"] = r["ppl"] == ref["ppl"]
        rows.append(r)
        print(json.dumps({"run": k, **r}), flush=True)
        if r["rc"] != 0 and r["rc"] in (124, 134, 137, 139, -6, -11):
            break
    if child is not None:
        r_hog = child.poll()
        if r_hog is None:
            child.terminate()
        child.wait(timeout=60)
    out = {"reference": ref, "runs": rows, "hog": child is not None and r_hog is None, "all_identical": all(r.get("bit_identical") for r in rows),
           "microbatches_x_windows": list(ref_nll.shape)}
    with open(os.path.join(a.out, "summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "runs"}))


if __name__ == "__main__":
    main()
