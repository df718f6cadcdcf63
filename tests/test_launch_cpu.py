"""The driver's multi-process launch paths on CPU (gloo): ``torch.distributed.run ... bench.py`` and the
pipeline entry point (BASELINE configs 1-5) under torchrun, compared with their single-process runs."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env():
    e = dict(os.environ, OMP_NUM_THREADS="2", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    e.pop("RANK", None)
    e.pop("WORLD_SIZE", None)
    return e


def _torchrun(n, args, cwd=ROOT, timeout=600):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    return subprocess.run(cmd, cwd=cwd, env=_env(), capture_output=True, text=True, timeout=timeout)


BENCH = ["bench.py", "--model", "tiny-qwen2", "--batch", "2", "--microbatches", "2", "--steps", "2", "--warmup", "1",
         "--max-length", "128", "--split", "1"]


def _json_line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [1, 2, 4])
def test_bench_contract_cpu(n):
    if n == 1:
        r = subprocess.run([sys.executable] + BENCH + ["--gpus", "1"], cwd=ROOT, env=_env(), capture_output=True,
                           text=True, timeout=600)
    else:
        r = _torchrun(n, BENCH + ["--gpus", str(n)])
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == n and d["steps"] == 2 and d["warmup"] == 1 and d["value"] > 0
    dp = max(1, n // 2)
    assert d["config"]["parallelism"] == (f"pp2xdp{dp}" if n > 1 else "local-pp2")
    assert d["config"]["global_batch"] == 2 * 2 * dp
    assert d["ppl_random_weights"] and d["ppl_random_weights"] > 1
    assert d["dtype"] == "fp32" and d["metric"].startswith("WikiText-2 PPL + inter-stage bytes/token")
    assert d["config"]["last_layer_rows"] == "scored"
    # the senders' measured byte counters: for a fixed-k codec exactly the wire layout's message size per token
    from llm_inference_in_distributed_edge_networks_amd import codec as C
    want = C.message_bytes(C.get_codec("mixed_int4_int8"), 2, 128, 256, 0.5, __import__("torch").float32) / (2 * 128)
    assert d["wire_bytes_per_token"] == [round(want, 2)]
    if n > 1:   # per-stage GPU-time breakdown rows, one per rank
        assert len(d["stages"]) == n and {s["stage"] for s in d["stages"]} == {0, 1}
        # the p2p probe of every pipeline edge (one per replica), a 1 MiB and a boundary-sized message
        assert len(d["p2p"]) == 2 * dp
        for row in d["p2p"]:
            assert row["stage"] == 0 and row["edge"][1] == row["edge"][0] + 1
            assert row["p2p_us"] > 0 and row["p2p_GBps"] > 0
        assert {row["bytes"] for row in d["p2p"]} == {1 << 20, round(d["wire_bytes_per_token"][0] * 2 * 128)}
    if n > 2:   # the secondary measurement: one n-stage pipeline over all the ranks (BASELINE config 4 at n = 4)
        _check_deep(d, n)
    else:
        assert "value_pp2" not in d and "pp2" not in d
    if n > 1:   # the per-transport check: torch p2p timed with its probe rows; the native ones need GPUs
        tr = d["transports"]
        assert tr["torch"]["ppl_random_weights"] > 1 and tr["torch"]["ms_per_step"] > 0
        assert len(tr["torch"]["p2p"]) == 2 * dp
        assert tr["rccl"] == tr["ipc"] == {"skipped": "CPU ranks: the native transports need GPUs"}
        assert tr["wall_s"] >= 0
    else:
        assert "transports" not in d
        # the reference's own workload (the notebook sweep) timed beside the headline
        sw = d["notebook_sweep"]
        assert sw["windows"] == 64 and sw["configs_per_window"] == 4 * 2 * 5 and sw["windows_per_s"] > 0
        assert len(sw["pass_seconds"]) == 3 and sw["seconds"] == sorted(sw["pass_seconds"])[1]
        assert d["sweep_speedup_vs_t4"] == round(16.19 / sw["s_per_window"], 1)


def _check_deep(d, n):
    assert d[f"value_pp{n}"] > 0, d.get(f"pp{n}")
    deep = d[f"pp{n}"]
    assert deep["parallelism"] == f"pp{n}xdp1" and len(deep["stage_layers"]) == n
    assert len(deep["stages"]) == n and {s["stage"] for s in deep["stages"]} == set(range(n))
    assert len(deep["wire_bytes_per_token"]) == n - 1 and all(w > 0 for w in deep["wire_bytes_per_token"])
    assert len(deep["p2p"]) == 2 * (n - 1) and {r["stage"] for r in deep["p2p"]} == set(range(n - 1))
    assert deep["ppl_random_weights"] > 1 and deep["ms_per_step"] > 0 and deep["wall_s"] > 0


@pytest.mark.parametrize("pp", [4, 8])
def test_bench_deep_pipeline_cpu(pp):
    """BASELINE configs 4-5 as real pp-stage pipelines (--pp), gloo ranks on CPU."""
    r = _torchrun(pp, BENCH[:-2] + ["--gpus", str(pp), "--pp", str(pp), "--model", "tiny-qwen2"]
                  if pp <= 4 else ["bench.py", "--model", "byte-qwen2", "--batch", "1", "--microbatches", "2",
                                   "--steps", "1", "--warmup", "1", "--max-length", "64", "--gpus", "8", "--pp", "8"],
                  timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["config"]["parallelism"] == f"pp{pp}xdp1" and len(d["config"]["stage_layers"]) == pp
    assert len(d["wire_bytes_per_token"]) == pp - 1 and len(d["stages"]) == pp


def test_bench_eight_ranks_reports_pp8_cpu():
    """The driver's default 8-GPU run (pp2 x dp4 headline) also times one 8-stage pipeline (BASELINE config 5's
    shape) and reports it beside the headline."""
    r = _torchrun(8, ["bench.py", "--model", "byte-qwen2", "--batch", "1", "--steps", "2", "--warmup", "1",
                      "--max-length", "64", "--split", "3", "--gpus", "8"], timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["config"]["parallelism"] == "pp2xdp4" and d["n_gpus"] == 8
    _check_deep(d, 8)


def test_pipeline_entry_distributed_equals_local(tmp_path):
    cfg = {"model": "tiny-qwen2", "num_stages": 2, "codec": "mixed_int4_int8", "methods": ["last_row"],
           "ratios": [0, 0.5], "max_length": 128, "stride": 32, "window_batch": 3, "dataset": "synthetic",
           "synthetic_tokens": 1200, "device": "cpu", "resume": False}
    res = {}
    for n in (1, 2):
        d = tmp_path / f"n{n}"
        d.mkdir()
        (d / "params.json").write_text(json.dumps(dict(cfg, output_dir=str(d))))
        main = os.path.join(ROOT, "Experiments", "Pipeline", "main.py")
        if n == 1:
            r = subprocess.run([sys.executable, main], cwd=d, env=_env(), capture_output=True, text=True, timeout=600)
        else:
            r = _torchrun(2, [main], cwd=d)
        assert r.returncode == 0, r.stderr[-3000:]
        res[n] = json.loads((d / "pipeline_results.json").read_text())
    for r in ("0", "0.5"):
        a, b = res[1]["results"]["last_row"][r], res[2]["results"]["last_row"][r]
        assert abs(a["ppl"] - b["ppl"]) / a["ppl"] < 1e-6
        assert a["wire_bytes_per_token"] == pytest.approx(b["wire_bytes_per_token"], rel=1e-6)
    assert res[1]["results"]["last_row"]["0.5"]["wire_bytes_per_token"] < \
        res[1]["results"]["last_row"]["0"]["wire_bytes_per_token"]


def test_baseline_config_files_load():
    from llm_inference_in_distributed_edge_networks_amd.config import Params
    from llm_inference_in_distributed_edge_networks_amd.codec import get_codec
    d = os.path.join(ROOT, "Experiments", "Pipeline", "configs")
    names = sorted(os.listdir(d))
    assert len(names) == 5
    for n in names:
        p = Params.load(os.path.join(d, n))
        get_codec(p.codec)
        assert p.num_stages > 1 or p.split_layers


def test_bench_self_launch_equals_local():
    """``python bench.py --gpus 4`` without a launcher starts the 4 ranks itself (pp2 x dp2 over gloo here) and
    reports them; its PPL equals the single-process run over the same windows (--microbatches doubled at N=1:
    both process batches 0..2m-1 of the pool per step)."""
    base = BENCH[:4] + BENCH[6:]          # without "--microbatches 2"
    r4 = subprocess.run([sys.executable] + base + ["--microbatches", "2", "--gpus", "4", "--pp", "2"], cwd=ROOT,
                        env=_env(), capture_output=True, text=True, timeout=600)
    assert r4.returncode == 0, r4.stderr[-3000:]
    d4 = _json_line(r4.stdout)
    assert d4["n_gpus"] == 4 and d4["world_size"] == 4 and d4["launch"] == "self" and d4["backend"] == "gloo"
    assert [x["rank"] for x in d4["rank_devices"]] == [0, 1, 2, 3]
    assert d4["config"]["parallelism"] == "pp2xdp2"
    r1 = subprocess.run([sys.executable] + base + ["--microbatches", "4", "--gpus", "1"], cwd=ROOT, env=_env(),
                        capture_output=True, text=True, timeout=600)
    assert r1.returncode == 0, r1.stderr[-3000:]
    d1 = _json_line(r1.stdout)
    assert d1["launch"] == "single" and d1["config"]["global_batch"] == d4["config"]["global_batch"]
    assert d4["ppl_random_weights"] == pytest.approx(d1["ppl_random_weights"], rel=1e-9)


def test_bench_refuses_gpus_world_size_mismatch():
    r = _torchrun(2, BENCH + ["--gpus", "4"])
    assert r.returncode != 0
    assert "--gpus 4 but the launcher started WORLD_SIZE=2" in r.stderr


@pytest.mark.parametrize("rank", [1, 0])
def test_bench_failed_rank_exits_nonzero_without_json(rank):
    """A rank that dies (here on purpose, after its measurement) must leave the self-launching parent with a
    non-zero exit code and NO JSON line: rank 0 reports only after every rank passed the final barrier."""
    env = dict(_env(), EDGE_BENCH_FAIL_RANK=str(rank), EDGE_TUNING="1")   # a tuning-mode-only test hook
    r = subprocess.run([sys.executable] + BENCH + ["--gpus", "2"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode != 0
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")], r.stdout
    assert "fails on purpose" in r.stderr


def test_visible_gpu_count_without_hip(monkeypatch):
    """The launcher parent counts GPUs from sysfs / the visibility variables, never through the HIP runtime."""
    sys.path.insert(0, ROOT)
    import bench
    for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    base = bench.visible_gpu_count()          # 0 here (no KFD topology), the GPU count on a GPU box
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1,2")
    assert bench.visible_gpu_count() == (min(base, 3) if base else 3)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert bench.visible_gpu_count() == 0
    src = open(os.path.join(ROOT, "bench.py")).read()
    launch = src[src.index("def launch_mode"):src.index("def self_launch")]
    assert "torch.cuda" not in launch


@pytest.mark.parametrize("hook,rc", [("EDGE_BENCH_FAIL_SECONDARY=transports.torch:*", 0),
                                     ("EDGE_BENCH_HANG_SECONDARY=transports.torch:1", 0)])
def test_bench_secondary_failure_keeps_headline(hook, rc):
    """A secondary measurement that raises on every rank is recorded in its field and the run exits 0; one that hangs
    on one rank (its peers then wait in a collective) ends through the watchdog: the JSON line still carries the
    headline with the hung measurement marked, and every rank exits (bench.Guard)."""
    k, v = hook.split("=")
    env = dict(_env(), EDGE_TUNING="1", **{k: v})
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port())] + BENCH +
                       ["--gpus", "2", "--deep-pp-timeout", "10"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == rc, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["value"] > 0 and d["ppl_random_weights"] > 1
    assert "error" in d["transports"]["torch"]
    if "FAIL" in k:
        assert "fails transports.torch on purpose" in d["transports"]["torch"]["error"]
        assert "skipped" in d["transports"]["rccl"]
    else:
        assert "still running after 10 s" in d["transports"]["torch"]["error"]
