"""Window-bootstrap statistics of the quality experiments (eval/stats.py) and the sweep's kept per-window NLL."""
import math

import torch

from llm_inference_in_distributed_edge_networks_amd.eval import stats
from llm_inference_in_distributed_edge_networks_amd.eval.data import synthetic_stream
from llm_inference_in_distributed_edge_networks_amd.eval.sweep import SweepConfig, SweepEngine, run_sweep
from llm_inference_in_distributed_edge_networks_amd.eval.windows import batches, sliding_windows
from llm_inference_in_distributed_edge_networks_amd.models import TINY_QWEN2, DecoderLM


def _cells(n=400, seed=0):
    g = torch.Generator().manual_seed(seed)
    base = 2.0 + 0.3 * torch.randn(n, generator=g, dtype=torch.float64)
    w = torch.randint(1, 33, (n,), generator=g).double()
    return base, w


def test_point_estimate_is_token_weighted_log_ppl():
    base, w = _cells()
    nll = torch.stack([base, base + 0.1], 1)
    pt = stats.log_ppl(nll, w)
    assert torch.allclose(pt[0], (w * base).sum() / w.sum())
    assert torch.allclose(pt[1] - pt[0], torch.tensor(0.1, dtype=torch.float64))


def test_bootstrap_replicates_are_paired_and_centred():
    base, w = _cells()
    nll = torch.stack([base, base + 0.05 * torch.sin(base)], 1)
    bs = stats.bootstrap_log_ppl(nll, w, reps=2000, seed=3)
    assert bs.shape == (2000, 2)
    pt = stats.log_ppl(nll, w)
    assert torch.allclose(bs.mean(0), pt, atol=5e-3)             # centred on the point estimate
    # the same replicates for every cell: a constant shift is exactly constant on every replicate
    shifted = torch.stack([base, base + 0.2], 1)
    d = stats.bootstrap_log_ppl(shifted, w, reps=500, seed=3)
    assert torch.allclose(d[:, 1] - d[:, 0], torch.full((500,), 0.2, dtype=torch.float64))
    # and the same seed gives the same replicates
    assert torch.equal(stats.bootstrap_log_ppl(nll, w, reps=50, seed=9), stats.bootstrap_log_ppl(nll, w, reps=50, seed=9))


def test_paired_diff_verdicts():
    base, w = _cells()
    same = torch.stack([base, base], 1)
    r = stats.paired_diff(same, w, 0, 1)
    assert r["diff"] == 0 and r["ci"] == [0.0, 0.0] and r["verdict"] == "not resolved"
    worse = torch.stack([base + 0.01, base], 1)                   # a worse on every window
    r = stats.paired_diff(worse, w, 0, 1)
    assert r["verdict"] == "a worse" and math.isclose(r["diff"], 0.01, rel_tol=1e-9)
    assert r["ci"][0] <= 0.01 + 1e-12 and r["ci"][1] >= 0.01 - 1e-12
    better = torch.stack([base - 0.01, base], 1)
    assert stats.paired_diff(better, w, 0, 1)["verdict"] == "b worse"
    # pure noise around the same mean: the interval covers 0
    g = torch.Generator().manual_seed(5)
    noisy = torch.stack([base + 0.05 * torch.randn(base.numel(), generator=g, dtype=torch.float64), base], 1)
    r = stats.paired_diff(noisy - noisy[:, :1].mean() + base.mean(), w, 0, 1)
    assert r["ci"][0] < r["diff"] < r["ci"][1]


def test_damage_table_against_base_cell():
    base, w = _cells()
    nll = torch.stack([base, base + 0.02, base + 0.1], 1)
    tab = stats.damage_table(nll, w, base=0, reps=500)
    assert tab[0]["rel"] == 0 and tab[0]["ci"] == [0.0, 0.0]
    for c, dl in ((1, 0.02), (2, 0.1)):
        assert math.isclose(tab[c]["rel"], math.expm1(dl), rel_tol=1e-9)
        assert math.isclose(tab[c]["ci"][0], math.expm1(dl), rel_tol=1e-6)   # a constant shift: zero-width interval
        assert math.isclose(tab[c]["ppl"], math.exp(float(stats.log_ppl(nll, w)[c])), rel_tol=1e-12)


def test_sweep_keeps_per_window_nll_consistent_with_its_ppl():
    """SweepEngine(keep_windows=True): the per-window NLL and weights reproduce the engine's own PPL table."""
    m = DecoderLM.random_init(TINY_QWEN2, 0, std=0.06)
    tok = synthetic_stream(900, 512, 1)
    wins = sliding_windows(900, 128, 32)
    sc = SweepConfig(["last_row", "regular_importance"], [1, 2], [0, 0.5, 1], codec="ref_int4_global")
    eng = SweepEngine(m, sc, keep_windows=True)
    res = run_sweep(eng, batches(tok, wins, 3))
    nll, w = eng.window_results()
    assert nll.shape == (len(wins), 2, 2, 3) and w.shape == (len(wins),)
    pt = stats.log_ppl(nll.reshape(len(wins), -1), w).reshape(2, 2, 3).exp()
    assert torch.allclose(pt, torch.tensor(res["avg_ppl_results"], dtype=torch.float64), rtol=1e-5)
