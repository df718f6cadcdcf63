"""Sliding-window PPL harness == the reference's HF loop (Experiments/Qwen2-0.5B/main.py:151-204)."""
import math

import pytest
import torch

from llm_inference_in_distributed_edge_networks_amd.eval.data import synthetic_stream
from llm_inference_in_distributed_edge_networks_amd.eval.windows import (PPLAccumulator, batches, make_batch,
                                                                         sliding_windows)
from llm_inference_in_distributed_edge_networks_amd.models import TINY_NEOX, TINY_QWEN2
from llm_inference_in_distributed_edge_networks_amd.parallel import BoundaryConfig, LocalPipeline, PipelinePlan

from helpers import hf_neox, hf_qwen2, ours_from_hf


def reference_loop(hf, ids, max_length, stride):
    """Verbatim semantics of the reference window loop with an HF model (B=1)."""
    total_nll, n_tokens, prev_end = 0.0, 0, 0
    N = ids.size(1)
    for begin in range(0, N, stride):
        end = min(begin + max_length, N)
        trg_len = end - prev_end
        inp = ids[:, begin:end]
        tgt = inp.clone()
        tgt[:, :-trg_len] = -100
        with torch.no_grad():
            logits = hf(inp).logits
        nll = torch.nn.functional.cross_entropy(logits[:, :-1].reshape(-1, logits.size(-1)), tgt[:, 1:].reshape(-1),
                                                ignore_index=-100)
        num_valid = (tgt != -100).sum().item()
        num_loss = num_valid - tgt.size(0)
        total_nll += nll.item() * num_loss
        n_tokens += num_loss
        prev_end = end
        if end == N:
            break
    return math.exp(total_nll / n_tokens)


def test_windows_enumeration():
    w = sliding_windows(1000, 512, 32)
    assert w[0].begin == 0 and w[0].trg_len == 512 and w[0].first_scored == 0
    assert all(x.trg_len == 32 for x in w[1:-1])
    assert w[-1].end == 1000 and w[-2].end < 1000
    assert w[1].first_scored == 512 - 33


@pytest.mark.parametrize("cfg,mk", [(TINY_QWEN2, hf_qwen2), (TINY_NEOX, hf_neox)])
@pytest.mark.parametrize("bs", [1, 5])
def test_ppl_matches_reference_loop(cfg, mk, bs):
    hf = mk(cfg)
    ours = ours_from_hf(cfg, hf)
    ids = synthetic_stream(700, cfg.vocab_size, 3)
    ref = reference_loop(hf, ids, 200, 32)
    pipe = LocalPipeline(ours, PipelinePlan.from_split_layers(cfg.num_layers, [1]), BoundaryConfig())
    acc = pipe.evaluate(batches(ids, sliding_windows(700, 200, 32), bs))
    assert abs(acc.ppl() - ref) / ref < 1e-5


def test_batch_rows_and_targets():
    ids = torch.arange(100).view(1, -1)
    wins = sliding_windows(100, 40, 16)
    b = make_batch(ids, wins[1:3])
    assert b.S == 40 and b.B == 2
    # window 1: begin 16, trg_len 16 -> rows 23..38 predict tokens 16+24..16+39
    r0 = b.rows[b.row_window == 0]
    assert r0.tolist() == list(range(23, 39))
    assert b.targets[b.row_window == 0].tolist() == list(range(40, 56))
