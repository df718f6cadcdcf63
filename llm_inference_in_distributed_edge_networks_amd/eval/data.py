"""Token streams: WikiText-2 (when available offline) or a deterministic synthetic stream.

Reference: ``load_dataset("Salesforce/wikitext", "wikitext-2-raw-v1", split="test")`` then
``tokenizer("\\n\\n".join(test["text"]))`` (``Experiments/Pythia-70M/last_row_exp.py:49-55``,
``Experiments/Qwen2-0.5B/main.py:122-124``).  This machine has no network, so the
loader only uses local HF caches and otherwise returns a seeded synthetic stream
of the WikiText-2 test length (299,078 Qwen2 tokens,
``Notebooks/qwen2-0.5B_experiment.ipynb`` JSON line 156) - plumbing and
throughput only, never a PPL claim.
"""
from __future__ import annotations

import os

import torch

WIKITEXT2_TEST_TOKENS = 299_078


def synthetic_stream(num_tokens: int, vocab_size: int, seed: int = 0) -> torch.Tensor:
    """Deterministic token ids [1, N] (Zipf-like so the stream is not uniform noise)."""
    g = torch.Generator().manual_seed(seed)
    ranks = torch.arange(1, vocab_size + 1, dtype=torch.float64)
    probs = (1.0 / ranks ** 1.1)
    probs /= probs.sum()
    ids = torch.multinomial(probs.float(), num_tokens, replacement=True, generator=g)
    perm = torch.randperm(vocab_size, generator=g)
    return perm[ids].view(1, -1).to(torch.int64)


def load_wikitext_tokens(hf_id: str, split: str = "test") -> torch.Tensor | None:
    """WikiText-2 raw tokenized with the model's tokenizer, from local caches only (None if absent)."""
    if not hf_id:
        return None
    os.environ.setdefault("HF_HUB_OFFLINE", "1")
    os.environ.setdefault("HF_DATASETS_OFFLINE", "1")
    try:
        from datasets import load_dataset
        from transformers import AutoTokenizer
        tok = AutoTokenizer.from_pretrained(hf_id, local_files_only=True)
        ds = load_dataset("Salesforce/wikitext", "wikitext-2-raw-v1", split=split)
    except Exception:
        return None
    enc = tok("\n\n".join(ds["text"]), return_tensors="pt")
    return enc.input_ids.to(torch.int64)


def token_stream(dataset: str, hf_id: str, vocab_size: int, synthetic_tokens: int = 0, seed: int = 0):
    """Returns (ids [1, N], provenance)."""
    if dataset == "wikitext":
        ids = load_wikitext_tokens(hf_id)
        if ids is not None:
            return ids, "wikitext-2-raw-v1/test"
    n = synthetic_tokens or WIKITEXT2_TEST_TOKENS
    return synthetic_stream(n, vocab_size, seed), f"synthetic(n={n},seed={seed})"
