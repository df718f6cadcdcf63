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
LAST_EXCLUDED = 0   # extra train-large files dropped as copies of held-out (eval) files by the last local_text_bytes


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


def local_text_bytes(split: str = "eval", root: str = "", max_bytes: int = 256 << 20) -> torch.Tensor:
    """Byte ids [1, N] of real local text: the Python standard-library sources of this image, sorted by path;
    every 10th file is the held-out ``eval`` split, the rest ``train``.  Used with the byte-level model
    (``byte-qwen2``) for quality experiments, since no pretrained checkpoint or WikiText copy is reachable.
    ``train-large``: the ``train`` files plus the Python sources of the installed packages (dist-/site-packages,
    files under 200 KB, sorted by path, up to ``max_bytes``): ~25x the text, so a few minutes of training never
    revisit a byte and the model does not overfit the 10 MB stdlib split; returned as uint8 [1, N] (cast per batch)."""
    import glob
    import sys
    root = root or os.path.join(sys.base_prefix, "lib", f"python{sys.version_info.major}.{sys.version_info.minor}")
    files = sorted(glob.glob(os.path.join(root, "**", "*.py"), recursive=True))
    files = [f for f in files if "site-packages" not in f and "dist-packages" not in f]
    if not files:
        raise FileNotFoundError(f"no python sources under {root}")
    pick = [f for i, f in enumerate(files) if (i % 10 == 0) == (split == "eval")]
    if split == "train-large":
        import hashlib
        import site
        global LAST_EXCLUDED
        roots = [d for d in {*site.getsitepackages(), os.path.join(root, "site-packages")} if os.path.isdir(d)]
        extra = sorted({f for d in roots for f in glob.glob(os.path.join(d, "**", "*.py"), recursive=True)})
        extra = [f for f in extra if os.path.getsize(f) < 200_000]
        # packages vendor copies of stdlib modules (setuptools/_distutils, pip/_vendor, backports): drop every extra
        # file whose content equals a held-out (eval) file, or whose path ends in an eval file's stdlib-relative path
        evf = [f for i, f in enumerate(files) if i % 10 == 0]

        def digest(f):
            try:
                with open(f, "rb") as fh:
                    return hashlib.sha1(fh.read()).hexdigest()
            except OSError:
                return None
        ev_hash = {digest(f) for f in evf} - {None}
        ev_tail = {os.path.relpath(f, root) for f in evf}

        def tails(f):   # every path suffix of f made of whole components
            parts = f.split(os.sep)
            return {os.sep.join(parts[i:]) for i in range(1, len(parts))}
        keep = [f for f in extra if digest(f) not in ev_hash and not (tails(f) & ev_tail)]
        LAST_EXCLUDED = len(extra) - len(keep)
        pick += keep
    buf = bytearray()
    for f in pick:
        if len(buf) >= max_bytes:
            break
        try:
            with open(f, "rb") as fh:
                buf += fh.read()
        except OSError:
            continue
        buf += b"\n\n"
    t = torch.frombuffer(buf, dtype=torch.uint8).view(1, -1)
    return t.clone() if split == "train-large" else t.to(torch.int64)


class DatasetUnavailable(FileNotFoundError):
    pass


def token_stream(dataset: str, hf_id: str, vocab_size: int, synthetic_tokens: int = 0, seed: int = 0,
                 strict: bool = False):
    """Returns (ids [1, N], provenance).  ``dataset="wikitext"`` without a local cache falls back to the synthetic
    stream with a loud warning (``strict``: raises instead); ``dataset="synthetic"`` asks for it explicitly."""
    if dataset in ("pysrc", "pysrc-eval", "pysrc-train"):
        split = "train" if dataset == "pysrc-train" else "eval"
        ids = local_text_bytes(split)
        if synthetic_tokens:
            ids = ids[:, :synthetic_tokens]
        return ids, f"python-stdlib-bytes/{split}(n={ids.shape[1]})"
    if dataset == "wikitext":
        ids = load_wikitext_tokens(hf_id)
        if ids is not None:
            return ids, "wikitext-2-raw-v1/test"
        msg = (f"WikiText-2 (or the {hf_id} tokenizer) is not available locally: the PPL below is on a SYNTHETIC "
               "token stream, not WikiText-2 (set dataset='synthetic' to ask for it, strict_data=true to fail)")
        if strict:
            raise DatasetUnavailable(msg)
        import warnings
        warnings.warn(msg, RuntimeWarning, stacklevel=2)
        print(f"WARNING: {msg}", flush=True)
    elif dataset != "synthetic":
        raise ValueError(f"unknown dataset {dataset!r} (wikitext | synthetic | pysrc | pysrc-eval | pysrc-train)")
    n = synthetic_tokens or WIKITEXT2_TEST_TOKENS
    return synthetic_stream(n, vocab_size, seed), f"synthetic(n={n},seed={seed})"
