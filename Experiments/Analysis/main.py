"""Layer-divergence analysis (reference: Notebooks/distributions_distance_across_layers.ipynb).

Reads ``./params.json`` (``model``, ``min_chars`` = 125, ``max_lines``, ``dataset``) and writes
``js_divergence.json``: the layers x layers Jensen-Shannon divergence (log2) between per-layer
column-mean attention importance, averaged over WikiText-2 test lines with >= min_chars characters
(synthetic token lines when WikiText/tokenizer are not available offline).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from llm_inference_in_distributed_edge_networks_amd.config import Params, dump_json, resolve_device, resolve_dtype  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.analysis import js_matrix  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.data import synthetic_stream  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.models import build_model, get_config  # noqa: E402


def lines(cfg, dataset, max_lines, seed):
    if dataset == "wikitext":
        try:
            os.environ.setdefault("HF_HUB_OFFLINE", "1")
            os.environ.setdefault("HF_DATASETS_OFFLINE", "1")
            from datasets import load_dataset
            from transformers import AutoTokenizer
            tok = AutoTokenizer.from_pretrained(cfg.hf_id, local_files_only=True)
            ds = load_dataset("Salesforce/wikitext", "wikitext-2-raw-v1", split="test")
            texts = [t for t in ds["text"]][: max_lines * 4]
            seqs = [tok(t, return_tensors="pt").input_ids for t in texts]
            return seqs, texts, "wikitext-2-raw-v1/test"
        except Exception:
            pass
    g = torch.Generator().manual_seed(seed)
    lens = torch.randint(30, 200, (max_lines,), generator=g).tolist()
    seqs = [synthetic_stream(n, cfg.vocab_size, seed + i) for i, n in enumerate(lens)]
    return seqs, ["x" * 200] * len(seqs), "synthetic"


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", default="params.json")
    ap.add_argument("--device", default=None)
    a = ap.parse_args()
    p = Params.load(a.params, device=a.device)
    cfg = get_config(p.model or "pythia-70m")
    dev = resolve_device(p)
    model, prov = build_model(cfg, dev, resolve_dtype(p, dev), weights=p.weights, seed=p.seed)
    seqs, texts, src = lines(cfg, p.dataset, int(p.extra.get("max_lines", 200)), p.seed)
    mat = js_matrix(model, seqs, int(p.extra.get("min_chars", 125)), texts)
    out = {"model": cfg.name, "weights": prov, "data": src, "js_divergence": mat.tolist()}
    dump_json(out, os.path.join(p.output_dir, "js_divergence.json"))
    print(json.dumps({"data": src, "js(0,last)": mat[0, -1].item()}))
