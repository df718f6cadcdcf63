"""Measured error of the bf16 HIP relevance engine against the fp32 CPU engine (== the autograd oracle), on the
tiny configs of tests/test_lrp_gpu.py::test_relevance_engine_gpu_vs_cpu, so that its tolerance pins what is measured.
Prints one JSON line per config."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from llm_inference_in_distributed_edge_networks_amd.models import DecoderLM  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.models.configs import TINY_NEOX, TINY_QWEN2  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.relevance.engine import RelevanceEngine  # noqa: E402


def rel_err(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def main():
    dev = torch.device("cuda:0")
    for cfg in (TINY_QWEN2, TINY_NEOX):
        for seed in (2, 3, 4):
            mg = DecoderLM.random_init(cfg, 3, device=dev, dtype=torch.bfloat16, std=0.05)
            mc = DecoderLM.random_init(cfg, 3, std=0.05)
            for Lg, Lc in zip(mg.layers, mc.layers):
                for kk in Lc:
                    Lc[kk] = Lg[kk].float().cpu() if kk in Lg else Lc[kk]
            for kk in ("embed", "head", "norm_w", "norm_b"):
                if mc.w.get(kk) is not None:
                    mc.w[kk] = mg.w[kk].float().cpu()
            mc.layers = mc.w["layers"]
            ids = torch.randint(0, cfg.vocab_size, (4, 128), generator=torch.Generator().manual_seed(seed))
            rg, _, mxg = RelevanceEngine(mg).head_relevance(ids.to(dev))
            rc, _, mxc = RelevanceEngine(mc).head_relevance(ids)
            wg, wc = rg.sum(0), rc.sum(0)
            print(json.dumps({"cfg": cfg.name, "seed": seed, "max_rel": rel_err(mxg, mxc), "rel": rel_err(rg, rc),
                              "table": rel_err(wg / wg.sum(-1, keepdim=True), wc / wc.sum(-1, keepdim=True))}),
                  flush=True)


if __name__ == "__main__":
    main()
