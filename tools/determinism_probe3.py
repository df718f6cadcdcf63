"""Sweep engine vs split runner on GPU, per entry and per batch."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_inference_in_distributed_edge_networks_amd import codec as C  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.data import synthetic_stream  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.sweep import SweepConfig, SweepEngine  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.windows import batches, sliding_windows  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.models import TINY_QWEN2, DecoderLM  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.parallel import BoundaryConfig, LocalPipeline, PipelinePlan  # noqa: E402

m = DecoderLM.random_init(TINY_QWEN2, 0, device="cuda", dtype=torch.bfloat16, std=0.05)
toks = synthetic_stream(3000, 512, 4)
bl = [b.to("cuda") for b in batches(toks, sliding_windows(3000, 256, 32), 4)]
sc = SweepConfig(["regular_importance", "last_row"], [1, 2], [0, 0.5, 1.0], codec="mixed_int4_int8")
eng = SweepEngine(m, sc)
for bi, b in enumerate(bl):
    out = eng.run_batch(b)
    for mi, meth in enumerate(sc.methods):
        for li, L in enumerate(sc.layers):
            for ri, r in enumerate(sc.ratios):
                p = LocalPipeline(m, PipelinePlan.from_split_layers(4, [L]), BoundaryConfig("mixed_int4_int8", r, meth),
                                  use_graphs=False)
                wn = p.run_batch(b)
                if not torch.equal(wn, out[mi, li, ri]):
                    print(f"batch{bi} B={b.B} S={b.S} {meth} L={L} r={r} maxdiff={(wn-out[mi,li,ri]).abs().max().item():.3g}")
# deeper: batch 1, regular L=1 r=0.5: compare boundary tensors
b = bl[1]
x = m.embed(b.ids)
x1, st1 = m.layer(0, x, b.B, b.S)
x1, st = m.layer(1, x1, b.B, b.S, stats="colsum")
x1b, stb = m.layer(1, m.layer(0, x, b.B, b.S)[0], b.B, b.S, stats=("colsum", "lastrow"))
print("x equal", torch.equal(x1, x1b), "colsum equal", torch.equal(st.colsum, stb.colsum))
