"""Pipeline-level repeatability over all batches of a corpus (incl. the short last window)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_inference_in_distributed_edge_networks_amd import ops  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.data import synthetic_stream  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.windows import batches, sliding_windows  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.models import TINY_QWEN2, DecoderLM  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.parallel import BoundaryConfig, LocalPipeline, PipelinePlan  # noqa: E402

m = DecoderLM.random_init(TINY_QWEN2, 1, device="cuda", dtype=torch.bfloat16, std=0.05)
toks = synthetic_stream(3000, 512, 4)
bl = [b.to("cuda") for b in batches(toks, sliding_windows(3000, 256, 32), 4)]
for codec, ratio, meth in [("passthrough", 0, "last_row"), ("mixed_int4_int8", 0.5, "regular_importance"),
                           ("ref_int4_global", 0.25, "last_row")]:
    p = LocalPipeline(m, PipelinePlan.from_split_layers(4, [1, 2]), BoundaryConfig(codec, ratio, meth), use_graphs=False)
    ref = [p.run_batch(b).clone() for b in bl]
    for rep in range(3):
        for i, b in enumerate(bl):
            o = p.run_batch(b)
            if not torch.equal(o, ref[i]):
                print(f"BAD {codec} rep{rep} batch{i} B={b.B} S={b.S} diff={(o-ref[i]).abs().max().item():.3g}", flush=True)
    print("done", codec, flush=True)
# op-level on the short batch
b = bl[-1]
print("last batch", b.B, b.S)
x = m.embed(b.ids)
for i in range(4):
    outs = [m.layer(i, x, b.B, b.S)[0] for _ in range(4)]
    print("layer", i, all(torch.equal(outs[0], o) for o in outs[1:]))
    L = m.layers[i]
    h = ops.rmsnorm(x, L["ln1_w"], 1e-6)
    qs = [ops.qkv_rope(h, L["wqkv"], L["bqkv"], m.cos, m.sin, b.B, b.S, 4, 2, 64, 64, m.q_scale) for _ in range(4)]
    for j, nm in enumerate("q k vt".split()):
        print("  ", nm, all(torch.equal(qs[0][j], q[j]) for q in qs[1:]))
    q, k, vt = qs[0]
    at = [ops.attention(q, k, vt, b.S, True) for _ in range(4)]
    print("   attn", all(torch.equal(at[0][0], a[0]) for a in at[1:]), all(torch.equal(at[0][1], a[1]) for a in at[1:]))
    x = outs[0]
