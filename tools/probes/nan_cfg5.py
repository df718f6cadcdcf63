"""Debug probe: config-5 (8 stages, mixed_rgroup_int8, LRP-weighted) at ratio 1 on the GPU - locate non-finite values."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from llm_inference_in_distributed_edge_networks_amd import codec as C  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.data import synthetic_stream  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.windows import batches, sliding_windows  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.models import DecoderLM, get_config  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.parallel import BoundaryConfig, LocalPipeline, PipelinePlan  # noqa

cfg = get_config("qwen2-0.5b")
dev = "cuda"
m = DecoderLM.random_init(cfg, 0, device=dev)
toks = synthetic_stream(299078, cfg.vocab_size, 0)
NW = int(os.environ.get("NW", "2048"))
wins = [w for w in sliding_windows(toks.shape[1], 512, 32)][:NW]
here = os.path.dirname(os.path.abspath(__file__))
grel = json.load(open(os.path.join(here, "cfg5_group_relevance.json")))
hw = torch.tensor(json.load(open(os.path.join(here, "cfg5_head_weights.json"))))
plan = PipelinePlan.balanced(cfg, 8, 512)
bc = BoundaryConfig("mixed_rgroup_int8", 1.0, "weighted_importance", hw, group_relevance=grel, group_avg_bits=4)
pipe = LocalPipeline(m, plan, bc, use_graphs=False)
gpipe = LocalPipeline(m, plan, bc, use_graphs=True)
bad = 0
for bi, b in enumerate(batches(toks, wins, 32)):
    b = b.to(dev)
    msg = carry = None
    for st in pipe.stages:
        if not st.first:
            x_in = C.decode(msg, st.spec_in, st.layout_in(b), torch.float32)
            if not torch.isfinite(x_in).all():
                print("batch", bi, "stage", st.stage, "decoded input non-finite:", int((~torch.isfinite(x_in)).sum()))
                bad += 1
        out = st.forward(b.ids, b.rows, b.targets, b.row_window, b.n_rows, msg, carry)
        if st.last:
            if not torch.isfinite(out).all():
                print("batch", bi, "window nll non-finite", out.tolist())
                bad += 1
            break
        msg, carry = out
        # same x through the CPU codec: identical message?
    wg = gpipe.run_batch(b)
    if not torch.isfinite(wg).all():
        print("batch", bi, "graph-replayed window nll non-finite", wg.tolist())
        bad += 1
    if bad:
        break
print("batches checked", bi + 1, "bad", bad)
