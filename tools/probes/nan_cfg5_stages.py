"""Debug probe: config 5 at ratio 1 with one HIP graph per stage (as DistributedPipeline) vs eager, batch by batch:
the first stage whose graph-replayed output differs from the eager one."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from llm_inference_in_distributed_edge_networks_amd import codec as C  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.data import synthetic_stream  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.windows import batches, sliding_windows  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.models import get_config, DecoderLM  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.parallel import BoundaryConfig, PipelinePlan  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.parallel.pipeline import StageRunner  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.utils.graphs import GraphCache  # noqa: E402

cfg = get_config("qwen2-0.5b")
dev = "cuda"
m = DecoderLM.random_init(cfg, 0, device=dev)
toks = synthetic_stream(299078, cfg.vocab_size, 0)
wins = [w for w in sliding_windows(toks.shape[1], 512, 32)][:int(os.environ.get("NW", "2048"))]
here = os.path.dirname(os.path.abspath(__file__))
grel = json.load(open(os.path.join(here, "cfg5_group_relevance.json")))
hw = torch.tensor(json.load(open(os.path.join(here, "cfg5_head_weights.json"))))
plan = PipelinePlan.balanced(cfg, 8, 512)
bc = BoundaryConfig("mixed_rgroup_int8", float(os.environ.get("RATIO", "1.0")), "weighted_importance", hw,
                    group_relevance=grel, group_avg_bits=4)
stages = [StageRunner(m, plan, s, bc) for s in range(8)]
graphs = [GraphCache(st.forward) for st in stages]
first_bad = None
for bi, b in enumerate(batches(toks, wins, 32)):
    b = b.to(dev)
    args = (b.ids, b.rows, b.targets, b.row_window, b.n_rows)
    msg_e = carry_e = msg_g = None
    for si, st in enumerate(stages):
        ins_e = args if st.first else args + (msg_e, torch.empty(0, device=dev))
        out_e = st.forward(*ins_e)
        ins_g = args if st.first else args + (msg_g, torch.empty(0, device=dev))
        out_g = graphs[si](*ins_g)
        if st.last:
            same = torch.equal(out_e, out_g)
            if not same or not torch.isfinite(out_g).all():
                print(f"batch {bi} last stage: eager finite {bool(torch.isfinite(out_e).all())}, graph finite "
                      f"{bool(torch.isfinite(out_g).all())}, equal {same}")
                first_bad = first_bad or bi
            break
        msg_e, msg_g = out_e[0], out_g[0]
        if not torch.equal(msg_e, msg_g):
            d = (msg_e != msg_g).nonzero().flatten()
            L = st.layout(b)
            print(f"batch {bi} stage {si}: messages differ at {d.numel()} bytes, first {d[:8].tolist()}, layout "
                  f"off_lo {L.off_lo} total {L.total}")
            xe = C.decode(msg_e, st.spec_out, L, torch.float32)
            xg = C.decode(msg_g, st.spec_out, L, torch.float32)
            print("   decoded finite eager / graph", bool(torch.isfinite(xe).all()), bool(torch.isfinite(xg).all()))
            first_bad = first_bad or bi
            msg_g = msg_g.clone()
    if first_bad is not None and bi > first_bad + 1:
        break
print("done, batches", bi + 1, "first bad", first_bad)
