"""Run every op twice on identical inputs and report any bitwise difference (race / atomics detector)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_inference_in_distributed_edge_networks_amd import codec as C  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd import ops  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.data import synthetic_stream  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.windows import batches, sliding_windows, window_nll  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.models import TINY_QWEN2, QWEN2_0_5B, DecoderLM  # noqa: E402


def same(name, f, reps=5):
    outs = [f() for _ in range(reps)]
    outs = [o if isinstance(o, tuple) else (o,) for o in outs]
    bad = []
    for i, t in enumerate(outs[0]):
        if t is None:
            continue
        for o in outs[1:]:
            if not torch.equal(o[i], t):
                d = (o[i].float() - t.float()).abs().max().item()
                bad.append(f"out{i} maxdiff={d:.3g}")
                break
    print(f"{'OK ' if not bad else 'BAD'} {name} {' '.join(bad)}", flush=True)


def main():
    dev = "cuda"
    for cfg, B, S in ((TINY_QWEN2, 4, 256), (QWEN2_0_5B.replace(num_layers=2), 8, 512)):
        m = DecoderLM.random_init(cfg, 0, device=dev, dtype=torch.bfloat16, std=0.05)
        toks = synthetic_stream(8000, cfg.vocab_size, 1)
        b = next(batches(toks, sliding_windows(8000, S, 32)[1:], B)).to(dev)
        L = m.layers[0]
        x = m.embed(b.ids)
        print(f"== {cfg.name} B={B} S={S} M={x.shape[0]}")
        same("embed", lambda: m.embed(b.ids))
        same("rmsnorm", lambda: ops.rmsnorm(x, L["ln1_w"], 1e-6))
        h = ops.rmsnorm(x, L["ln1_w"], 1e-6)
        same("qkv_rope", lambda: ops.qkv_rope(h, L["wqkv"], L["bqkv"], m.cos, m.sin, B, S, cfg.num_heads,
                                               cfg.num_kv_heads, 64, cfg.rotary_dim, m.q_scale))
        q, k, vt = ops.qkv_rope(h, L["wqkv"], L["bqkv"], m.cos, m.sin, B, S, cfg.num_heads, cfg.num_kv_heads, 64,
                                cfg.rotary_dim, m.q_scale)
        same("attention", lambda: ops.attention(q, k, vt, S, True))
        o, lse = ops.attention(q, k, vt, S, True)
        same("lastrow", lambda: ops.attn_lastrow(q, k, S))
        same("colsum", lambda: ops.attn_colsum(q, k, lse, S))
        same("o_proj+resid", lambda: ops.linear(o, L["wo"], residual=x))
        y = ops.linear(o, L["wo"], residual=x)
        same("gate_up", lambda: ops.linear(h, L["wgu"], act="swiglu_il"))
        a = ops.linear(h, L["wgu"], act="swiglu_il")
        same("down", lambda: ops.linear(a, L["wd"], residual=y))
        same("layer", lambda: m.layer(0, x, B, S)[0])
        imp = torch.rand(B, S, device=dev)
        for name in C.CODECS:
            same(f"codec {name}", lambda: C.encode(x, C.get_codec(name), B, S, 0.5, imp)[0])
        xs = m.forward_hidden(b.ids)
        same("head_nll", lambda: m.row_nll(xs, b.rows, b.targets))
        nll = m.row_nll(xs, b.rows, b.targets)
        same("window_nll(index_add)", lambda: window_nll(nll, b))


if __name__ == "__main__":
    main()
