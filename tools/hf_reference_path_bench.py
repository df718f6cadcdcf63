"""Same-node baseline: the reference's computation, written on stock HF transformers + PyTorch eager, on this GPU.

BASELINE.md's numbers are from a T4.  To compare against the reference's *implementation strategy* on the same
MI355X, this runs what the reference does per 512-token window (``/root/reference/Experiments/Qwen2-0.5B/main.py:
151-180``: one HF forward with ``output_attentions=True`` for the importance maps; then, per configuration, a
layer-by-layer HF forward that quantizes the ``ratio`` least important tokens of the boundary layer with one global
int4 scale, ``qwen_layer_wise.py:41-76``; shifted CE with the sliding-window targets) with HF Qwen2 modules of the
Qwen2-0.5B shape (random init, fp32, no download).  The code here is written for this harness from that description,
not taken from the reference.

``--configs 1`` is the work of one evaluated configuration (what ``bench.py`` does per window: config 3, column-mean
importance at layer 11, ratio 0.5); ``--configs 100`` is the reference's notebook sweep (4 methods x 5 layers x 5
ratios per window).  ``--batch 1`` is the reference's loop (one window per call); ``--batch 64`` the same work batched,
the best plain PyTorch eager can do with it.  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from llm_inference_in_distributed_edge_networks_amd.eval.data import synthetic_stream  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.eval.windows import batches, sliding_windows  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.models import get_config  # noqa: E402


def hf_model(cfg, attn: str, dev, seed=0):
    from transformers import Qwen2Config, Qwen2ForCausalLM
    hc = Qwen2Config(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
                     num_hidden_layers=cfg.num_layers, num_attention_heads=cfg.num_heads,
                     num_key_value_heads=cfg.num_kv_heads, max_position_embeddings=cfg.max_position,
                     rope_theta=cfg.rope_theta, tie_word_embeddings=cfg.tie_embeddings, rms_norm_eps=cfg.norm_eps,
                     attn_implementation=attn)
    torch.manual_seed(seed)
    return Qwen2ForCausalLM(hc).to(dev).eval()


def column_mean_importance(att: torch.Tensor) -> torch.Tensor:
    """[B, H, S, S] attention probabilities -> [B, S]: mean over heads, then over query rows."""
    return att.mean(dim=1).mean(dim=1)


def int4_global_lowest(h: torch.Tensor, imp: torch.Tensor, ratio: float) -> torch.Tensor:
    """The reference's Q1 per window: the k = int(ratio S) lowest-importance tokens to symmetric int4 with one max-abs
    scale over all of them (levels -8..7, scale max / 7)."""
    B, S, H = h.shape
    k = int(ratio * S)
    if k == 0:
        return h
    pos = torch.argsort(imp, dim=1)[:, :k]                              # [B, k]
    idx = pos[..., None].expand(B, k, H)
    sel = torch.gather(h, 1, idx)
    mx = sel.abs().amax(dim=(1, 2), keepdim=True)
    q = torch.round(torch.clamp(sel / mx * 7.0, -8.0, 7.0)) / 7.0 * mx
    return h.scatter(1, idx, q)


def split_forward_nll(m, ids, targets_mask, layer: int, imp, ratio: float):
    """Layer-by-layer forward with the boundary after ``layer`` quantized; mean NLL over the scored targets."""
    core = m.model
    h = core.embed_tokens(ids)
    pos = torch.arange(ids.shape[1], device=ids.device)[None].expand(ids.shape[0], -1)
    pe = core.rotary_emb(h, pos)
    for i, lyr in enumerate(core.layers):
        out = lyr(h, position_embeddings=pe)
        h = out[0] if isinstance(out, tuple) else out
        if i == layer and ratio > 0:
            h = int4_global_lowest(h, imp, ratio)
    logits = m.lm_head(core.norm(h))[:, :-1]
    tgt = torch.where(targets_mask[:, 1:], ids[:, 1:], torch.full_like(ids[:, 1:], -100))
    return torch.nn.functional.cross_entropy(logits.reshape(-1, logits.shape[-1]), tgt.reshape(-1),
                                             ignore_index=-100, reduction="sum")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen2-0.5b")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--windows", type=int, default=32, help="timed windows")
    ap.add_argument("--warmup", type=int, default=2, help="untimed batches")
    ap.add_argument("--configs", type=int, default=1, help="quantized forwards per window (1 = bench, 100 = sweep)")
    ap.add_argument("--layer", type=int, default=11)
    ap.add_argument("--ratio", type=float, default=0.5)
    a = ap.parse_args()
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    cfg = get_config(a.model)
    eager = hf_model(cfg, "eager", dev)            # output_attentions needs the eager attention
    split = hf_model(cfg, "sdpa", dev)             # the reference's layer-wise model uses sdpa
    split.load_state_dict(eager.state_dict())
    toks = synthetic_stream(299_078, cfg.vocab_size, 0)
    wins = sliding_windows(toks.numel(), 512, 32)
    need = (a.warmup * a.batch + a.windows)
    bl = list(batches(toks, wins[:need], a.batch))
    layers = [22, 18, 3, 23, 11]
    ratios = [0, 0.25, 0.5, 0.75, 1.0]

    def run(b):
        ids = b.ids.to(dev)
        S = ids.shape[1]
        first = torch.tensor([w.first_scored for w in b.windows], device=dev)
        tmask = torch.arange(S, device=dev)[None] >= first[:, None] + 1   # token p+1 is scored from row p
        with torch.no_grad():
            att = eager(input_ids=ids, output_attentions=True).attentions
            nll = []
            for c in range(a.configs):
                if a.configs == 1:
                    L, r = a.layer, a.ratio
                else:
                    L, r = layers[(c // 5) % 5] % cfg.num_layers, ratios[c % 5]
                imp = column_mean_importance(att[L])
                nll.append(split_forward_nll(split, ids, tmask, L, imp, r))
            del att
            return torch.stack(nll)

    for b in bl[:a.warmup]:
        run(b)
    torch.cuda.synchronize() if dev == "cuda" else None
    t0 = time.perf_counter()
    n = 0
    for b in bl[a.warmup:]:
        run(b)
        n += b.B
    torch.cuda.synchronize() if dev == "cuda" else None
    dt = time.perf_counter() - t0
    print(json.dumps({"what": "reference computation on HF transformers + PyTorch eager (fp32)", "device": dev,
                      "gpu": torch.cuda.get_device_name(0) if dev == "cuda" else "cpu",
                      "model": cfg.name, "batch": a.batch, "configs_per_window": a.configs, "windows": n,
                      "seconds": round(dt, 3), "s_per_window": round(dt / n, 5),
                      "window_tokens_per_s": round(n * 512 / dt, 1),
                      "forward_tokens_per_s": round(n * 512 * (1 + a.configs) / dt, 1),
                      "torch": torch.__version__}), flush=True)


if __name__ == "__main__":
    main()
