"""Same-node baseline: the reference's computation on stock HF transformers + PyTorch eager, on this device.

BASELINE.md's throughput is from a T4.  To compare against the reference's *implementation strategy* on the same
hardware, this runs what the reference does per 512-token window (``/root/reference/Experiments/Qwen2-0.5B/main.py:
151-180``: one HF forward with ``output_attentions=True`` for the importance maps; then, per configuration, a
layer-by-layer HF forward that quantizes the ``ratio`` least important tokens of the boundary layer with one global
int4 scale, ``qwen_layer_wise.py:41-76``; shifted CE with the sliding-window targets) with HF Qwen2 modules of the
model's shape (random init, fp32, no download).  Written for this framework from that description, not taken from
the reference.  ``bench.py`` records it next to its own number (``same_node_reference_path``) and
``tools/hf_reference_path_bench.py`` runs it standalone.
"""
from __future__ import annotations

import time

import torch

from .data import synthetic_stream
from .windows import batches, sliding_windows

NOTEBOOK_LAYERS = (22, 18, 3, 23, 11)
NOTEBOOK_RATIOS = (0.0, 0.25, 0.5, 0.75, 1.0)


def hf_qwen2(cfg, attn: str, dev, seed: int = 0):
    """A random-init HF ``Qwen2ForCausalLM`` of ``cfg``'s shape, fp32, eval mode, built on ``dev``."""
    from transformers import Qwen2Config, Qwen2ForCausalLM
    hc = Qwen2Config(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
                     num_hidden_layers=cfg.num_layers, num_attention_heads=cfg.num_heads,
                     num_key_value_heads=cfg.num_kv_heads, max_position_embeddings=cfg.max_position,
                     rope_theta=cfg.rope_theta, tie_word_embeddings=cfg.tie_embeddings, rms_norm_eps=cfg.norm_eps,
                     attn_implementation=attn)
    torch.manual_seed(seed)
    with torch.device(dev):
        m = Qwen2ForCausalLM(hc)
    return m.to(torch.float32).eval()


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
    """Layer-by-layer forward with the boundary after ``layer`` quantized; summed NLL over the scored targets."""
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


class ReferencePath:
    """The two HF models (eager for ``output_attentions``, sdpa for the layer-wise split, as the reference) with the
    same weights, and a timer for the reference's per-window work."""

    def __init__(self, cfg, dev, seed: int = 0):
        self.cfg, self.dev = cfg, torch.device(dev)
        self.eager = hf_qwen2(cfg, "eager", self.dev, seed)   # output_attentions needs the eager attention
        self.split = hf_qwen2(cfg, "sdpa", self.dev, seed)    # the reference's layer-wise model uses sdpa
        self.split.load_state_dict(self.eager.state_dict())

    @torch.no_grad()
    def run(self, b, configs: int = 1, layer: int = 11, ratio: float = 0.5):
        """One window batch: the importance forward plus ``configs`` quantized split forwards -> NLL per config."""
        ids = b.ids.to(self.dev)
        S = ids.shape[1]
        first = torch.tensor([w.first_scored for w in b.windows], device=self.dev)
        tmask = torch.arange(S, device=self.dev)[None] >= first[:, None] + 1   # token p+1 is scored from row p
        att = self.eager(input_ids=ids, output_attentions=True).attentions
        nll = []
        for c in range(configs):
            if configs == 1:
                L, r = layer, ratio
            else:
                L, r = NOTEBOOK_LAYERS[(c // 5) % 5] % self.cfg.num_layers, NOTEBOOK_RATIOS[c % 5]
            nll.append(split_forward_nll(self.split, ids, tmask, L, column_mean_importance(att[L]), r))
        del att
        return torch.stack(nll)

    def throughput(self, batch: int = 1, windows: int = 32, warmup: int = 2, configs: int = 1, layer: int = 11,
                   ratio: float = 0.5, max_length: int = 512, stride: int = 32, seed: int = 0) -> dict:
        """Time ``windows`` windows (after ``warmup`` untimed batches) in batches of ``batch``."""
        toks = synthetic_stream(299_078, self.cfg.vocab_size, seed)
        wins = [w for w in sliding_windows(toks.shape[1], max_length, stride) if w.length == max_length]
        bl = list(batches(toks, wins[: warmup * batch + windows], batch))
        cuda = self.dev.type == "cuda"
        for b in bl[:warmup]:
            self.run(b, configs, layer, ratio)
        if cuda:
            torch.cuda.synchronize(self.dev)
        t0 = time.perf_counter()
        n = 0
        for b in bl[warmup:]:
            self.run(b, configs, layer, ratio)
            n += b.B
        if cuda:
            torch.cuda.synchronize(self.dev)
        dt = time.perf_counter() - t0
        return {"batch": batch, "configs_per_window": configs, "windows": n, "seconds": round(dt, 3),
                "s_per_window": round(dt / n, 5), "window_tokens_per_s": round(n * max_length / dt, 1),
                "forward_tokens_per_s": round(n * max_length * (1 + configs) / dt, 1)}

    def close(self):
        del self.eager, self.split
