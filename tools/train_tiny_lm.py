"""Train the byte-level Qwen2-architecture model (``byte-qwen2``) on local text, for quality experiments.

No pretrained checkpoint or WikiText copy is reachable from this machine, so PPL-vs-compression curves on
random weights would be meaningless.  This trains a small model of the same architecture family as
Qwen2-0.5B (GQA, RoPE, RMSNorm, SwiGLU, tied head) on local Python sources (byte tokens: by default
``eval.data.local_text_bytes('train-large')``, the stdlib's training split plus the installed packages' sources,
~270 MB, so a few minutes of training never revisit a byte), then saves it with ``DecoderLM.save_native``; the
experiment drivers load it with ``weights=<file>.safetensors``.

Held-out-driven stop: every ``--eval-every`` seconds the loss on 128 random windows of the held-out stdlib split AND
on 128 random windows of the stdlib training split (the same distribution) is measured; the best held-out
checkpoint is kept, and training stops once the held-out loss has not improved for ``--patience`` evaluations (or
the time budget ends).  The last line is a JSON summary with the train / held-out gap of the kept checkpoint, the
epochs trained, and a memorisation check: the loss on the first two training batches (seen) against fresh windows
of the same training stream.

The training forward is plain PyTorch autograd (bf16 autocast, SDPA) over the framework's own weight
layout (fused qkv, interleaved gate|up), so the checkpoint is exactly what the HIP inference path runs.
"""
import argparse
import json
import math
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from llm_inference_in_distributed_edge_networks_amd.eval.data import local_text_bytes  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.models import DecoderLM, get_config  # noqa: E402
from llm_inference_in_distributed_edge_networks_amd.ops import reference as R  # noqa: E402


def forward(w, cfg, ids, cos, sin, capture=None):
    """Logits; ``capture`` = {layer: None}: filled with the residual stream leaving those layers (the boundary
    tensors of a split after them)."""
    B, S = ids.shape
    Hq, Hkv, D = cfg.num_heads, cfg.num_kv_heads, cfg.head_dim
    x = w["embed"][ids]
    c, s = cos[:S], sin[:S]
    for li, L in enumerate(w["layers"]):
        h = F.rms_norm(x, (cfg.hidden_size,), L["ln1_w"], cfg.norm_eps)
        y = (h @ L["wqkv"].t() + L["bqkv"]).view(B, S, Hq + 2 * Hkv, D).transpose(1, 2)
        q, k, v = y[:, :Hq], y[:, Hq:Hq + Hkv], y[:, Hq + Hkv:]
        q, k = R.apply_rope(q.float(), c, s, cfg.rotary_dim).to(x.dtype), R.apply_rope(k.float(), c, s,
                                                                                      cfg.rotary_dim).to(x.dtype)
        o = F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=True)
        x = x + o.transpose(1, 2).reshape(B, S, Hq * D) @ L["wo"].t()
        h = F.rms_norm(x, (cfg.hidden_size,), L["ln2_w"], cfg.norm_eps)
        g, u = R.deinterleave_gate_up((h @ L["wgu"].t()).view(B * S, -1))
        x = x + (F.silu(g) * u).view(B, S, -1) @ L["wd"].t()
        if capture is not None and li in capture:
            capture[li] = x.detach().float()
    x = F.rms_norm(x, (cfg.hidden_size,), w["norm_w"], cfg.norm_eps)
    return x @ w["embed"].t()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="byte-qwen2")
    ap.add_argument("--out", default="/tmp/byte_qwen2.safetensors")
    ap.add_argument("--minutes", type=float, default=4.0)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--lr", type=float, default=2e-3)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--warmup", type=int, default=200, help="linear learning-rate warmup steps")
    ap.add_argument("--eval-every", type=float, default=15.0, help="seconds between held-out evaluations")
    ap.add_argument("--corpus", default="large", choices=["large", "stdlib"],
                    help="large: stdlib train split + installed packages' sources; stdlib: the 10 MB split alone")
    ap.add_argument("--patience", type=int, default=4, help="evaluations without a held-out improvement to stop")
    ap.add_argument("--weight-decay", type=float, default=0.1)
    ap.add_argument("--bos", type=int, default=-1,
                    help="byte id >= 256 put at position 0 of every training / probe window (a fixed start-of-window "
                         "token, the position a sink forms at); -1: none")
    ap.add_argument("--probe-layers", default="3,11,18,22,23",
                    help="layers whose output (a boundary tensor) is probed for outliers at every evaluation")
    a = ap.parse_args()
    torch.manual_seed(a.seed)
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    cfg = get_config(a.model)
    m = DecoderLM.random_init(cfg, a.seed, device=dev, dtype=torch.float32)
    params = [m.w["embed"], m.w["norm_w"]] + [t for L in m.layers for t in L.values()]
    for p in params:
        p.requires_grad_(True)
    w = {"embed": m.w["embed"], "norm_w": m.w["norm_w"], "layers": m.layers}
    data = local_text_bytes("train-large" if a.corpus == "large" else "train").view(-1).to(dev)
    def sample(stream, n, seed):   # n random windows spread over the whole stream (not its first files)
        gs = torch.Generator().manual_seed(seed)
        idx = torch.randint(0, stream.numel() - a.seq - 1, (n,), generator=gs).tolist()
        return torch.stack([stream[i:i + a.seq + 1] for i in idx]).long().to(dev)
    # held-out: the stdlib eval split (every 10th file); train sample: the stdlib TRAIN split, the held-out split's own
    # distribution (the gap between them is a generalisation gap, not the packages' sources being other text)
    held = sample(local_text_bytes("eval").view(-1), 128, 4321)
    trs = sample(local_text_bytes("train").view(-1), 128, 1234)
    bos = a.bos if a.bos >= 0 else None
    if bos is not None:
        held[:, 0] = bos
        trs[:, 0] = bos
    from llm_inference_in_distributed_edge_networks_amd.eval import data as D
    probe_layers = [int(x) for x in a.probe_layers.split(",") if x.strip() and int(x) < cfg.num_layers]

    def probe(step):
        """Outliers of the boundary tensors on 8 held-out windows: peak / RMS over the whole tensor (what one global
        int4 scale sees), and the position-0 token's and the other tokens' largest |x| over the RMS."""
        cap = {L: None for L in probe_layers}
        with torch.no_grad(), torch.autocast(dev, dtype=torch.bfloat16):
            forward(w, cfg, held[:8, :-1], cos, sin, capture=cap)
        row = {"probe_step": step}
        for L, x in cap.items():
            rms = x.pow(2).mean().sqrt()
            row[str(L)] = {"peak_over_rms": round(float(x.abs().max() / rms), 2),
                           "pos0_peak_over_rms": round(float(x[:, 0].abs().max() / rms), 2),
                           "rest_peak_over_rms": round(float(x[:, 1:].abs().max() / rms), 2),
                           "top_channel": int(x[:, 0].abs().amax(0).argmax())}
        print(json.dumps(row), flush=True)
        return row
    # memorisation: the first two training batches (windows the model was trained on) against fresh windows of the
    # same training stream
    fresh = sample(data, 2 * a.batch, 999)
    seen = []
    opt = torch.optim.AdamW(params, lr=a.lr, betas=(0.9, 0.95), weight_decay=a.weight_decay)
    cos, sin = m.cos, m.sin
    print(f"training {cfg.name}: {sum(p.numel() for p in params) / 1e6:.1f}M params, {data.numel() / 1e6:.1f}M train "
          f"bytes ({D.LAST_EXCLUDED} package files dropped as copies of held-out files), batch {a.batch}x{a.seq}, "
          f"{a.minutes} min, bos {bos}", flush=True)
    probes = [probe(0)]
    t0, step, budget = time.time(), 0, a.minutes * 60
    g = torch.Generator(device=dev).manual_seed(a.seed)
    last_print = 0.0
    best = (float("inf"), 0, None, 0.0)  # held-out loss, step, CPU snapshot, train-sample loss

    def nll(x):
        out = 0.0
        for c in x.split(32):
            with torch.no_grad(), torch.autocast(dev, dtype=torch.bfloat16):
                lg = forward(w, cfg, c[:, :-1], cos, sin).float()
            out += float(F.cross_entropy(lg.view(-1, cfg.vocab_size), c[:, 1:].reshape(-1), reduction="sum"))
        return out / (x.shape[0] * (x.shape[1] - 1))
    stale = 0
    while True:
        el = time.time() - t0
        if el > budget:
            break
        frac = el / budget
        lr = a.lr * min(1.0, (step + 1) / a.warmup) * (0.1 + 0.9 * 0.5 * (1 + math.cos(math.pi * frac)))
        for grp in opt.param_groups:
            grp["lr"] = lr
        idx = torch.randint(0, data.numel() - a.seq - 1, (a.batch,), device=dev, generator=g)
        chunk = torch.stack([data[i:i + a.seq + 1] for i in idx.tolist()]).long()
        if bos is not None:
            chunk[:, 0] = bos
        if step < 2:
            seen.append(chunk)
        with torch.autocast(dev, dtype=torch.bfloat16):
            logits = forward(w, cfg, chunk[:, :-1], cos, sin)
        loss = F.cross_entropy(logits.float().view(-1, cfg.vocab_size), chunk[:, 1:].reshape(-1))
        opt.zero_grad(set_to_none=True)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(params, 1.0)
        opt.step()
        step += 1
        if el - last_print > a.eval_every:
            last_print = el
            hl, tl = nll(held), nll(trs)
            if hl < best[0]:
                best = (hl, step, [p.detach().to("cpu", copy=True) for p in params], tl)
                stale = 0
            else:
                stale += 1
            print(f"step {step} t={el:.0f}s lr={lr:.2e} batch {loss.item():.3f} train-sample {tl:.3f} "
                  f"held-out {hl:.3f} nats/byte ({hl / math.log(2):.3f} bits/byte)", flush=True)
            probes.append(probe(step))
            if stale >= a.patience:
                print(f"held-out loss has not improved for {stale} evaluations: stopping", flush=True)
                break
    for p in params:
        p.requires_grad_(False)
    if best[2] is not None:
        for p, b in zip(params, best[2]):
            p.copy_(b.to(p.device))
        print(f"keeping the best held-out checkpoint: step {best[1]}, {best[0]:.3f} nats/byte", flush=True)
    seen_l, fresh_l = nll(torch.cat(seen)), nll(fresh)
    print(json.dumps({"best_step": best[1], "steps": step, "held_out_nats_per_byte": round(best[0], 4),
                      "train_sample_nats_per_byte": round(best[3], 4),
                      "gap": round((best[0] - best[3]) / best[0], 4) if best[0] < float("inf") else None,
                      "seen_nats_per_byte": round(seen_l, 4), "fresh_nats_per_byte": round(fresh_l, 4),
                      "memorisation_gap": round((fresh_l - seen_l) / fresh_l, 4),
                      "epochs": round(step * a.batch * a.seq / data.numel(), 4),
                      "corpus": a.corpus, "train_bytes": int(data.numel()), "seed": a.seed, "bos": bos,
                      "excluded_eval_copies": D.LAST_EXCLUDED, "final_probe": probe(step)}), flush=True)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    DecoderLM(cfg, {"embed": m.w["embed"], "norm_w": m.w["norm_w"], "head": m.w["embed"], "layers": m.layers},
              "cpu", torch.float32).save_native(a.out)
    print(f"saved {a.out} after {step} steps", flush=True)


if __name__ == "__main__":
    main()
