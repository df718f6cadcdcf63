"""AttnLRP per-head relevance calibration (reference C8: ``Experiments/Relevance/main.py``,
``Notebooks/attention_head_weights_via_relevance.ipynb``).

The reference monkey-patches HF Qwen2 with ``lxt.efficient`` rules (``Relevance/main.py:41``),
embeds each window with ``requires_grad``, runs a forward that returns the attention
probabilities, seeds the backward with the max logit at the last position
(``max_logit.backward(max_logit)``, ``:87-88``) and takes per-head relevance
``sum_{i,j} A * dA/d..`` (``:96-103``), accumulated over windows and normalised per layer so each
layer's heads sum to 1 (signed, ``:111-118``).

``lxt`` is not available here, so the rules are re-implemented as autograd functions on this
framework's own model weights ("efficient" LRP = Input x modified-Gradient):

* linear layers, residual adds, RoPE: plain gradient (epsilon-LRP / Gradient x Input);
* RMSNorm / LayerNorm: identity rule - the normaliser is treated as a constant (detached);
* SiLU / GELU: identity rule - backward multiplies by f(x)/x instead of f'(x);
* element-wise gate*up and the two attention matmuls (Q K^T, A V): uniform rule - each input
  receives half of the Gradient x Input relevance (backward scaled by 0.5);
* softmax: Gradient x Input of the softmax (the bias-free Taylor rule), -inf logits zeroed.

The tests check per-rule conservation (Gradient x Input through each rule sums to the output relevance)
and that the head relevance computed from the head outputs equals the literal S x S probability hook.
``head_relevance`` here is the autograd oracle (fp32, one window).  The production passes are the explicit-backward
engines, batched over windows and checked against this oracle by the tests: ``engine_f32.RelevanceEngineH3`` at the
reference's precision (fp32: h3 GEMMs, ``csrc/lrp_f32.hip``) and ``engine.RelevanceEngine`` with bf16 storage
(``csrc/lrp.hip``).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from .. import ops
from ..ops import reference as R


class _IdentityAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kind: str):
        y = F.silu(x) if kind == "silu" else F.gelu(x)
        ctx.save_for_backward(x, y)
        return y

    @staticmethod
    def backward(ctx, g):
        x, y = ctx.saved_tensors
        ratio = torch.where(x.abs() > 1e-6, y / torch.where(x.abs() > 1e-6, x, torch.ones_like(x)),
                            torch.full_like(x, 0.5))
        return g * ratio, None


class _UniformMul(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        ctx.save_for_backward(a, b)
        return a * b

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        return 0.5 * g * b, 0.5 * g * a


class _UniformMatmul(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        ctx.save_for_backward(a, b)
        return a @ b

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        return 0.5 * (g @ b.transpose(-1, -2)), 0.5 * (a.transpose(-1, -2) @ g)


class _Softmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        s = torch.softmax(x, -1)
        ctx.save_for_backward(s)
        return s

    @staticmethod
    def backward(ctx, g):
        (s,) = ctx.saved_tensors
        gi = s * (g - (s * g).sum(-1, keepdim=True))
        return gi


def _rmsnorm_id(x, w, eps):
    rstd = torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps).detach()
    return x * rstd * w


def _layernorm_id(x, w, b, eps):
    mu = x.mean(-1, keepdim=True)
    xc = x - mu
    rstd = torch.rsqrt(xc.pow(2).mean(-1, keepdim=True) + eps).detach()
    return xc * rstd * w + b


def _lin(x, w, b=None):
    y = x @ w.t()
    return y + b if b is not None else y


def lrp_forward(model, ids: torch.Tensor, dtype=torch.float32, keep_probs: bool = True, keep_x: bool = False):
    """Differentiable forward with AttnLRP rules.

    Returns (logits_last [B, V], embeds, per-layer tensors[, layer inputs]): the attention probabilities A
    (S x S per head, ``keep_probs``) or the per-head attention outputs O = A V (S x D per head).  Under the
    uniform rule on A V, dA = 0.5 dO V^T, hence sum_ij A_ij dA_ij = 0.5 sum_i dO_i . O_i: the head relevance
    needs only O and its gradient - an S/D-times smaller tensor than A (8x at S=512).  ``keep_x`` also returns
    the residual stream entering every layer (gradients retained: the boundary-channel relevance)."""
    cfg = model.cfg
    f = lambda t: None if t is None else t.to(dtype)  # noqa: E731
    B, S = ids.shape
    Hq, Hkv, D = cfg.num_heads, cfg.num_kv_heads, cfg.head_dim
    emb = f(model.w["embed"]).index_select(0, ids.reshape(-1).to(model.device)).detach().requires_grad_(True)
    x = emb
    cos, sin = model.cos[:S].to(dtype), model.sin[:S].to(dtype)
    probs = []
    xs = []
    for L in model.layers:
        if keep_x:
            if x is not emb:
                x.retain_grad()
            xs.append(x)
        if cfg.arch == "qwen2":
            h = _rmsnorm_id(x, f(L["ln1_w"]), cfg.norm_eps)
        else:
            h = _layernorm_id(x, f(L["ln1_w"]), f(L["ln1_b"]), cfg.norm_eps)
            h2 = _layernorm_id(x, f(L["ln2_w"]), f(L["ln2_b"]), cfg.norm_eps)
        y = _lin(h, f(L["wqkv"]), f(L["bqkv"])).view(B, S, Hq + 2 * Hkv, D).permute(0, 2, 1, 3)
        q, k, v = y[:, :Hq], y[:, Hq:Hq + Hkv], y[:, Hq + Hkv:]
        q = R.apply_rope(q, cos, sin, cfg.rotary_dim) * model.q_scale
        k = R.apply_rope(k, cos, sin, cfg.rotary_dim)
        k = k.repeat_interleave(Hq // Hkv, 1)
        v = v.repeat_interleave(Hq // Hkv, 1)
        sc = _UniformMatmul.apply(q, k.transpose(-1, -2))
        mask = torch.ones(S, S, dtype=torch.bool, device=sc.device).triu(1)
        sc = sc.masked_fill(mask, float("-inf"))
        A = _Softmax.apply(sc)
        oh = _UniformMatmul.apply(A, v)          # [B, Hq, S, D]
        if keep_probs:
            A.retain_grad()
            probs.append(A)
        else:
            oh.retain_grad()
            probs.append(oh)
        o = oh.permute(0, 2, 1, 3).reshape(B * S, Hq * D)
        if cfg.arch == "qwen2":
            x = x + _lin(o, f(L["wo"]))
            h = _rmsnorm_id(x, f(L["ln2_w"]), cfg.norm_eps)
            g, u = R.deinterleave_gate_up(_lin(h, f(L["wgu"])))
            x = x + _lin(_UniformMul.apply(_IdentityAct.apply(g, "silu"), u), f(L["wd"]))
        else:
            a = _lin(o, f(L["wo"]), f(L["bo"]))
            mlp = _lin(_IdentityAct.apply(_lin(h2, f(L["wfc"]), f(L["bfc"])), "gelu"), f(L["wproj"]), f(L["bproj"]))
            x = x + a + mlp
    last = x.view(B, S, -1)[:, -1]
    if cfg.arch == "qwen2":
        hN = _rmsnorm_id(last, f(model.w["norm_w"]), cfg.norm_eps)
    else:
        hN = _layernorm_id(last, f(model.w["norm_w"]), f(model.w["norm_b"]), cfg.norm_eps)
    logits = _lin(hN, f(model.w["head"]))
    if keep_x:
        return logits, emb, probs, xs
    return logits, emb, probs


def head_relevance(model, ids: torch.Tensor, dtype=torch.float32, via_probs: bool = False):
    """Per-(layer, head) relevance of one window (B=1): sum_{i,j} A * dA, after seeding the max logit.

    ``via_probs`` computes it literally from the retained S x S probabilities (the reference's hook,
    ``Relevance/main.py:96-103``); the default uses the exact identity 0.5 * sum dO . O.
    Returns (rel [layers, heads], input relevance sum, seed logit)."""
    logits, emb, probs = lrp_forward(model, ids, dtype, keep_probs=via_probs)
    mx = logits[0].max()
    mx.backward(mx.detach())
    scale = 1.0 if via_probs else 0.5
    rel = torch.stack([scale * (T * T.grad).sum(dim=(0, 2, 3)) for T in probs]).detach()
    in_rel = (emb * emb.grad).sum().detach()
    return rel, in_rel, mx.detach()


def head_relevance_batched(model, ids: torch.Tensor, dtype=torch.float32, group: int = 64, want_sens: bool = False):
    """``head_relevance`` for B windows at once (windows are independent: each seeds its own max logit), plus the
    relevance of the residual stream entering every layer per ``group``-channel block (head-sized groups):
    chan[b, l, g] = sum over tokens and the group's channels of |x * dx| (LRP Gradient x Input, magnitude: the
    bit-allocation signal of the head-group boundary codec).  Returns (rel [B, layers, heads], in_rel [B],
    seed logit [B], chan [B, layers, H / group][, sens [B, layers, H / group]]: ``want_sens``, the groups'
    quantization sensitivity, ``ops.reference.group_sens``).  Plain PyTorch ops (autograd, library GEMMs): the
    reference-precision path of the offline calibration on any device."""
    B, S = ids.shape
    with torch.enable_grad():
        logits, emb, outs, xs = lrp_forward(model, ids, dtype, keep_probs=False, keep_x=True)
        mx = logits.max(-1).values
        torch.autograd.backward(mx, grad_tensors=mx.detach())
    rel = torch.stack([0.5 * (T * T.grad).sum(dim=(2, 3)) for T in outs], 1).detach()
    in_rel = (emb * emb.grad).view(B, S, -1).sum((1, 2)).detach()
    H = emb.shape[-1]
    chan = torch.stack([(x * x.grad).abs().view(B, S, H // group, group).sum((1, 3)) for x in xs], 1).detach()
    out = (rel.float(), in_rel.float(), mx.detach().float(), chan.float())
    if want_sens:
        from ..ops import reference as R
        out += (torch.stack([R.group_sens(x.detach(), x.grad, B, S, group) for x in xs], 1).float(),)
    return out


def normalize_per_layer(rel: torch.Tensor) -> torch.Tensor:
    """Each layer's heads divided by the layer sum (signed); a zero sum divides by 1e-9 as the reference does
    (``Experiments/Relevance/main.py:111-118``) instead of producing NaN head weights."""
    s = rel.sum(-1, keepdim=True)
    return rel / torch.where(s != 0, s, torch.full_like(s, 1e-9))


def relevance_main(p) -> list:
    """Entry point of Experiments/Relevance/main.py: writes attention_head_weights.json."""
    import json

    from ..config import dump_json, resolve_dtype
    from ..eval.data import token_stream
    from ..eval.windows import sliding_windows
    from ..models import build_model, get_config
    from ..parallel.dist import all_reduce_sum, init_distributed
    from ..utils.logging import log, progress_bar
    env = init_distributed(p.device)
    device = str(env.device)
    cfg = get_config(p.model or "qwen2-0.5b")
    # engine: on a GPU the explicit-backward HIP engines - fp32 ("auto" = the reference's precision): h3 GEMMs on
    # the transposed weights + the fp32 attention rule (engine_f32.RelevanceEngineH3, head table within 1e-4 of the
    # CPU fp32 oracle); bf16: csrc/lrp.hip with bf16 storage (engine.RelevanceEngine, within ~3 %).  The autograd
    # rules (head_relevance_batched) run on the CPU, or anywhere with lrp_engine "autograd".
    dtype = resolve_dtype(p, device) if p.dtype != "auto" else torch.float32
    if p.window_batch <= 0:   # auto: 8 windows per relevance batch (forward + AttnLRP backward)
        p.window_batch = 8
    kind = getattr(p, "lrp_engine", "auto")
    if kind not in ("auto", "hip", "autograd"):
        raise ValueError(f"lrp_engine must be auto, hip or autograd (got {kind!r})")
    on_gpu = device.startswith("cuda")
    if kind == "hip" and not on_gpu:
        raise ValueError("lrp_engine 'hip' needs a GPU")
    use_hip = on_gpu and kind != "autograd"
    model, prov = build_model(cfg, device, dtype, weights=p.weights, seed=p.seed)
    ids, data_prov = token_stream(p.dataset, cfg.hf_id, cfg.vocab_size, p.synthetic_tokens, p.seed,
                                  strict=p.strict_data)
    wins = sliding_windows(ids.shape[1], p.max_length or 512, p.stride)
    if p.max_windows:
        wins = wins[: p.max_windows]
    dname = str(dtype).replace("torch.", "")
    log(f"relevance: model={cfg.name} weights={prov} data={data_prov} windows={len(wins)} "
        f"engine={('hip-' if use_hip else 'autograd-') + dname}")
    from ..eval.windows import batches
    eng = None
    if use_hip:
        from .engine import RelevanceEngine
        from .engine_f32 import RelevanceEngineH3
        eng = RelevanceEngineH3(model) if dtype == torch.float32 else RelevanceEngine(model)
    G = cfg.hidden_size // 64
    acc = torch.zeros(cfg.num_layers, cfg.num_heads, dtype=torch.float64, device=device)
    cacc = torch.zeros(cfg.num_layers, G, dtype=torch.float64, device=device)
    sacc = torch.zeros(cfg.num_layers, G, dtype=torch.float64, device=device)
    pb = progress_bar(len(wins), env.is_main)
    for bi, b in enumerate(batches(ids, wins, max(1, p.window_batch))):
        if bi % env.world_size != env.rank:
            continue
        if eng is not None:
            rel, _, _, chan, sens = eng.head_relevance(b.ids, want_channels=True, want_sens=True)
        else:
            rel, _, _, chan, sens = head_relevance_batched(model, b.ids.to(device), dtype, want_sens=True)
        acc += rel.double().sum(0)
        cacc += chan.double().sum(0)
        sacc += sens.double().sum(0)
        pb.update(b.B * env.world_size)
    pb.close()
    all_reduce_sum(acc)
    all_reduce_sum(cacc)
    all_reduce_sum(sacc)
    weights = normalize_per_layer(acc).float().cpu().tolist()
    chan_w = normalize_per_layer(cacc).float().cpu().tolist()
    # the groups' quantization sensitivity, per layer relative to its mean (the allocation only compares the groups
    # of one boundary)
    sens_w = (sacc / sacc.mean(-1, keepdim=True).clamp_min(1e-300)).float().cpu().tolist()
    if env.is_main:
        out = os.path.join(p.output_dir, "attention_head_weights.json")
        dump_json(weights, out)
        cout = os.path.join(p.output_dir, "channel_group_relevance.json")
        dump_json(chan_w, cout)
        dump_json(sens_w, os.path.join(p.output_dir, "channel_group_sensitivity.json"))
        log(f"wrote {out} and {cout}")
    return weights
