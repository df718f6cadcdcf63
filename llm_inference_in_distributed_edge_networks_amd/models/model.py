"""Decoder-only LMs (Qwen2, GPT-NeoX/Pythia) with layer-range execution.

Counterpart of the reference's layer-wise runners ``QwenPointFiveBModel``
(``Experiments/Qwen2-0.5B/qwen_layer_wise.py:5-167``) and ``Pythia70Model``
(``Experiments/Pythia-70M/pythia_model.py:13-206``), which drive HF modules
one layer at a time so that a boundary can be inserted after any layer.  Here the
model is our own: weights are stored in the layouts the gfx950 kernels want
(fused QKV with q|k|v row order, interleaved gate/up, tied head) and each layer is
a short sequence of fused kernels:

Qwen2 layer (7 launches)::

    rmsnorm -> QKV GEMM(+bias+RoPE+head-major scatter) -> flash attention
            -> O GEMM(+residual) -> rmsnorm -> gate/up GEMM(+SiLU*up) -> down GEMM(+residual)

GPT-NeoX layer (parallel residual, 6 launches)::

    dual layernorm -> QKV GEMM(+RoPE on 16 dims) -> flash attention -> O GEMM(+bias+residual)
                   -> fc GEMM(+bias+GELU) -> proj GEMM(+bias+residual)

At a boundary layer the attention can additionally emit the statistics the
importance scorers need (last-row probabilities, or row LSE + column sums), so
the S x S attention map of the reference's second "eager" model copy
(``Qwen2-0.5B/main.py:132-134``) is never materialised.

Precision.  The reference evaluates fp32 models (``qwen_layer_wise.py:17`` and
``pythia_model.py:25`` load without ``torch_dtype``).  On the GPU a model built with
``dtype=torch.float32`` runs the fp32 execution mode: the residual stream, norms,
attention, softmax statistics and the boundary codec are fp32, and every GEMM takes its
operands in the h3 split-fp16 layout (``ops.reference.h3_act`` / ``h3_weight``: a power-of-two
scaled operand as two fp16 planes, three fp16 MFMA products per fp32 product, error below the
CPU fp32 GEMM's).  Producers of GEMM inputs (norms, attention, the SwiGLU / GELU epilogues) write
the two planes of their scaled output directly (the GEMM's A loader expands them); weights are
split once at load.  The activation scales come from bounds on every GEMM input that hold for
any model input (``_h3_bounds``), so no plane can leave the fp16 range.  ``dtype=torch.bfloat16``
is the faster bf16 mode.
"""
from __future__ import annotations

import glob
import math
import os
from dataclasses import dataclass

import torch

from .. import ops
from .configs import ModelConfig


@dataclass
class AttnStats:
    """Per-head attention statistics of one layer for the importance scorers."""
    lastrow: torch.Tensor | None = None   # [B, Hq, S] P[S-1, j]
    colsum: torch.Tensor | None = None    # [B, Hq, S] sum_i P[i, j]


_H3_KEYS = ("wqkv", "wo", "wgu", "wd", "wfc", "wproj")
# fp32 mode: the QKV GEMM writes K / V^T also as h3 planes and the attention stages them by LDS DMA (bit-identical
# to the kernel's own per-tile split of fp32 K / V^T, which the tests compare against by clearing this flag)
_KV_PLANES = True


def _rownorm(w: torch.Tensor) -> torch.Tensor:
    return w.float().norm(dim=1)


def _h3_bounds(cfg: ModelConfig, L: dict) -> dict:
    """Bounds on |x| of every GEMM input of one decoder layer, valid for any layer input (exact arithmetic; the
    power-of-two scales leave a factor 2 of headroom for rounding):

    * norm outputs: |x_hat_i| <= ||x_hat||_2 <= sqrt(H) for RMSNorm and LayerNorm, so |g_i x_hat_i + b_i| <=
      sqrt(H) max|g| + max|b| and ||y||_2 <= sqrt(H) max|g| + ||b||_2 =: n;
    * attention output: a convex combination of value rows, |o| <= max_j |v_j| <= max_j n ||Wv_j||_2 + |bv_j|;
    * attention inputs (the split-plane attention kernel): v as above; q and k after RoPE, which mixes pairs of
      components (|x1 c - x2 s| <= sqrt(2) max |x_i|), so |q| <= sqrt(2) max_j (n ||Wq_j||_2 + |bq_j|) (times the
      1/sqrt(d) pre-scale), and the same for k;
    * SwiGLU output: |silu(g) u| <= |g| |u| <= n^2 max_j ||Wg_j||_2 ||Wu_j||_2;
    * GELU output: |gelu(f)| <= |f| <= max_j n ||Wfc_j||_2 + |bfc_j|."""
    H = cfg.hidden_size
    rH = math.sqrt(H)

    def norm_bound(g, b):
        e = rH * g.float().abs().max().item()
        if b is None:
            return e, e
        return e + b.float().abs().max().item(), e + b.float().norm().item()

    qkv, n1 = norm_bound(L["ln1_w"], L.get("ln1_b"))
    mlp, n2 = norm_bound(L["ln2_w"], L.get("ln2_b"))
    def proj_bound(r0, r1):
        return (n1 * _rownorm(L["wqkv"][r0:r1]) + L["bqkv"][r0:r1].float().abs()).max().item()

    q0, k0, v0 = 0, cfg.q_size, cfg.q_size + cfg.kv_size
    o = proj_bound(v0, v0 + cfg.kv_size)
    att_q = math.sqrt(2.0) * proj_bound(q0, k0) / math.sqrt(cfg.head_dim)
    att_k = math.sqrt(2.0) * proj_bound(k0, v0)
    if cfg.arch == "qwen2":
        g, u = ops.deinterleave_gate_up(L["wgu"].t().contiguous())
        down = n2 * n2 * (_rownorm(g.t()) * _rownorm(u.t())).max().item()
    else:
        down = (n2 * _rownorm(L["wfc"]) + L["bfc"].float().abs()).max().item()
    return dict(qkv=qkv, o=o, mlp=mlp, down=down, att_q=att_q, att_k=att_k)


class DecoderLM:
    def __init__(self, cfg: ModelConfig, weights: dict, device="cpu", dtype=torch.float32, h3: bool | None = None):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.w = weights
        self.layers = weights["layers"]
        # fp32 execution on the GPU: h3 operands (h3=True also runs the same op sequence on CPU, for tests)
        self.h3 = (self.device.type == "cuda" and dtype == torch.float32) if h3 is None else bool(h3)
        # per layer: activation scales s (GEMM inputs) and product scales alpha = 1 / (s_x s_w) of the h3 GEMMs
        self.h3_layer: list[dict | None] = [None] * len(self.layers)
        self.h3_head: dict | None = None
        if self.h3:
            if dtype != torch.float32:
                raise ValueError("the h3 (fp32) execution mode needs fp32 weights")
            S = ops.reference.h3_scale
            for i, L in enumerate(self.layers):
                if L is None:
                    continue
                bd = _h3_bounds(cfg, L)
                sc = {k: S(v) for k, v in bd.items()}
                ins = dict(wqkv="qkv", wo="o", wgu="mlp", wd="down", wfc="mlp", wproj="down")
                for k in _H3_KEYS:
                    if k in L:
                        L[k + "3"], sw = ops.reference.h3_weight(L[k])
                        sc["a_" + k] = 1.0 / (sc[ins[k]] * sw)
                if cfg.arch == "qwen2":
                    # fused RMSNorm-2 (the O-projection's epilogue writes the gate/up GEMM's planes, linear_h3_np):
                    # |o @ Wo^T| <= max|o| max_n ||Wo_n||_1, the gate/up product without the static activation scale
                    sc["np_po"] = bd["o"] * L["wo"].float().abs().sum(1).max().item()
                    sc["np_g2"] = L["ln2_w"].float().abs().max().item()
                    sc["a_wgu_np"] = sc["a_wgu"] * sc["mlp"]
                self.h3_layer[i] = sc
            if weights.get("head") is not None:
                g, b = weights["norm_w"], weights.get("norm_b")
                bound = math.sqrt(cfg.hidden_size) * g.float().abs().max().item() + \
                    (0.0 if b is None else b.float().abs().max().item())
                weights["head3"], sw = ops.reference.h3_weight(weights["head"])
                s_in = S(bound)
                self.h3_head = dict(s=s_in, a=1.0 / (s_in * sw))
        cos, sin = ops.rope_tables(cfg.max_position, cfg.rotary_dim, cfg.rope_theta)
        self.cos = cos.to(self.device).contiguous()
        self.sin = sin.to(self.device).contiguous()
        self.q_scale = 1.0 / math.sqrt(cfg.head_dim)
        # fp32 (h3) mode, Qwen2: RMSNorm-2 fused into the O-projection's epilogue (linear_h3_np) when the GPU kernel
        # runs the shape.  Off by default: same-box, the bench step is 0.7-1.3 % SLOWER with it (the epilogue's plane
        # stores cost the O-projection +28 us, more than the 34 us norm pass they replace once the gate/up GEMM that
        # follows is counted; docs/RESULTS.md section 6, profiles/r06/fused_norm/).  EDGE_FUSED_NORM_F32=1 turns it on;
        # tests set the attribute directly (also on CPU models, the oracle of the fused path)
        self.fuse_norm_f32 = (self.h3 and cfg.arch == "qwen2" and self.device.type == "cuda"
                              and os.environ.get("EDGE_FUSED_NORM_F32", "0") not in ("", "0"))
        # GPU fast path for RMSNorm models: the norm weight is folded into the consuming GEMM's weight and
        # the row scale is applied in its epilogue, from sum-of-squares partials the residual GEMMs emit.
        self.fuse_norm = (self.device.type == "cuda" and cfg.arch == "qwen2" and dtype == torch.bfloat16
                          and cfg.hidden_size % 64 == 0)
        if self.fuse_norm:
            for L in self.layers:
                if L is not None:
                    L["wqkv_n"] = ops.reference.fold_norm_weight(L["wqkv"], L["ln1_w"]).contiguous()
                    L["wgu_n"] = ops.reference.fold_norm_weight(L["wgu"], L["ln2_w"]).contiguous()

    # ------------------------------------------------------------------ construction
    @classmethod
    def random_init(cls, cfg: ModelConfig, seed: int = 0, device="cpu", dtype=torch.float32, std: float = 0.02,
                    layers: range | None = None, with_embed: bool = True, with_head: bool = True,
                    h3: bool | None = None, values: torch.dtype | None = None):
        """Seeded random weights of the given architecture (HF ``_init_weights`` style: N(0, 0.02)).

        ``layers`` restricts allocation to a layer range (a pipeline stage only holds its own layers);
        the generator is advanced identically so every stage sees the same weights as a full model.
        ``values`` = torch.bfloat16 / float16 rounds every weight to that storage precision (held in ``dtype``): the
        HF checkpoints are released that way (Qwen2-0.5B ``torch_dtype: bfloat16``, Pythia fp16) and the reference
        upcasts them to fp32 (``Experiments/Qwen2-0.5B/qwen_layer_wise.py:17``).
        """
        g = torch.Generator().manual_seed(seed)
        H, I, V = cfg.hidden_size, cfg.intermediate_size, cfg.vocab_size
        keep = set(range(cfg.num_layers)) if layers is None else set(layers)

        def rn(*shape, s=std):
            return (torch.randn(*shape, generator=g) * s)

        def fin(t):
            if values is not None:
                t = t.to(values)
            return t.to(device=device, dtype=dtype).contiguous()

        w: dict = {"layers": []}
        emb = rn(V, H)
        w["embed"] = fin(emb) if (with_embed or (with_head and cfg.tie_embeddings)) else None
        for i in range(cfg.num_layers):
            if cfg.arch == "qwen2":
                shapes = dict(wqkv=(cfg.qkv_size, H), bqkv=(cfg.qkv_size,), wo=(H, cfg.q_size),
                              wg=(I, H), wu=(I, H), wd=(H, I))
            else:
                shapes = dict(wqkv=(cfg.qkv_size, H), bqkv=(cfg.qkv_size,), wo=(H, cfg.q_size), bo=(H,),
                              wfc=(I, H), bfc=(I,), wproj=(H, I), bproj=(H,))
            raw = {k: rn(*s) for k, s in shapes.items()}
            ln = {k: 1.0 + rn(H, s=0.05) for k in ("ln1_w", "ln2_w")}
            if cfg.arch == "gpt_neox":
                ln.update({k: rn(H, s=0.05) for k in ("ln1_b", "ln2_b")})
            if i not in keep:
                w["layers"].append(None)
                continue
            L = {k: fin(v) for k, v in ln.items()}
            if cfg.arch == "qwen2":
                L.update(wqkv=fin(raw["wqkv"]), bqkv=fin(raw["bqkv"]), wo=fin(raw["wo"]),
                         wgu=fin(ops.interleave_gate_up(raw["wg"], raw["wu"])), wd=fin(raw["wd"]))
            else:
                L.update({k: fin(v) for k, v in raw.items()})
            w["layers"].append(L)
        w["norm_w"] = fin(1.0 + rn(H, s=0.05))
        if cfg.arch == "gpt_neox":
            w["norm_b"] = fin(rn(H, s=0.05))
        if cfg.tie_embeddings:
            w["head"] = w["embed"] if with_head else None
        else:
            hd = rn(V, H)
            w["head"] = fin(hd) if with_head else None
        if not with_embed and not cfg.tie_embeddings:
            w["embed"] = None
        return cls(cfg, w, device, dtype, h3=h3)

    @classmethod
    def from_state_dict(cls, cfg: ModelConfig, sd: dict, device="cpu", dtype=torch.float32,
                        layers: range | None = None):
        """Build from an HF-format state dict (transformers ``Qwen2ForCausalLM`` / ``GPTNeoXForCausalLM``)."""
        keep = set(range(cfg.num_layers)) if layers is None else set(layers)

        def fin(t):
            return t.detach().to(device=device, dtype=dtype).contiguous()

        def get(*names):
            for n in names:
                if n in sd:
                    return sd[n]
            raise KeyError(f"none of {names} in state dict")

        w: dict = {"layers": []}
        H, D = cfg.hidden_size, cfg.head_dim
        if cfg.arch == "qwen2":
            w["embed"] = fin(get("model.embed_tokens.weight"))
            for i in range(cfg.num_layers):
                if i not in keep:
                    w["layers"].append(None)
                    continue
                p = f"model.layers.{i}."
                wq, wk, wv = (get(p + f"self_attn.{n}_proj.weight") for n in "qkv")
                bq, bk, bv = (get(p + f"self_attn.{n}_proj.bias") for n in "qkv")
                w["layers"].append(dict(
                    ln1_w=fin(get(p + "input_layernorm.weight")), ln2_w=fin(get(p + "post_attention_layernorm.weight")),
                    wqkv=fin(torch.cat([wq, wk, wv], 0)), bqkv=fin(torch.cat([bq, bk, bv], 0)),
                    wo=fin(get(p + "self_attn.o_proj.weight")),
                    wgu=fin(ops.interleave_gate_up(get(p + "mlp.gate_proj.weight").float(),
                                                   get(p + "mlp.up_proj.weight").float())),
                    wd=fin(get(p + "mlp.down_proj.weight"))))
            w["norm_w"] = fin(get("model.norm.weight"))
            w["head"] = w["embed"] if cfg.tie_embeddings else fin(get("lm_head.weight"))
        else:
            Hh = cfg.num_heads
            w["embed"] = fin(get("gpt_neox.embed_in.weight"))
            for i in range(cfg.num_layers):
                if i not in keep:
                    w["layers"].append(None)
                    continue
                p = f"gpt_neox.layers.{i}."
                wqkv = get(p + "attention.query_key_value.weight").reshape(Hh, 3, D, H).permute(1, 0, 2, 3)
                bqkv = get(p + "attention.query_key_value.bias").reshape(Hh, 3, D).permute(1, 0, 2)
                w["layers"].append(dict(
                    ln1_w=fin(get(p + "input_layernorm.weight")), ln1_b=fin(get(p + "input_layernorm.bias")),
                    ln2_w=fin(get(p + "post_attention_layernorm.weight")),
                    ln2_b=fin(get(p + "post_attention_layernorm.bias")),
                    wqkv=fin(wqkv.reshape(3 * Hh * D, H)), bqkv=fin(bqkv.reshape(-1)),
                    wo=fin(get(p + "attention.dense.weight")), bo=fin(get(p + "attention.dense.bias")),
                    wfc=fin(get(p + "mlp.dense_h_to_4h.weight")), bfc=fin(get(p + "mlp.dense_h_to_4h.bias")),
                    wproj=fin(get(p + "mlp.dense_4h_to_h.weight")), bproj=fin(get(p + "mlp.dense_4h_to_h.bias"))))
            w["norm_w"] = fin(get("gpt_neox.final_layer_norm.weight"))
            w["norm_b"] = fin(get("gpt_neox.final_layer_norm.bias"))
            w["head"] = fin(get("embed_out.weight", "lm_head.weight"))
        return cls(cfg, w, device, dtype)

    @classmethod
    def from_pretrained_dir(cls, cfg: ModelConfig, path: str, device="cpu", dtype=torch.float32, layers=None):
        """Load ``*.safetensors`` (or ``pytorch_model.bin`` with weights_only) from a local HF snapshot."""
        files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
        sd = {}
        if files:
            from safetensors.torch import load_file
            for f in files:
                sd.update(load_file(f))
        else:
            binf = os.path.join(path, "pytorch_model.bin")
            if not os.path.exists(binf):
                raise FileNotFoundError(f"no safetensors / pytorch_model.bin under {path}")
            sd = torch.load(binf, map_location="cpu", weights_only=True)
        return cls.from_state_dict(cfg, sd, device, dtype, layers)

    # ------------------------------------------------------------------ native checkpoints
    _LAYER_KEYS = ("ln1_w", "ln1_b", "ln2_w", "ln2_b", "wqkv", "bqkv", "wo", "bo", "wgu", "wd", "wfc", "bfc",
                   "wproj", "bproj")

    def save_native(self, path: str) -> None:
        """Weights in this framework's layouts (fused qkv, interleaved gate|up) as one safetensors file."""
        from safetensors.torch import save_file
        sd = {}
        for k in ("embed", "norm_w", "norm_b"):
            if self.w.get(k) is not None:
                sd[k] = self.w[k]
        if not self.cfg.tie_embeddings and self.w.get("head") is not None:
            sd["head"] = self.w["head"]
        for i, L in enumerate(self.layers):
            if L is not None:
                for k in self._LAYER_KEYS:
                    if k in L:
                        sd[f"layers.{i}.{k}"] = L[k]
        save_file({k: v.detach().contiguous().cpu() for k, v in sd.items()}, path,
                  metadata={"model": self.cfg.name})

    @classmethod
    def load_native(cls, cfg: ModelConfig, path: str, device="cpu", dtype=torch.float32, layers=None):
        """Inverse of ``save_native`` (safetensors: nothing in the file is executed)."""
        from safetensors.torch import load_file
        sd = load_file(path)
        keep = set(range(cfg.num_layers)) if layers is None else set(layers)

        def fin(t):
            return t.to(device=device, dtype=dtype).contiguous()
        w: dict = {"layers": []}
        for k in ("embed", "norm_w", "norm_b"):
            w[k] = fin(sd[k]) if k in sd else None
        for i in range(cfg.num_layers):
            if i not in keep:
                w["layers"].append(None)
                continue
            w["layers"].append({k: fin(sd[f"layers.{i}.{k}"]) for k in cls._LAYER_KEYS if f"layers.{i}.{k}" in sd})
        w["head"] = w["embed"] if cfg.tie_embeddings else fin(sd["head"])
        return cls(cfg, w, device, dtype)

    # ------------------------------------------------------------------ execution
    def embed(self, ids: torch.Tensor) -> torch.Tensor:
        """ids [B, S] -> hidden [B*S, H]."""
        return ops.embedding(ids.to(self.device), self.w["embed"])

    def layer(self, i: int, x: torch.Tensor, B: int, S: int, stats: str | None = None):
        """Run decoder layer ``i`` on ``x`` ([B*S, H], not modified).  Returns (y, AttnStats|None).

        ``stats``: None, "lastrow" (P[S-1, :] per head), "colsum" (column sums of P per head) or a tuple of both.
        """
        cfg, L = self.cfg, self.layers[i]
        if L is None:
            raise RuntimeError(f"layer {i} is not resident on this stage")
        if self.h3:
            return self._layer_h3(i, x, B, S, stats)
        Hq, Hkv, D = cfg.num_heads, cfg.num_kv_heads, cfg.head_dim
        if self.fuse_norm:
            ssq = getattr(x, "_edge_ssq", None)
            if ssq is None:           # stage input / decoded boundary / embedding: one light kernel
                ssq = ops.row_ssq(x)
            q, k, vt = ops.qkv_rope(x, L["wqkv_n"], L["bqkv"], self.cos, self.sin, B, S, Hq, Hkv, D,
                                    cfg.rotary_dim, self.q_scale, norm=(ssq, cfg.norm_eps))
        else:
            if cfg.arch == "qwen2":
                h = ops.rmsnorm(x, L["ln1_w"], cfg.norm_eps)
            else:
                h, h2 = ops.layernorm_dual(x, L["ln1_w"], L["ln1_b"], L["ln2_w"], L["ln2_b"], cfg.norm_eps)
            q, k, vt = ops.qkv_rope(h, L["wqkv"], L["bqkv"], self.cos, self.sin, B, S, Hq, Hkv, D,
                                    cfg.rotary_dim, self.q_scale)
        kinds = () if stats is None else ((stats,) if isinstance(stats, str) else tuple(stats))
        for kd in kinds:
            if kd not in ("lastrow", "colsum"):
                raise ValueError(kd)
        o, lse = ops.attention(q, k, vt, S, need_lse=("colsum" in kinds))
        st = None
        if kinds:
            st = AttnStats(lastrow=ops.attn_lastrow(q, k, S) if "lastrow" in kinds else None,
                           colsum=ops.attn_colsum(q, k, lse, S) if "colsum" in kinds else None)
        if self.fuse_norm:
            y = ops.linear(o, L["wo"], residual=x, want_ssq=True)
            a = ops.linear(y, L["wgu_n"], act="swiglu_il", norm=(y._edge_ssq, cfg.norm_eps))
            y = ops.linear(a, L["wd"], residual=y, out=y, want_ssq=True)   # in place; fresh ssq attached
        elif cfg.arch == "qwen2":
            y = ops.linear(o, L["wo"], residual=x)
            h = ops.rmsnorm(y, L["ln2_w"], cfg.norm_eps)
            a = ops.linear(h, L["wgu"], act="swiglu_il")
            y = ops.linear(a, L["wd"], residual=y, out=y)
        else:
            y = ops.linear(o, L["wo"], L["bo"], residual=x)
            f = ops.linear(h2, L["wfc"], L["bfc"], act="gelu")
            y = ops.linear(f, L["wproj"], L["bproj"], residual=y, out=y)
        return y, st

    @staticmethod
    def _stat_kinds(stats):
        kinds = () if stats is None else ((stats,) if isinstance(stats, str) else tuple(stats))
        for kd in kinds:
            if kd not in ("lastrow", "colsum"):
                raise ValueError(kd)
        return kinds

    def _np_fused(self, M: int) -> bool:
        """RMSNorm-2 fused into the O-projection for an M-row layer (linear_h3_np on the GPU's 256x224 tiles)."""
        if not self.fuse_norm_f32:
            return False
        H = self.cfg.hidden_size
        return self.device.type != "cuda" or ops.gemm_np_supported(M, H, 2 * H)

    def _attn_h3(self, i, x, B, S, need_lse=False, n_rows=None, need_k=True, rstd_out=None):
        """fp32 mode: norm(s) -> h3 QKV GEMM (+bias+RoPE) -> fp32 attention with h3 output (``need_k=False``: no
        fp32 K on the GPU, only its planes for the attention - k is then None).  ``rstd_out``: RMSNorm-1's row
        normalisers are written there too (the fused RMSNorm-2's bound)."""
        cfg, L, sc = self.cfg, self.layers[i], self.h3_layer[i]
        h23 = None
        if cfg.arch == "qwen2":
            h3 = ops.rmsnorm(x, L["ln1_w"], cfg.norm_eps, h3=sc["qkv"], rstd_out=rstd_out)
        else:
            h3, h23 = ops.layernorm_dual(x, L["ln1_w"], L["ln1_b"], L["ln2_w"], L["ln2_b"], cfg.norm_eps,
                                         h3=(sc["qkv"], sc["mlp"]))
        kvp = None
        if _KV_PLANES and x.is_cuda:   # the QKV GEMM also emits K / V^T planes; attention stages them by LDS DMA
            q, k, vt, kp, vp = ops.qkv_rope_h3(h3, L["wqkv3"], sc["a_wqkv"], L["bqkv"], self.cos, self.sin, B, S,
                                               cfg.num_heads, cfg.num_kv_heads, cfg.head_dim, cfg.rotary_dim,
                                               self.q_scale, kv_scales=(sc["att_k"], sc["o"]),
                                               need_k=need_k)
            kvp = (kp, vp)
        else:
            q, k, vt = ops.qkv_rope_h3(h3, L["wqkv3"], sc["a_wqkv"], L["bqkv"], self.cos, self.sin, B, S,
                                       cfg.num_heads, cfg.num_kv_heads, cfg.head_dim, cfg.rotary_dim, self.q_scale)
        o3, lse = ops.attention(q, k, vt, S, need_lse=need_lse, n_rows=n_rows, h3=sc["o"],
                                in_scales=(sc["att_q"], sc["att_k"], sc["o"]), kv_planes=kvp)
        return q, k, o3, lse, h23

    def _mlp_h3(self, i, o3, x, h23, rstd1=None):
        cfg, L, sc = self.cfg, self.layers[i], self.h3_layer[i]
        if cfg.arch == "qwen2" and rstd1 is not None:
            # RMSNorm-2 in the O-projection's epilogue: its planes of p_m (y_m * ln2_w) feed the gate/up GEMM with the row
            # scale rsqrt(mean(y_m^2) + eps) / p_m (no separate norm pass over y)
            y, planes, prinv, ssq = ops.linear_h3_np(o3, L["wo3"], sc["a_wo"], x, L["ln2_w"], rstd1, sc["np_g2"],
                                                     sc["np_po"])
            rs = ops.row_rscale_mul(ssq, prinv, cfg.hidden_size, cfg.norm_eps)
            a3 = ops.linear_h3(planes, L["wgu3"], sc["a_wgu_np"], act="swiglu_il", out_scale=sc["down"], rscale=rs)
            return ops.linear_h3(a3, L["wd3"], sc["a_wd"], residual=y, out=y)
        if cfg.arch == "qwen2":
            y = ops.linear_h3(o3, L["wo3"], sc["a_wo"], residual=x)
            a3 = ops.linear_h3(ops.rmsnorm(y, L["ln2_w"], cfg.norm_eps, h3=sc["mlp"]), L["wgu3"], sc["a_wgu"],
                               act="swiglu_il", out_scale=sc["down"])
            return ops.linear_h3(a3, L["wd3"], sc["a_wd"], residual=y, out=y)
        y = ops.linear_h3(o3, L["wo3"], sc["a_wo"], L["bo"], residual=x)
        f3 = ops.linear_h3(h23, L["wfc3"], sc["a_wfc"], L["bfc"], act="gelu", out_scale=sc["down"])
        return ops.linear_h3(f3, L["wproj3"], sc["a_wproj"], L["bproj"], residual=y, out=y)

    def _layer_h3(self, i, x, B, S, stats):
        kinds = self._stat_kinds(stats)
        rstd1 = torch.empty(x.shape[0], dtype=torch.float32, device=x.device) if self._np_fused(x.shape[0]) else None
        q, k, o3, lse, h23 = self._attn_h3(i, x, B, S, need_lse="colsum" in kinds, need_k=bool(kinds), rstd_out=rstd1)
        st = None
        if kinds:   # the scores on the forward's scaled fp16 planes (consistent with its LSE)
            sc = self.h3_layer[i]
            qk = (sc["att_q"], sc["att_k"])
            st = AttnStats(lastrow=ops.attn_lastrow(q, k, S, in_scales=qk) if "lastrow" in kinds else None,
                           colsum=ops.attn_colsum(q, k, lse, S, in_scales=qk) if "colsum" in kinds else None)
        return self._mlp_h3(i, o3, x, h23, rstd1), st

    def layer_rows(self, i: int, x: torch.Tensor, B: int, S: int, rows: torch.Tensor,
                   n_rows: torch.Tensor | None = None) -> torch.Tensor:
        """Decoder layer ``i`` evaluated only at the flat row indices ``rows`` -> hidden [len(rows), H].

        For the LAST layer only the scored rows reach the LM head (``row_nll``), so everything after the
        K/V projection - attention queries, O-proj, MLP - is needed at those rows only (1/16 of the rows
        with the reference's 512/32 window/stride).  K and V still come from every row.  ``n_rows`` lets
        the attention kernel skip query blocks below the first scored row of each window."""
        cfg, L = self.cfg, self.layers[i]
        if L is None:
            raise RuntimeError(f"layer {i} is not resident on this stage")
        Hq, Hkv, D = cfg.num_heads, cfg.num_kv_heads, cfg.head_dim
        rows = rows.to(self.device)
        if self.h3:
            _, _, o3, _, h23 = self._attn_h3(i, x, B, S, n_rows=n_rows, need_k=False)
            return self._mlp_h3(i, o3.index_select(0, rows), x.index_select(0, rows),
                                None if h23 is None else h23.index_select(0, rows))
        h2 = None
        if self.fuse_norm:
            ssq = getattr(x, "_edge_ssq", None)
            if ssq is None:
                ssq = ops.row_ssq(x)
            q, k, vt = ops.qkv_rope(x, L["wqkv_n"], L["bqkv"], self.cos, self.sin, B, S, Hq, Hkv, D,
                                    cfg.rotary_dim, self.q_scale, norm=(ssq, cfg.norm_eps))
        else:
            if cfg.arch == "qwen2":
                h = ops.rmsnorm(x, L["ln1_w"], cfg.norm_eps)
            else:
                h, h2 = ops.layernorm_dual(x, L["ln1_w"], L["ln1_b"], L["ln2_w"], L["ln2_b"], cfg.norm_eps)
            q, k, vt = ops.qkv_rope(h, L["wqkv"], L["bqkv"], self.cos, self.sin, B, S, Hq, Hkv, D,
                                    cfg.rotary_dim, self.q_scale)
        o, _ = ops.attention(q, k, vt, S, n_rows=n_rows)
        og, xg = o.index_select(0, rows), x.index_select(0, rows)
        if self.fuse_norm:
            y = ops.linear(og, L["wo"], residual=xg, want_ssq=True)
            a = ops.linear(y, L["wgu_n"], act="swiglu_il", norm=(y._edge_ssq, cfg.norm_eps))
            return ops.linear(a, L["wd"], residual=y, out=y)
        if cfg.arch == "qwen2":
            y = ops.linear(og, L["wo"], residual=xg)
            a = ops.linear(ops.rmsnorm(y, L["ln2_w"], cfg.norm_eps), L["wgu"], act="swiglu_il")
            return ops.linear(a, L["wd"], residual=y, out=y)
        y = ops.linear(og, L["wo"], L["bo"], residual=xg)
        f = ops.linear(h2.index_select(0, rows), L["wfc"], L["bfc"], act="gelu")
        return ops.linear(f, L["wproj"], L["bproj"], residual=y, out=y)

    def final_norm(self, x: torch.Tensor, rows: torch.Tensor | None = None) -> torch.Tensor:
        if self.cfg.arch == "qwen2":
            return ops.rmsnorm(x, self.w["norm_w"], self.cfg.norm_eps, rows)
        return ops.layernorm(x, self.w["norm_w"], self.w["norm_b"], self.cfg.norm_eps, rows)

    def row_nll(self, x: torch.Tensor, rows: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
        """Per-row NLL of the scored rows only (final norm + LM head + CE fused)."""
        if self.h3:
            rows, hs = rows.to(self.device), self.h3_head
            if self.cfg.arch == "qwen2":
                h3 = ops.rmsnorm(x, self.w["norm_w"], self.cfg.norm_eps, rows, h3=hs["s"])
            else:
                h3 = ops.layernorm(x, self.w["norm_w"], self.w["norm_b"], self.cfg.norm_eps, rows, h3=hs["s"])
            return ops.head_nll_h3(h3, self.w["head3"], hs["a"], targets.to(self.device))
        h = self.final_norm(x, rows.to(self.device))
        return ops.head_nll(h, self.w["head"], targets.to(self.device))

    def logits(self, x: torch.Tensor) -> torch.Tensor:
        """Full logits (tests / debugging only; the eval path never materialises them)."""
        h = self.final_norm(x)
        return ops.reference.linear(h, self.w["head"], out_dtype=torch.float32)

    def forward_hidden(self, ids: torch.Tensor, start: int = 0, end: int | None = None) -> torch.Tensor:
        B, S = ids.shape
        x = self.embed(ids)
        for i in range(start, self.cfg.num_layers if end is None else end):
            x, _ = self.layer(i, x, B, S)
        return x

    def resident_bytes(self) -> int:
        seen, n = set(), 0

        def add(t):
            nonlocal n
            if t is not None and id(t) not in seen:
                seen.add(id(t))
                n += t.numel() * t.element_size()
        for L in self.layers:
            if L:
                for t in L.values():
                    add(t)
        for k in ("embed", "head", "norm_w", "norm_b"):
            add(self.w.get(k))
        return n


def find_hf_snapshot(hf_id: str) -> str | None:
    """Locate a local HF-hub snapshot of ``hf_id`` (no network is ever used)."""
    if not hf_id:
        return None
    roots = [os.environ.get("HF_HOME", os.path.expanduser("~/.cache/huggingface")), "/root/.cache/huggingface"]
    for r in roots:
        d = os.path.join(r, "hub", "models--" + hf_id.replace("/", "--"), "snapshots")
        for snap in sorted(glob.glob(os.path.join(d, "*"))):
            if glob.glob(os.path.join(snap, "*.safetensors")) or os.path.exists(os.path.join(snap, "pytorch_model.bin")):
                return snap
    return None


def build_model(cfg: ModelConfig, device="cpu", dtype=torch.float32, weights: str = "", seed: int = 0,
                layers: range | None = None, with_embed=True, with_head=True,
                values: torch.dtype | None = None) -> tuple[DecoderLM, str]:
    """Model from explicit weights dir, else a local HF snapshot, else seeded random init (``values``: the random
    weights' storage precision, see ``DecoderLM.random_init``).

    Returns (model, provenance string)."""
    path = weights or find_hf_snapshot(cfg.hf_id)
    if path and os.path.isfile(path) and path.endswith(".safetensors"):
        return DecoderLM.load_native(cfg, path, device, dtype, layers), f"native:{path}"
    if path and os.path.isdir(path):
        return DecoderLM.from_pretrained_dir(cfg, path, device, dtype, layers), f"hf:{path}"
    tag = "" if values is None else f", {str(values).replace('torch.', '')} values"
    return (DecoderLM.random_init(cfg, seed, device, dtype, layers=layers, with_embed=with_embed,
                                  with_head=with_head, values=values), f"random-init(seed={seed}{tag})")
