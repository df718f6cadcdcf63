"""Batched AttnLRP head relevance on the framework's own kernels.

Same quantity as ``attnlrp.head_relevance`` (the reference's ``Relevance/main.py:84-103``: seed the max
logit of the last position with its own value, backpropagate with the AttnLRP rules, sum ``A * dA`` per
head), computed without autograd and without any S x S tensor:

* forward with saves: the regular fused layer kernels (QKV+RoPE with the RMSNorm row scale folded in,
  flash attention with its row LSE, O / gate-up / down GEMMs), keeping q, k, v, o, lse, the gate|up
  pre-activations and the norm row scales of every layer;
* seed: only the B last rows carry gradient (``d hN = mx * W_head[argmax]``, detached final norm), so the last
  layer runs its O projection and MLP on those rows only, forward and backward;
* backward per layer, in reverse: input-gradient GEMMs with the transposed weights (norm row scale and
  residual in the epilogue), the SwiGLU / GELU / LayerNorm rules, and the attention backward kernel
  (``csrc/lrp.hip``) that also emits the per-(window, head) relevance ``0.5 sum_i dO_i . O_i``.

CUDA tensors run the gfx950 kernels (bf16 storage, fp32 accumulation); CPU tensors run the fp32 reference
ops, which the tests check against the autograd oracle.  Windows of one batch are independent, so a
batch of B windows gives B relevance tables in one pass.
"""
from __future__ import annotations


import torch

from .. import ops
from ..ops import reference as R
from ..models.model import DecoderLM



class RelevanceEngine:
    def __init__(self, model: DecoderLM):
        self.m = model
        cfg = model.cfg
        if cfg.head_dim != 64:
            raise ValueError("relevance engine is specialised for head_dim 64")
        if any(L is None for L in model.layers) or model.w.get("embed") is None or model.w.get("head") is None:
            raise ValueError("relevance engine needs the whole model resident")
        self.qwen = cfg.arch == "qwen2"
        self.T = []          # per-layer transposed / folded weights of the backward GEMMs
        for L in model.layers:
            t = {}
            if self.qwen:
                wqkv_n = L.get("wqkv_n")
                wgu_n = L.get("wgu_n")
                if wqkv_n is None:
                    wqkv_n = ops.reference.fold_norm_weight(L["wqkv"], L["ln1_w"]).contiguous()
                    wgu_n = ops.reference.fold_norm_weight(L["wgu"], L["ln2_w"]).contiguous()
                t.update(wqkv_n=wqkv_n, wgu_n=wgu_n, wqkvT=wqkv_n.t().contiguous(), woT=L["wo"].t().contiguous(),
                         wguT=wgu_n.t().contiguous(), wdT=L["wd"].t().contiguous())
            else:
                t.update(wqkvT=L["wqkv"].t().contiguous(), woT=L["wo"].t().contiguous(),
                         wfcT=L["wfc"].t().contiguous(), wprojT=L["wproj"].t().contiguous())
            self.T.append(t)

    # ------------------------------------------------------------------------------------------------
    def _forward(self, ids: torch.Tensor):
        m, cfg = self.m, self.m.cfg
        B, S = ids.shape
        H, Hq, Hkv, D = cfg.hidden_size, cfg.num_heads, cfg.num_kv_heads, cfg.head_dim
        x = m.embed(ids)
        emb = x
        saves = []
        last = torch.arange(B, device=ids.device) * S + (S - 1)   # the seeded rows
        nl = len(m.layers)
        for i, L in enumerate(m.layers):
            t = self.T[i]
            sv = {"x": x}
            if self.qwen:
                ssq1 = ops.row_ssq(x)
                sv["rs1"] = ops.row_rscale(ssq1, H, cfg.norm_eps)
                q, k, vt = ops.qkv_rope(x, t["wqkv_n"], L["bqkv"], m.cos, m.sin, B, S, Hq, Hkv, D, cfg.rotary_dim,
                                        m.q_scale, norm=(ssq1, cfg.norm_eps))
            else:
                sv["rs1"] = ops.ln_rstd(x, cfg.norm_eps)
                h1, h2 = ops.layernorm_dual(x, L["ln1_w"], L["ln1_b"], L["ln2_w"], L["ln2_b"], cfg.norm_eps)
                q, k, vt = ops.qkv_rope(h1, L["wqkv"], L["bqkv"], m.cos, m.sin, B, S, Hq, Hkv, D, cfg.rotary_dim,
                                        m.q_scale)
            o, lse = ops.attention(q, k, vt, S, need_lse=True)
            sv.update(q=q, k=k, v=vt[..., :S].transpose(-1, -2).contiguous(), o=o, lse=lse.contiguous())
            if i == nl - 1:   # only the seeded rows reach the seed: O-proj and MLP on those rows
                sv["rows"] = last
                o, x = o.index_select(0, last), x.index_select(0, last)
                if not self.qwen:
                    h2 = h2.index_select(0, last)
            if self.qwen:
                y = ops.linear(o, L["wo"], residual=x, want_ssq=True)
                ssq2 = y._edge_ssq
                sv["rs2"] = ops.row_rscale(ssq2, H, cfg.norm_eps)
                # one GEMM: the SwiGLU activation and the saved pre-activations for its rule
                a, sv["gu"] = ops.linear_swiglu_raw(y, t["wgu_n"], norm=(ssq2, cfg.norm_eps))
                x = ops.linear(a, L["wd"], residual=y)
            else:
                a = ops.linear(h2, L["wfc"], L["bfc"])
                sv["a"] = a
                f = ops.linear(h2, L["wfc"], L["bfc"], act="gelu")
                y = ops.linear(o, L["wo"], L["bo"], residual=x)
                x = ops.linear(f, L["wproj"], L["bproj"], residual=y)
            saves.append(sv)
        return emb, x, saves

    def _seed(self, x: torch.Tensor, B: int, S: int):
        """Gradient of ``mx * mx`` w.r.t. the final hidden state (x: the last row of each window, [B, H]) -> (the
        seed gradient [B, H], the seed logits)."""
        m, cfg = self.m, self.m.cfg
        last = x.float()
        w = m.w["norm_w"].float()
        if self.qwen:
            rstd = torch.rsqrt(last.pow(2).mean(-1, keepdim=True) + cfg.norm_eps)
            hN = last * rstd * w
        else:
            xc = last - last.mean(-1, keepdim=True)
            rstd = torch.rsqrt(xc.pow(2).mean(-1, keepdim=True) + cfg.norm_eps)
            hN = xc * rstd * w + m.w["norm_b"].float()
        head = m.w["head"]
        logits = hN @ head.float().t() if head.device.type == "cpu" else (hN.to(head.dtype) @ head.t()).float()
        mx, idx = logits.max(-1)
        dhN = mx.view(-1, 1) * head.index_select(0, idx).float()
        g = dhN * rstd * w
        if not self.qwen:
            g = g - g.mean(-1, keepdim=True)
        return g.to(x.dtype).contiguous(), mx

    @torch.no_grad()
    def head_relevance(self, ids: torch.Tensor, want_channels: bool = False, group: int = 64,
                       want_sens: bool = False):
        """ids [B, S] (B windows of equal length) -> (rel [B, layers, heads] fp32, input relevance [B],
        seed logit [B][, chan [B, layers, H / group]][, sens [B, layers, H / group]]).  rel[b, l, h] = sum_{i,j}
        A_ij dA_ij of head h, layer l, window b; chan (``want_channels``) = sum over tokens and the group's channels
        of |x * dx| of the residual stream entering layer l (as ``attnlrp.head_relevance_batched``); sens
        (``want_sens``) = the groups' quantization sensitivity (``ops.reference.group_sens``)."""
        m, cfg = self.m, self.m.cfg
        ids = ids.to(m.device)
        B, S = ids.shape
        Hq, Hkv = cfg.num_heads, cfg.num_kv_heads
        emb, x, saves = self._forward(ids)
        if saves[-1].get("rows") is None:   # (A/B: the last layer ran on every row) seed its last rows only
            dx, mx = self._seed(x.view(B, S, -1)[:, -1].contiguous(), B, S)
            dx = torch.zeros(B * S, x.shape[1], dtype=dx.dtype, device=dx.device).index_copy_(
                0, torch.arange(B, device=dx.device) * S + (S - 1), dx)
        else:
            dx, mx = self._seed(x, B, S)
        rel = torch.zeros(B, cfg.num_layers, Hq, dtype=torch.float32, device=m.device)
        H = cfg.hidden_size
        chan = torch.zeros(B, cfg.num_layers, H // group, dtype=torch.float32, device=m.device) if want_channels \
            else None
        sens = torch.zeros(B, cfg.num_layers, H // group, dtype=torch.float32, device=m.device) if want_sens else None
        for i in range(cfg.num_layers - 1, -1, -1):
            L, t, sv = m.layers[i], self.T[i], saves[i]
            rows = sv.get("rows")   # last layer: dx is the seeded rows only [B, H]
            if self.qwen:
                dm = ops.linear(dx, t["wdT"])
                dy = ops.linear_rowscale(ops.lrp_swiglu_bwd(dm, sv["gu"]), t["wguT"], sv["rs2"], residual=dx)
            else:
                dh2 = ops.linear(ops.lrp_gelu_bwd(ops.linear(dx, t["wprojT"]), sv["a"]), t["wfcT"])
                dy = dx
            dO = ops.linear(dy, t["woT"])
            if rows is not None:   # back to every row: zero outside the seeded rows
                dO = torch.zeros(B * S, dO.shape[1], dtype=dO.dtype, device=dO.device).index_copy_(0, rows, dO)
                dy = torch.zeros(B * S, H, dtype=dy.dtype, device=dy.device).index_copy_(0, rows, dy)
                if not self.qwen:
                    dh2 = torch.zeros(B * S, H, dtype=dh2.dtype, device=dh2.device).index_copy_(0, rows, dh2)
            _, r, dq, dk, dv = ops.lrp_attn_bwd(sv["q"], sv["k"], sv["v"], sv["o"], dO, sv["lse"])
            rel[:, i] = r
            dqkv = ops.lrp_rope_pack(dq, dk, dv, m.cos, m.sin, B, S, Hq, Hkv, cfg.rotary_dim, m.q_scale,
                                     dtype=dx.dtype)
            if self.qwen:
                dx = ops.linear_rowscale(dqkv, t["wqkvT"], sv["rs1"], residual=dy)
            else:
                dh1 = ops.linear(dqkv, t["wqkvT"])
                dx = ops.lrp_ln_bwd(dh1, sv["rs1"], L["ln1_w"], dh2, sv["rs1"], L["ln2_w"], dy)
            if want_channels:
                chan[:, i] = (sv["x"].float() * dx.float()).abs().view(B, S, H // group, group).sum((1, 3))
            if want_sens:
                sens[:, i] = R.group_sens(sv["x"], dx, B, S, group)
            saves[i] = None
        in_rel = (emb.float() * dx.float()).view(B, S, -1).sum((1, 2))
        return (rel, in_rel, mx) + ((chan,) if want_channels else ()) + ((sens,) if want_sens else ())
