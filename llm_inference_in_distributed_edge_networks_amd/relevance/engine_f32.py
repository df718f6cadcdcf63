"""AttnLRP head relevance at the reference's precision (fp32) on the framework's own kernels.

The reference's calibration (``Experiments/Relevance/main.py:84-103``) is an fp32 forward plus an fp32 backward with
the lxt AttnLRP rules: seed the max logit of the last position with its own value, propagate, and take the
relevance ``A * dA`` summed per head; ``:111-118`` then normalises every layer's heads to sum 1.
``engine.RelevanceEngine`` computes the same quantity with bf16 storage.  This engine keeps every tensor in fp32
and runs every matrix product at fp32 accuracy on the matrix cores:

* forward with saves = the model's fp32 execution mode (``DecoderLM`` with ``h3``): h3 split-fp16 GEMMs
  (csrc/gemm.hip), fp32 attention with its row LSE, fp32 norms; the saved tensors are the fp32 layer inputs, the
  norms' detached row scales, q / k / v / o / LSE and the gate|up (fc) pre-activations;
* backward per layer, in reverse, with no autograd and no S x S tensor:
  - input-gradient GEMMs on the TRANSPOSED weights, on the same h3 GEMM (weights split once at construction;
    the RMSNorm weights applied on those GEMMs' output columns, so a transpose of bf16-valued weights stays exact in
    fp16 and runs on two products).  A gradient has no a-priori bound, so every
    GEMM input row is split with its own power-of-two scale (max |row| just under 2^15) and the GEMM's per-row
    epilogue scale multiplies by the exact inverse - times the detached norm's rstd where a norm sits between;
  - the LRP rules that feed a GEMM (SwiGLU / GELU identity + uniform rules, inverse RoPE + GQA sum) write that
    scaled split directly (csrc/lrp_f32.hip), with the residual add in the GEMM epilogue; the SwiGLU rule runs in
    the epilogue of the GEMM producing its input (dm), at a power-of-two scale from an a-priori bound of the
    weights (``ops.lrp_swiglu_scale``) instead of the row max, which would need every column tile of dm;
  - the attention rule (uniform on Q K^T and A V, plain softmax gradient) on fp32 matrix cores
    (``v_mfma_f32_16x16x4_f32``), emitting rel[b, h] = sum_ij A_ij dA_ij = 0.5 sum_i dO_i . O_i;
  - the channel-group relevance sum |x dx| of the residual stream entering every layer (``group_absprod``).

The seed sits on the last position of each window, so in the LAST layer everything after the attention - O
projection, MLP, their norms - matters at those B rows only, forward and backward (the other rows' output
relevance is exactly zero): that layer runs them on the gathered rows and scatters dO / dy back (as
``DecoderLM.layer_rows`` does for the scored rows of the NLL path).

CPU tensors run the same sequence on the PyTorch reference ops (the model must then be built with ``h3=True``);
the tests check it against the autograd oracle ``attnlrp.head_relevance_batched``.
"""
from __future__ import annotations


import torch

from .. import ops
from ..models.model import DecoderLM



class RelevanceEngineH3:
    def __init__(self, model: DecoderLM):
        self.m = model
        cfg = model.cfg
        if not model.h3:
            raise ValueError("RelevanceEngineH3 needs a model in the fp32 (h3) execution mode")
        if cfg.head_dim != 64:
            raise ValueError("relevance engine is specialised for head_dim 64")
        if any(L is None for L in model.layers) or model.w.get("embed") is None or model.w.get("head") is None:
            raise ValueError("relevance engine needs the whole model resident")
        self.qwen = cfg.arch == "qwen2"
        R = ops.reference

        def t3(w):
            w3, s = R.h3_weight(w.t().contiguous())
            return w3, 1.0 / s
        self.T = []
        for L in model.layers:
            t = {}
            if self.qwen:
                # the RMSNorm weights stay out of the transposes (applied on the GEMMs' output columns, colscale):
                # the transposes of bf16 / fp16-valued weights are then exact in fp16 - two products, not three
                t["wqkvT3"], t["a_qkvT"] = t3(L["wqkv"])
                t["wguT3"], t["a_guT"] = t3(L["wgu"])
                t["wdT3"], t["a_dT"] = t3(L["wd"])
                t["c_swiglu"] = ops.lrp_swiglu_scale(L["wd"], L["wgu"], L["ln2_w"])
                # bound of the gate|up input-gradient GEMM's product per unit of its input row scale:
                # max_c |norm_w[c]| sum_k |W[k, c]| (dy's h3 planes come from that GEMM's epilogue)
                t["c_gu"] = float((L["wgu"].float().abs().sum(0) * L["ln2_w"].float().abs()).max())
            else:
                t["wqkvT3"], t["a_qkvT"] = t3(L["wqkv"])
                t["wfcT3"], t["a_fcT"] = t3(L["wfc"])
                t["wprojT3"], t["a_projT"] = t3(L["wproj"])
            t["woT3"], t["a_oT"] = t3(L["wo"])
            self.T.append(t)

    # ------------------------------------------------------------------------------------------------
    def _forward(self, ids: torch.Tensor):
        m, cfg = self.m, self.m.cfg
        B, S = ids.shape
        Hq, Hkv, D, eps = cfg.num_heads, cfg.num_kv_heads, cfg.head_dim, cfg.norm_eps
        x = m.embed(ids)
        emb = x
        saves = []
        last = torch.arange(B, device=ids.device) * S + (S - 1)   # the seeded rows
        nl = len(m.layers)
        for i, L in enumerate(m.layers):
            sc = m.h3_layer[i]
            sv = {"x": x}
            if self.qwen:   # the norms' own row normalisers, saved detached (no separate row_rstd pass)
                sv["rs1"] = torch.empty(x.shape[0], dtype=torch.float32, device=x.device)
                h13 = ops.rmsnorm(x, L["ln1_w"], eps, h3=sc["qkv"], rstd_out=sv["rs1"])
            else:
                sv["rs1"] = ops.row_rstd(x, eps, center=True)
                h13, h23 = ops.layernorm_dual(x, L["ln1_w"], L["ln1_b"], L["ln2_w"], L["ln2_b"], eps,
                                              h3=(sc["qkv"], sc["mlp"]))
            # the QKV epilogue also writes the K / V^T planes the attention stages by LDS DMA and V row-major for the
            # backward (no transpose pass)
            q, k, vt, kp, vp, v = ops.qkv_rope_h3(h13, L["wqkv3"], sc["a_wqkv"], L["bqkv"], m.cos, m.sin, B, S, Hq,
                                                  Hkv, D, cfg.rotary_dim, m.q_scale, kv_scales=(sc["att_k"], sc["o"]),
                                                  v_rows=True)
            # O as the O-projection's h3 planes and, for the backward, as fp32 rows - both from the attention kernel
            o3, lse, o = ops.attention(q, k, vt, S, need_lse=True, h3=sc["o"],
                                       in_scales=(sc["att_q"], sc["att_k"], sc["o"]),
                                       kv_planes=(kp, vp) if q.is_cuda else None, f32_out=True)
            sv.update(q=q, k=k, v=v, o=o, lse=lse.contiguous())
            if i == nl - 1:   # only the seeded rows reach the seed: O-proj and MLP on those rows
                sv["rows"] = last
                x = x.index_select(0, last)
                if not self.qwen:
                    h23 = h23.index_select(0, last)
                o3 = o3.index_select(0, last)
            if self.qwen:
                y = ops.linear_h3(o3, L["wo3"], sc["a_wo"], residual=x)
                sv["rs2"] = torch.empty(y.shape[0], dtype=torch.float32, device=y.device)
                h23 = ops.rmsnorm(y, L["ln2_w"], eps, h3=sc["mlp"], rstd_out=sv["rs2"])
                # one GEMM: the SwiGLU planes for the down projection and the saved pre-activations for its rule
                a3, sv["gu"] = ops.linear_h3_swiglu_raw(h23, L["wgu3"], sc["a_wgu"], sc["down"])
                x = ops.linear_h3(a3, L["wd3"], sc["a_wd"], residual=y)
            else:
                y = ops.linear_h3(o3, L["wo3"], sc["a_wo"], L["bo"], residual=x)
                a = ops.linear_h3(h23, L["wfc3"], sc["a_wfc"], L["bfc"])
                sv["a"] = a
                x = ops.linear_h3(ops.act_h3(a, "gelu", sc["down"]), L["wproj3"], sc["a_wproj"], L["bproj"],
                                  residual=y)
            saves.append(sv)
        return emb, x, saves

    def _seed(self, x: torch.Tensor, B: int, S: int):
        """d(mx * mx) / d x_final with the final norm's normaliser detached: only the last row of each window
        (x_final is already those rows, [B, H]) -> (the seed gradient [B, H], the seed logits)."""
        m, cfg = self.m, self.m.cfg
        last = x
        w = m.w["norm_w"]
        if self.qwen:
            rstd = ops.row_rstd(last, cfg.norm_eps)
            hN = last * rstd.view(-1, 1) * w
        else:
            rstd = ops.row_rstd(last, cfg.norm_eps, center=True)
            hN = (last - last.mean(-1, keepdim=True)) * rstd.view(-1, 1) * w + m.w["norm_b"]
        hs = m.h3_head
        logits = ops.linear_h3(ops.split_h3(hN.contiguous(), hs["s"]), m.w["head3"], hs["a"])
        mx, idx = logits.max(-1)
        g = mx.view(-1, 1) * m.w["head"].index_select(0, idx) * rstd.view(-1, 1) * w
        if not self.qwen:
            g = g - g.mean(-1, keepdim=True)
        return g.contiguous(), mx

    @torch.no_grad()
    def head_relevance(self, ids: torch.Tensor, want_channels: bool = False, group: int = 64,
                       want_sens: bool = False):
        """ids [B, S] -> (rel [B, layers, heads], input relevance [B], seed logit [B][, chan [B, layers, H/64]]
        [, sens [B, layers, H/64]]), all fp32; the same quantities as ``attnlrp.head_relevance_batched``."""
        if group != 64:
            raise ValueError("channel groups are 64 channels (one head) wide")
        m, cfg = self.m, self.m.cfg
        ids = ids.to(m.device)
        B, S = ids.shape
        Hq, Hkv, H = cfg.num_heads, cfg.num_kv_heads, cfg.hidden_size
        emb, x, saves = self._forward(ids)
        if saves[-1].get("rows") is None:   # (A/B: the last layer ran on every row) seed its last rows only
            dx, mx = self._seed(x.view(B, S, -1)[:, -1].contiguous(), B, S)
            dx = torch.zeros(B * S, x.shape[1], dtype=dx.dtype, device=dx.device).index_copy_(
                0, torch.arange(B, device=dx.device) * S + (S - 1), dx)
        else:
            dx, mx = self._seed(x, B, S)
        rel = torch.zeros(B, cfg.num_layers, Hq, dtype=torch.float32, device=m.device)
        chan = torch.zeros(B, cfg.num_layers, H // group, dtype=torch.float32, device=m.device) \
            if (want_channels or want_sens) else None
        sens = torch.zeros(B, cfg.num_layers, H // group, dtype=torch.float32, device=m.device) if want_sens else None
        for i in range(cfg.num_layers - 1, -1, -1):
            L, t, sv = m.layers[i], self.T[i], saves[i]
            rows = sv.get("rows")   # last layer: dx is the seeded rows only [B, H]
            dx3, rinv = ops.split_h3_dyn(dx)
            if self.qwen:
                # dm GEMM + SwiGLU rule in one kernel (the rule's planes at the weights' a-priori bound)
                dgu3, rinv_gu = ops.linear_h3_lrp_swiglu(dx3, t["wdT3"], t["a_dT"], sv["gu"], t["c_swiglu"], rinv,
                                                         post=sv["rs2"])
                # dy and its h3 planes in one GEMM: |dy| <= |dx| + rinv_gu 2^15 c_gu, |dx| < 2^15 rinv
                dy, dy3, rinv_y = ops.linear_h3(dgu3, t["wguT3"], t["a_guT"], rscale=rinv_gu, residual=dx,
                                                colscale=L["ln2_w"], planes_bound=(rinv, rinv_gu, t["c_gu"]))
            else:
                dp = ops.linear_h3(dx3, t["wprojT3"], t["a_projT"], rscale=rinv)
                dfc3, rinv_fc = ops.lrp_gelu_bwd_h3(dp, sv["a"])
                dh2 = ops.linear_h3(dfc3, t["wfcT3"], t["a_fcT"], rscale=rinv_fc)
                dy, dy3, rinv_y = dx, dx3, rinv           # parallel residual: the attention branch sees dx
            dO = ops.linear_h3(dy3, t["woT3"], t["a_oT"], rscale=rinv_y)
            if rows is not None:   # back to every row: zero outside the seeded rows
                dO = torch.zeros(B * S, dO.shape[1], dtype=dO.dtype, device=dO.device).index_copy_(0, rows, dO)
                dy = torch.zeros(B * S, H, dtype=dy.dtype, device=dy.device).index_copy_(0, rows, dy)
                if not self.qwen:
                    dh2 = torch.zeros(B * S, H, dtype=dh2.dtype, device=dh2.device).index_copy_(0, rows, dh2)
            # dk, dv summed over each GQA group in the kernel where it can (else the per-q-head partials)
            sc = m.h3_layer[i]   # the forward attention's plane scales: the sweeps run on the same scaled fp16 planes
            _, r, dq, dk, dv = ops.lrp_attn_bwd(sv["q"], sv["k"], sv["v"], sv["o"], dO, sv["lse"],
                                                gqa_sum=ops.lrp_gqa_sum_native(sv["q"]),
                                                in_scales=(sc["att_q"], sc["att_k"], sc["o"]))
            rel[:, i] = r
            dqkv3, rinv_q = ops.lrp_rope_pack_h3(dq, dk, dv, m.cos, m.sin, B, S, Hq, Hkv, cfg.rotary_dim, m.q_scale,
                                                 post=sv["rs1"] if self.qwen else None)
            if self.qwen:
                # (dx is re-split from its own row maxima at the next layer: bound-derived scales would compound -
                # rinv_q, rinv_gu are themselves a-priori bounds - and lose the planes' range within a few layers)
                dx = ops.linear_h3(dqkv3, t["wqkvT3"], t["a_qkvT"], rscale=rinv_q, residual=dy, colscale=L["ln1_w"])
            else:
                dh1 = ops.linear_h3(dqkv3, t["wqkvT3"], t["a_qkvT"], rscale=rinv_q)
                dx = ops.lrp_ln_bwd_f32(dh1, sv["rs1"], L["ln1_w"], dh2, L["ln2_w"], dy)
            if want_channels or want_sens:
                ops.group_absprod(sv["x"], dx, B, S, out=chan[:, i], sens_out=None if sens is None else sens[:, i])
            saves[i] = None
        in_rel = (emb * dx).view(B, -1).sum(1)
        return (rel, in_rel, mx) + ((chan,) if want_channels else ()) + ((sens,) if want_sens else ())
