"""Boundary codecs: what crosses a pipeline-stage boundary and how it is quantized.

The reference only *simulates* the device boundary with in-place fake
quantization of ``hidden_states`` after layer ``layer_of_interest``
(Q1 ``Experiments/Qwen2-0.5B/qwen_layer_wise.py:54-70``, Q5/Q6
``qwen_layer_wise.py:106-152``, Q2/Q4 ``Experiments/Pythia-70M/pythia_model.py:57-68,116-145``).
Here every boundary produces a real, self-describing byte message
(``wire.py``) that is shipped with RCCL ``send``/``recv`` between stages and
decoded on the receiving GPU; fake quantization is simply ``decode(encode(x))``.

Codecs (``CODECS``):

=====================  ==============  ==============  ===========  ==================================
name                   hi class        lo class        scales       reference
=====================  ==============  ==============  ===========  ==================================
passthrough            native dtype    --              --           no quantization (ratio 0)
ref_int4_global        native dtype    int4 [-8,7]     per window   Q1 (one global max-abs scale)
int4_token             native dtype    int4 [-7,7]     per token    Q1 with per-token scales
int8_token             int8            --              per token    BASELINE config 2 (uniform int8)
mixed_int4_int8        int8            int4            per token    BASELINE configs 3-5
mixed_int2_int8        int8            int2 ternary    per token    extra compression point
channel_8 / channel_4  int8 / int4     --              per channel  Q5
channel_1_mean/_max    int2 ternary    --              per channel  Q6
int8_token_keep        native dtype    int8            per token    Q2/Q4 (Pythia 'initial', intended semantics)
mxfp4 / mxfp8          MXFP4 / MXFP8   --              E8M0 / 32ch  OCP microscaling, every token (gfx950
                                                                    scaled converts)
mixed_mxfp4_mxfp8      MXFP8 (E4M3)    MXFP4 (E2M1)    E8M0 / 32ch  configs 3-5 at microscaling widths
mxfp4_keep             native dtype    MXFP4           E8M0 / 32ch  Q1 with MX blocks instead of one scale
rgroup                 head groups     --              per group    every 64-channel group (one head) its
                                                                    own max-abs scale and 2/4/8-bit width
mixed_rgroup_int8      int8            head groups     token/group  config 5 (relevance-allocated widths
                                                                    from channel_group_relevance.json)
=====================  ==============  ==============  ===========  ==================================

Head-group codecs carry their group bit plan in the message; a boundary's plan comes from
``wire.allocate_group_bits`` over the LRP relevance of its 64-channel groups (uniform without a table).

"hi"/"lo" classes: the ``k = int(ratio * S)`` least important tokens of a
window (ascending importance, ties broken by position) are the lo class.
"""
from .wire import (CODECS, CodecSpec, Layout, decode, encode, fake_quant, get_codec, layout, message_bytes,
                   select_mask)

__all__ = ["CODECS", "CodecSpec", "Layout", "decode", "encode", "fake_quant", "get_codec", "layout",
           "message_bytes", "select_mask"]
