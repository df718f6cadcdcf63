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
=====================  ==============  ==============  ===========  ==================================

"hi"/"lo" classes: the ``k = int(ratio * S)`` least important tokens of a
window (ascending importance, ties broken by position) are the lo class.
"""
from .wire import (CODECS, CodecSpec, Layout, decode, encode, fake_quant, get_codec, layout, message_bytes,
                   select_mask)

__all__ = ["CODECS", "CodecSpec", "Layout", "decode", "encode", "fake_quant", "get_codec", "layout",
           "message_bytes", "select_mask"]
