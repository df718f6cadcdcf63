"""MI355X-native split-LLM inference with importance-driven boundary quantization.

A from-scratch gfx950 framework with the capabilities of
``sv-goat/LLM-Inference-in-Distributed-Edge-Networks``: layer-wise split of
Pythia-70M / Qwen2-0.5B across pipeline stages (one process per GPU, RCCL p2p
over xGMI), token-importance scorers (column-mean, last-row, running aggregate,
LRP-weighted heads) and mixed-precision boundary codecs, evaluated with the HF
sliding-window WikiText-2 perplexity recipe.

Sub-packages: ``models`` (architectures, weights), ``ops`` (HIP kernels + fp32
oracle), ``codec`` (boundary wire format), ``importance`` (scorers),
``parallel`` (process groups, p2p, pipeline runtime), ``eval`` (data, PPL,
sweeps), ``relevance`` (AttnLRP head calibration), ``utils``.
"""
__version__ = "0.1.0"

from .utils import poison as _poison  # noqa: E402

_poison.from_env()   # EDGE_POISON=1: NaN / 0xFF-filled torch.empty (uninitialised-read detection)
