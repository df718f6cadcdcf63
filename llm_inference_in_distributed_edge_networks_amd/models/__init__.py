"""Model zoo: architecture presets and the layer-range executable decoder LM."""
from .configs import (BYTE_QWEN2, PRESETS, PYTHIA_70M, QWEN2_0_5B, TINY_NEOX, TINY_QWEN2, ModelConfig,
                      get_config)
from .model import AttnStats, DecoderLM, build_model, find_hf_snapshot

__all__ = ["BYTE_QWEN2", "PRESETS", "PYTHIA_70M", "QWEN2_0_5B", "TINY_NEOX", "TINY_QWEN2", "ModelConfig", "get_config",
           "AttnStats", "DecoderLM", "build_model", "find_hf_snapshot"]
