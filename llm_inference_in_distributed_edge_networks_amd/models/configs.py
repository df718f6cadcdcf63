"""Model architecture descriptions.

The reference loads its two models through HF ``AutoModelForCausalLM``
(``Experiments/Pythia-70M/pythia_model.py:25``, ``Experiments/Qwen2-0.5B/qwen_layer_wise.py:17``).
Here the architectures are described explicitly so that the framework can build
them without HF at runtime (random init, or weights from a local safetensors
checkpoint).  Dimensions are the ones printed in the reference notebooks
(``Notebooks/qwen2-0.5B_experiment.ipynb`` JSON lines 436-458,
``Notebooks/distributions_distance_across_layers.ipynb`` JSON lines 4452-4472).
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass


@dataclass(frozen=True)
class ModelConfig:
    name: str
    arch: str                     # "qwen2" | "gpt_neox"
    vocab_size: int
    hidden_size: int
    num_layers: int
    num_heads: int
    num_kv_heads: int
    head_dim: int
    intermediate_size: int
    norm_eps: float
    rope_theta: float
    rotary_dim: int               # number of rotated dims per head (partial rotary for GPT-NeoX)
    max_position: int
    tie_embeddings: bool
    parallel_residual: bool = False
    hf_id: str = ""

    @property
    def q_size(self) -> int:
        return self.num_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_kv_heads * self.head_dim

    @property
    def qkv_size(self) -> int:
        return self.q_size + 2 * self.kv_size

    @property
    def group_size(self) -> int:
        return self.num_heads // self.num_kv_heads

    def num_params(self) -> int:
        H, I, V = self.hidden_size, self.intermediate_size, self.vocab_size
        per_layer = H * self.qkv_size + self.q_size * H
        if self.arch == "qwen2":
            per_layer += 3 * H * I + self.qkv_size + 2 * H
        else:
            per_layer += 2 * H * I + self.qkv_size + H + I + H + 4 * H
        head = 0 if self.tie_embeddings else V * H
        return V * H + head + self.num_layers * per_layer

    def replace(self, **kw) -> "ModelConfig":
        return dataclasses.replace(self, **kw)


QWEN2_0_5B = ModelConfig(
    name="qwen2-0.5b", arch="qwen2", vocab_size=151936, hidden_size=896, num_layers=24,
    num_heads=14, num_kv_heads=2, head_dim=64, intermediate_size=4864, norm_eps=1e-6,
    rope_theta=1e6, rotary_dim=64, max_position=32768, tie_embeddings=True,
    hf_id="Qwen/Qwen2-0.5B",
)

PYTHIA_70M = ModelConfig(
    name="pythia-70m", arch="gpt_neox", vocab_size=50304, hidden_size=512, num_layers=6,
    num_heads=8, num_kv_heads=8, head_dim=64, intermediate_size=2048, norm_eps=1e-5,
    rope_theta=10000.0, rotary_dim=16, max_position=2048, tie_embeddings=False,
    parallel_residual=True, hf_id="EleutherAI/pythia-70m",
)

# Small configs with the same structural features (GQA, partial rotary, tied/untied
# head, parallel residual) used by the CPU test-suite.  Every dimension obeys the
# GEMM kernel's tiling contract (N % 128 == 0, K % 64 == 0) so the same configs run
# on the HIP path.
TINY_QWEN2 = ModelConfig(
    name="tiny-qwen2", arch="qwen2", vocab_size=512, hidden_size=256, num_layers=4,
    num_heads=4, num_kv_heads=2, head_dim=64, intermediate_size=512, norm_eps=1e-6,
    rope_theta=1e6, rotary_dim=64, max_position=1024, tie_embeddings=True,
)

TINY_NEOX = ModelConfig(
    name="tiny-neox", arch="gpt_neox", vocab_size=512, hidden_size=256, num_layers=4,
    num_heads=4, num_kv_heads=4, head_dim=64, intermediate_size=1024, norm_eps=1e-5,
    rope_theta=10000.0, rotary_dim=16, max_position=2048, tie_embeddings=False,
    parallel_residual=True,
)

# Byte-level Qwen2-architecture model for the quality experiments (tools/train_tiny_lm.py trains it on local
# text; no pretrained checkpoint is reachable here).  Vocab 512 = 256 byte ids padded to the GEMM tiling.
BYTE_QWEN2 = ModelConfig(
    name="byte-qwen2", arch="qwen2", vocab_size=512, hidden_size=512, num_layers=8,
    num_heads=8, num_kv_heads=2, head_dim=64, intermediate_size=1536, norm_eps=1e-6,
    rope_theta=1e4, rotary_dim=64, max_position=2048, tie_embeddings=True,
)

# The exact Qwen2-0.5B depth and width (24 layers, H 896, 14 / 2 heads, I 4864, rope theta 1e6) with a byte
# vocabulary: the quality experiments at the reference's real boundary depths (layers 3 / 11 / 18 / 22 / 23 of 24,
# Notebooks/qwen2-0.5B_experiment.ipynb) on a model trained here (tools/train_tiny_lm.py), since no checkpoint is
# reachable.
BYTE_QWEN2_24 = ModelConfig(
    name="byte-qwen2-24", arch="qwen2", vocab_size=512, hidden_size=896, num_layers=24,
    num_heads=14, num_kv_heads=2, head_dim=64, intermediate_size=4864, norm_eps=1e-6,
    rope_theta=1e6, rotary_dim=64, max_position=2048, tie_embeddings=True,
)

PRESETS = {c.name: c for c in (QWEN2_0_5B, PYTHIA_70M, TINY_QWEN2, TINY_NEOX, BYTE_QWEN2, BYTE_QWEN2_24)}
ALIASES = {
    "Qwen/Qwen2-0.5B": "qwen2-0.5b", "qwen2": "qwen2-0.5b", "Qwen2-0.5B": "qwen2-0.5b",
    "EleutherAI/pythia-70m": "pythia-70m", "pythia": "pythia-70m", "Pythia-70M": "pythia-70m",
}


def get_config(name: str) -> ModelConfig:
    key = ALIASES.get(name, name)
    if key not in PRESETS:
        raise KeyError(f"unknown model preset {name!r}; known: {sorted(PRESETS)}")
    return PRESETS[key]
