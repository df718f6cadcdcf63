"""``params.json`` configuration.

The reference reads a bare ``params.json`` from the working directory with no
schema, defaults or validation (``Experiments/Pythia-70M/main.py:24-25``,
``Experiments/Qwen2-0.5B/main.py:108-116``, ``Experiments/Relevance/main.py:49-50``).
This module keeps the same file format and keys and adds typed defaults for the
new options (pipeline stages, codec, dtype, synthetic data ...).  Unknown keys
are preserved in ``extra`` and never rejected, so every reference params file
loads unchanged.
"""
from __future__ import annotations

import dataclasses
import hashlib
import json
import os
from dataclasses import dataclass, field
from typing import Any


@dataclass
class Params:
    # ---- reference keys ------------------------------------------------------
    experiment: str = "last_row"            # Pythia: "last_row" | "initial"
    ratios: list = field(default_factory=lambda: [0, 0.25, 0.5, 0.75, 1])
    layers_of_interest: list = field(default_factory=lambda: [2])
    methods: list = field(default_factory=lambda: ["last_row"])
    stride: int = 32
    max_length: int | None = None            # None -> model max_position (Pythia reference behaviour)
    # ---- new keys (defaults reproduce the reference) -------------------------
    model: str = ""                          # preset name, filled by the entry point
    weights: str = ""                        # path to an HF safetensors dir; "" -> HF cache if present, else random
    dataset: str = "wikitext"                # "wikitext" | "synthetic" | "pysrc*"
    strict_data: bool = False                # wikitext requested but not cached locally: error instead of a warning
    synthetic_tokens: int = 0                # length of the synthetic stream (0 -> 299,078, the WikiText-2 test size)
    max_windows: int = 0                     # 0 = whole corpus
    window_batch: int = 0                    # windows per forward batch (0 = auto: 32 on a GPU, 8 on the CPU)
    dtype: str = "auto"                      # "auto" = "fp32" (the reference's precision, CPU and GPU) | "bf16"
    device: str = "auto"                     # "auto" | "cpu" | "cuda"
    codec: str = "ref_int4_global"           # boundary codec used for the ratio sweep (see codec/)
    num_stages: int = 1                      # pipeline stages for the distributed runner
    split_layers: list = field(default_factory=list)   # explicit stage boundaries (last layer of each stage but the last)
    head_weights: str = ""                   # path to attention_head_weights.json (weighted_importance)
    selection: str = "ratio"                 # "ratio" (int(ratio*S) least important) | "top_rho" (mass 1 - ratio kept)
    group_relevance: str = ""                # channel_group_relevance.json (head-group codecs rgroup / mixed_rgroup_int8)
    group_avg_bits: float = 4.0              # head-group codecs: average bits per channel of a group-quantized row
    lrp_engine: str = "auto"                 # relevance pass: "auto" (HIP engine on a GPU, autograd on the CPU) |
                                             # "hip" | "autograd" (AttnLRP rules as torch autograd, any device)
    output_dir: str = "."
    checkpoint_every: int = 1000             # windows between partial-result dumps (reference: 1000)
    resume: bool = True
    seed: int = 0
    extra: dict = field(default_factory=dict)

    @classmethod
    def from_dict(cls, d: dict) -> "Params":
        known = {f.name for f in dataclasses.fields(cls)}
        kw = {k: v for k, v in d.items() if k in known and k != "extra"}
        extra = {k: v for k, v in d.items() if k not in known}
        p = cls(**kw)
        p.extra = extra
        p.validate()
        return p

    @classmethod
    def load(cls, path: str = "params.json", **overrides) -> "Params":
        with open(path) as f:
            d = json.load(f)
        d.update({k: v for k, v in overrides.items() if v is not None})
        return cls.from_dict(d)

    def to_dict(self) -> dict:
        d = dataclasses.asdict(self)
        extra = d.pop("extra")
        d.update(extra)
        return d

    def config_hash(self) -> str:
        d = self.to_dict()
        for k in ("output_dir", "checkpoint_every", "resume"):
            d.pop(k, None)
        return hashlib.sha1(json.dumps(d, sort_keys=True, default=str).encode()).hexdigest()[:12]

    def validate(self) -> None:
        if self.stride <= 0:
            raise ValueError("stride must be positive")
        if self.max_length is not None and self.max_length <= 1:
            raise ValueError("max_length must be > 1")
        for r in self.ratios:
            if not isinstance(r, (int, float)) or r < 0:
                raise ValueError(f"bad ratio {r!r}")
        if self.num_stages < 1:
            raise ValueError("num_stages must be >= 1")
        if self.selection not in ("ratio", "top_rho"):
            raise ValueError(f"selection must be 'ratio' or 'top_rho', got {self.selection!r}")


def resolve_device(p: Params) -> str:
    import torch
    if p.device != "auto":
        return p.device
    return "cuda" if torch.cuda.is_available() else "cpu"


def resolve_window_batch(p: Params, device: str) -> int:
    """``window_batch`` 0 (auto): 32 windows per batch on a GPU (the fp32 notebook sweep runs 59 / 64 / 67 windows/s at
    8 / 16 / 32, larger GEMMs per launch), 8 on the CPU.  Fixed in ``p`` so checkpoints see the resolved value."""
    if p.window_batch <= 0:
        p.window_batch = 32 if str(device).startswith("cuda") else 8
    return p.window_batch


def resolve_dtype(p: Params, device: str):
    import torch
    if p.dtype == "fp32":
        return torch.float32
    if p.dtype == "bf16":
        if not device.startswith("cuda"):
            raise ValueError("dtype bf16 is a GPU execution mode; the CPU path is the fp32 oracle")
        return torch.bfloat16
    if p.dtype != "auto":
        raise ValueError(f"unknown dtype {p.dtype!r} (auto | fp32 | bf16)")
    return torch.float32   # the reference evaluates fp32 models (qwen_layer_wise.py:17: no torch_dtype)


def env_flag(name: str, default: bool = False) -> bool:
    v = os.environ.get(name)
    if v is None:
        return default
    return v not in ("0", "", "false", "False")


def dump_json(obj: Any, path: str) -> None:
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(obj, f, indent=1, default=float)
    os.replace(tmp, path)
