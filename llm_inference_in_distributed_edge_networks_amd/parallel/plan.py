"""Layer partitioning into pipeline stages.

The reference's split is a single layer index ``layer_of_interest``
(``qwen_layer_wise.py:54``): stage 1 = layers ``0..L``, stage 2 = ``L+1..end``.
``PipelinePlan`` generalises it to N contiguous stages.  Explicit boundaries come
from ``split_layers`` (the last layer of every stage but the last, i.e. the
reference's ``layer_of_interest`` values); otherwise a cost model balances the
stages: one unit per decoder layer, plus the LM head of the last stage computed
on the scored rows only (``scored_fraction`` = trg_len/S, 32/512 for the
reference recipe) and the embedding gather of the first stage (~free).
"""
from __future__ import annotations

from dataclasses import dataclass

from ..models.configs import ModelConfig


def layer_flops(cfg: ModelConfig, S: int) -> float:
    H, I = cfg.hidden_size, cfg.intermediate_size
    mlp = (3 if cfg.arch == "qwen2" else 2) * H * I
    proj = H * cfg.qkv_size + cfg.q_size * H
    attn = 2 * S * cfg.q_size  # causal QK^T + PV per token (halved)
    return 2.0 * (mlp + proj + attn)


def head_flops(cfg: ModelConfig, scored_fraction: float) -> float:
    return 2.0 * cfg.hidden_size * cfg.vocab_size * scored_fraction


@dataclass(frozen=True)
class PipelinePlan:
    num_layers: int
    bounds: tuple  # bounds[s] = first layer of stage s; bounds[-1] = num_layers

    @property
    def num_stages(self) -> int:
        return len(self.bounds) - 1

    def stage_layers(self, s: int) -> range:
        return range(self.bounds[s], self.bounds[s + 1])

    def boundary_layers(self) -> list[int]:
        """Last layer of every stage but the last: the reference's ``layer_of_interest`` values."""
        return [self.bounds[s + 1] - 1 for s in range(self.num_stages - 1)]

    @classmethod
    def from_split_layers(cls, num_layers: int, split_layers) -> "PipelinePlan":
        sl = sorted(int(x) for x in split_layers)
        if any(not 0 <= x < num_layers - 1 for x in sl) or len(set(sl)) != len(sl):
            raise ValueError(f"bad split layers {split_layers} for {num_layers} layers")
        return cls(num_layers, tuple([0] + [x + 1 for x in sl] + [num_layers]))

    @classmethod
    def balanced(cls, cfg: ModelConfig, num_stages: int, S: int = 512, scored_fraction: float = 32 / 512):
        n = cfg.num_layers
        if not 1 <= num_stages <= n:
            raise ValueError(f"cannot split {n} layers into {num_stages} stages")
        lf = layer_flops(cfg, S)
        head = head_flops(cfg, scored_fraction) / lf   # in layer units
        # exact min-max contiguous partition (n <= a few dozen): DP over (layers, stages)
        import functools

        @functools.lru_cache(maxsize=None)
        def best(start: int, stages: int):
            if stages == 1:
                return (n - start + head, (n,))
            res = None
            for end in range(start + 1, n - stages + 2):
                sub_cost, sub_b = best(end, stages - 1)
                cost = max(end - start, sub_cost)
                if res is None or cost < res[0] - 1e-9:
                    res = (cost, (end,) + sub_b)
            return res

        _, b = best(0, num_stages)
        return cls(n, tuple([0] + list(b)))
