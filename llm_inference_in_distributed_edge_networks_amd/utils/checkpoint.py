"""Resumable sweep state.

The reference pickles running ``total_nll``/``n_tokens`` every 1000 windows but never reads them back
and does not record the window index (``Experiments/Qwen2-0.5B/main.py:184-192``).  ``SweepState``
writes ``{config_hash, windows_done, engine state}`` atomically as JSON (no pickle) and ``load()``
returns it only if the config hash matches, so a restarted job skips completed windows.
"""
from __future__ import annotations

import json
import os


class ShardMismatch(RuntimeError):
    """A checkpoint of this configuration was written under another data-parallel sharding."""


class SweepState:
    def __init__(self, path: str, config_hash: str, enabled: bool = True, shard: tuple | None = None):
        """``shard`` = (rank, world_size, scheme): which windows this rank processes.  Resuming under a different
        sharding would skip windows this rank never saw and count others twice, so it is refused."""
        self.path, self.hash, self.enabled = path, config_hash, enabled
        self.shard = list(shard) if shard is not None else None

    def load(self):
        if not self.enabled or not os.path.exists(self.path):
            return None
        try:
            with open(self.path) as f:
                st = json.load(f)
        except (OSError, json.JSONDecodeError):
            return None
        if st.get("config_hash") != self.hash:
            return None
        if self.shard is not None and st.get("shard") != self.shard:
            raise ShardMismatch(f"{self.path} was written with sharding (rank, world, scheme) = {st.get('shard')}, "
                                f"this run is {self.shard}: resume with the same world size, or delete the "
                                "checkpoints / set resume=false to start over")
        return st

    def save(self, st: dict) -> None:
        if not self.enabled:
            return
        st = dict(st, config_hash=self.hash, shard=self.shard)
        os.makedirs(os.path.dirname(os.path.abspath(self.path)), exist_ok=True)
        tmp = self.path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(st, f)
        os.replace(tmp, self.path)

    def clear(self) -> None:
        if os.path.exists(self.path):
            os.remove(self.path)
