"""Process-group setup and point-to-point helpers (one process per GPU).

The reference has no distributed code at all (the device
boundary is simulated in one process).  Here each pipeline stage is its own
process: ``torch.distributed`` with backend ``"nccl"`` (RCCL on ROCm, over xGMI)
for GPU ranks, ``"gloo"`` for CPU ranks (tests).  Launch with
``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ...``.

Failure handling: the process group gets a finite timeout, so a
dead peer turns into an exception on every survivor instead of a hang; the
evaluation loop checkpoints per-window progress so a restarted job resumes.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistEnv:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: torch.device = torch.device("cpu")

    @property
    def is_dist(self) -> bool:
        return self.world_size > 1

    @property
    def is_main(self) -> bool:
        return self.rank == 0


_ENV: DistEnv | None = None


def init_distributed(device: str = "auto", timeout_s: float = 600.0) -> DistEnv:
    """Initialise from torchrun env vars (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*); no-op for 1 process."""
    global _ENV
    if _ENV is not None:
        return _ENV
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_cuda = (device == "cuda") or (device == "auto" and torch.cuda.is_available())
    # EDGE_SHARED_GPU=1: every rank on cuda:0 with a gloo process group and host-staged p2p - a rehearsal of
    # the multi-GPU code path (CUDA tensors, graphs, pipeline protocol) on a one-GPU machine.  RCCL refuses
    # two ranks on one device, so this is never the production path.
    shared = use_cuda and os.environ.get("EDGE_SHARED_GPU", "0") not in ("", "0")
    if use_cuda:
        local_dev = 0 if shared else local
        torch.cuda.set_device(local_dev)
        dev = torch.device("cuda", local_dev)
    else:
        dev = torch.device("cpu")
    backend = "none"
    if world > 1:
        backend = "nccl" if (use_cuda and not shared) else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if not dist.is_initialized():
            kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
            if backend == "nccl":
                kw["device_id"] = dev
            dist.init_process_group(**kw)
    _ENV = DistEnv(rank, world, local, backend, dev)
    return _ENV


def get_env() -> DistEnv:
    return _ENV if _ENV is not None else DistEnv()


def shutdown() -> None:
    global _ENV
    if dist.is_available() and dist.is_initialized():
        try:
            dist.barrier()
        except Exception:
            pass
        dist.destroy_process_group()
    _ENV = None


def barrier() -> None:
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def _all_reduce(t: torch.Tensor, op, group=None) -> torch.Tensor:
    if dist.is_available() and dist.is_initialized():
        if t.is_cuda and dist.get_backend(group) == "gloo":   # EDGE_SHARED_GPU rehearsal: host-staged
            h = t.cpu()
            dist.all_reduce(h, op=op, group=group)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=op, group=group)
    return t


def all_reduce_sum(t: torch.Tensor, group=None) -> torch.Tensor:
    return _all_reduce(t, dist.ReduceOp.SUM, group)


def all_reduce_max_(t: torch.Tensor, group=None) -> torch.Tensor:
    return _all_reduce(t, dist.ReduceOp.MAX, group)


def all_reduce_max(x: float) -> float:
    if not (dist.is_available() and dist.is_initialized()):
        return x
    env = get_env()
    t = torch.tensor([x], dtype=torch.float64, device=env.device if env.backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def broadcast_object(obj, src: int = 0):
    if not (dist.is_available() and dist.is_initialized()):
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=src)
    return lst[0]


def isend(t: torch.Tensor, dst: int, group=None):
    return dist.isend(t, dst, group=group)


def irecv(t: torch.Tensor, src: int, group=None):
    return dist.irecv(t, src, group=group)


@dataclass(frozen=True)
class Grid:
    """rank -> (data-parallel replica, pipeline stage); stages of a replica are consecutive ranks."""
    world: int
    pp: int

    def __post_init__(self):
        if self.world % self.pp:
            raise ValueError(f"world size {self.world} not divisible by pp={self.pp}")

    @property
    def dp(self) -> int:
        return self.world // self.pp

    def coords(self, rank: int) -> tuple[int, int]:
        return rank // self.pp, rank % self.pp

    def rank_of(self, dp_idx: int, stage: int) -> int:
        return dp_idx * self.pp + stage
