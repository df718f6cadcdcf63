"""Parallelism: process groups (RCCL/gloo), stage partitioning and the pipeline runtime."""
from .dist import DistEnv, Grid, all_reduce_sum, barrier, get_env, init_distributed, shutdown
from .pipeline import BoundaryConfig, DistributedPipeline, LocalPipeline, StageRunner
from .plan import PipelinePlan

__all__ = ["DistEnv", "Grid", "all_reduce_sum", "barrier", "get_env", "init_distributed", "shutdown",
           "BoundaryConfig", "DistributedPipeline", "LocalPipeline", "StageRunner", "PipelinePlan"]
