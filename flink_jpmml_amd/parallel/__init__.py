"""Multi-GPU data parallelism over RCCL/xGMI (and gloo for CPU tests)."""

from .dist import (
    DistContext,
    all_gather_scores,
    all_gather_varlen,
    all_to_all_varlen,
    broadcast_control,
    broadcast_object,
    broadcast_plan,
    broadcast_tensors,
    init_from_env,
    shard_range,
    shutdown,
)
from .sinks import GatherSink, gather_varlen
from .tree_shard import TreeShardedScorer, finish_epilogue, host_partial, tree_shard_supported

__all__ = [
    "DistContext", "all_gather_scores", "all_gather_varlen", "all_to_all_varlen", "broadcast_control", "broadcast_object",
    "broadcast_plan", "broadcast_tensors", "init_from_env", "shard_range", "shutdown",
    "GatherSink", "gather_varlen", "TreeShardedScorer", "finish_epilogue", "host_partial", "tree_shard_supported",
]
