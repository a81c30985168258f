"""Data parallelism over RCCL (xGMI): process bootstrap, flat parameter
storage, bucketed all-reduce overlapped with backward, local launcher."""

from zookeeper_amd.parallel.ddp import GradBucketer, all_reduce_buffers, broadcast_module
from zookeeper_amd.parallel.dist import CommConfig, DistInfo, barrier, info, init, shutdown
from zookeeper_amd.parallel.flat import FlatParams

__all__ = [
    "all_reduce_buffers",
    "barrier",
    "broadcast_module",
    "CommConfig",
    "DistInfo",
    "FlatParams",
    "GradBucketer",
    "info",
    "init",
    "shutdown",
]
