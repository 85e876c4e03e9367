"""Data parallelism over RCCL/xGMI (one process per GPU): process group, bucketed gradient
all-reduce overlapped with backward, rank-sharded data, metric reduction, launcher."""
from .dist import (DistInfo, all_gather_object, all_reduce_, allreduce_bandwidth, barrier,  # noqa: F401
                   broadcast_module_, info, init, reduce_metrics, shutdown)
from .launch import self_launch  # noqa: F401
from .ddp import GradSync  # noqa: F401
