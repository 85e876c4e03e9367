"""Data parallelism over RCCL/xGMI (one process per GPU): process group, bucketed gradient
all-reduce overlapped with backward, rank-sharded data, metric reduction, launcher."""
from .dist import (DistInfo, all_gather_object, all_reduce_, barrier, broadcast_module_, info, init,  # noqa: F401
                   reduce_metrics, shutdown)
from .ddp import GradSync  # noqa: F401
