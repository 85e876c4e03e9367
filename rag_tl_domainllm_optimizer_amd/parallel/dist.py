"""Process-group setup for one-process-per-GPU data parallelism.

``torch.distributed`` with backend "nccl" is RCCL on ROCm (collectives over xGMI between the 8
MI355X of a node); "gloo" is used for CPU runs and the multi-process CPU tests. Rank/world come
from torchrun-style environment variables (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT). The
reference is single-process, single-device (reinforcement_learning_optimization_after_rag.py:166).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: Optional[str] = None
    device: torch.device = torch.device("cpu")

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def enabled(self) -> bool:
        return dist.is_initialized()


_INFO = DistInfo()


def info() -> DistInfo:
    return _INFO


def init(backend: Optional[str] = None, timeout_s: float = 900.0, device: Optional[str] = None,
         force_group: bool = False) -> DistInfo:
    """Initialise from env (no process group for a single process unless ``force_group`` or
    RAGTL_FORCE_PG=1). Sets the current GPU to LOCAL_RANK. The timeout makes a hung collective
    (e.g. a dead peer) surface as an error instead of a silent hang."""
    global _INFO
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_cuda = (device or ("cuda" if torch.cuda.is_available() else "cpu")).startswith("cuda")
    if use_cuda:
        torch.cuda.set_device(local % max(torch.cuda.device_count(), 1))
        dev = torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    # RAGTL_DIST_BACKEND=gloo runs several ranks on one GPU (RCCL needs one GPU per rank): used to
    # rehearse the multi-rank GPU code path on a single-GPU box
    be = backend or os.environ.get("RAGTL_DIST_BACKEND") or ("nccl" if use_cuda else "gloo")
    force_group = force_group or os.environ.get("RAGTL_FORCE_PG", "0") == "1"
    if (world > 1 or force_group) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        kw = dict(backend=be, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if be == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(**kw)
    _INFO = DistInfo(rank, world, local, be if (world > 1 or dist.is_initialized()) else None, dev)
    return _INFO


def barrier():
    if _INFO.enabled:
        if _INFO.backend == "nccl":
            dist.barrier(device_ids=[_INFO.device.index])
        else:
            dist.barrier()


def all_reduce_(t: torch.Tensor, op: str = "sum") -> torch.Tensor:
    if _INFO.enabled:
        dist.all_reduce(t, op={"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op])
    return t


def _is_time_key(k: str) -> bool:
    return k.startswith("time/") or k.endswith("time_s")


def reduce_metrics(values: dict, device=None, max_keys=None) -> dict:
    """Scalar metrics over ranks: the MEAN of every key, except durations (``time/*``, ``*time_s``
    and ``max_keys``), which take the MAX over ranks — a data-parallel step lasts as long as its
    slowest rank, and throughput derived from it must match the bench's max-over-ranks clock.
    Two packed all-reduces (sum, max)."""
    if not _INFO.enabled or not values:
        return dict(values)
    max_keys = set(max_keys or ())
    keys = sorted(values)
    mk = [k for k in keys if _is_time_key(k) or k in max_keys]
    sk = [k for k in keys if k not in set(mk)]
    dev = device or _INFO.device
    out = {}
    if sk:
        vec = torch.tensor([float(values[k]) for k in sk], dtype=torch.float64, device=dev)
        dist.all_reduce(vec)
        vec /= _INFO.world
        out.update(zip(sk, vec.tolist()))
    if mk:
        vec = torch.tensor([float(values[k]) for k in mk], dtype=torch.float64, device=dev)
        dist.all_reduce(vec, op=dist.ReduceOp.MAX)
        out.update(zip(mk, vec.tolist()))
    return {k: float(out[k]) for k in keys}


def broadcast_module_(module: torch.nn.Module, src: int = 0):
    if not _INFO.enabled:
        return
    for p in module.parameters():
        dist.broadcast(p.data, src)


def all_gather_object(obj):
    if not _INFO.enabled:
        return [obj]
    out = [None] * _INFO.world
    dist.all_gather_object(out, obj)
    return out


def allreduce_bandwidth(nbytes: int = 168 << 20, iters: int = 5, warmup: int = 2) -> Optional[dict]:
    """One-shot all-reduce probe on the job's process group: an fp32 tensor of ``nbytes`` (default
    168 MiB, the Mistral-7B LoRA r=16 all-linear gradient payload) summed ``iters``
    times after ``warmup``. Returns the mean time and the algorithm / bus bandwidth (bus = algbw x
    2(N-1)/N, the bytes each rank's links carry in a ring all-reduce); None without a group. On
    RCCL this is the xGMI figure the scaling curve rests on; over gloo it measures the host path."""
    if not _INFO.enabled:
        return None
    import time

    n = max(1, nbytes // 4)
    dev = _INFO.device
    t = torch.ones(n, dtype=torch.float32, device=dev)
    on_gpu = dev.type == "cuda"
    for _ in range(warmup):
        dist.all_reduce(t)
    if on_gpu:
        torch.cuda.synchronize(dev)
    barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        dist.all_reduce(t)
    if on_gpu:
        torch.cuda.synchronize(dev)
    el = torch.tensor([(time.perf_counter() - t0) / iters], dtype=torch.float64, device=dev)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    sec = float(el)
    w = _INFO.world
    algbw = n * 4 / sec
    return {"bytes": n * 4, "time_s": sec, "algbw_GBps": algbw / 1e9, "busbw_GBps": algbw * 2 * (w - 1) / w / 1e9,
            "backend": _INFO.backend, "world": w}


def shutdown():
    if dist.is_initialized():
        dist.destroy_process_group()
