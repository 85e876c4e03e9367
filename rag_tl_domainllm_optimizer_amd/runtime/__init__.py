"""Runtime helpers: HIP streams for overlapped phases, event timers, roctx ranges."""
from __future__ import annotations

import contextlib
import time
from collections import defaultdict

import torch


def _roctx():
    try:
        return torch.cuda.nvtx  # maps to roctx on ROCm builds
    except Exception:  # pragma: no cover
        return None


@contextlib.contextmanager
def range_(name: str):
    """roctx range (visible in rocprofv3 --marker-trace) around a phase."""
    nv = _roctx() if torch.cuda.is_available() else None
    if nv is not None:
        try:
            nv.range_push(name)
        except Exception:
            nv = None
    try:
        yield
    finally:
        if nv is not None:
            nv.range_pop()


class PhaseTimer:
    """Phase timer on HIP events: a phase is the device time between an event recorded on the
    current stream when it opens and one recorded when it closes (work the phase waits for on other
    streams, e.g. the reward encoder joined back, is included). Nothing synchronises at phase
    boundaries, so phases overlap freely; ``as_dict`` resolves the pending events (host wall clock
    on CPU-only runs). ``sync=True`` restores the old behaviour (device sync around each phase)."""

    def __init__(self, sync: bool = False, device=None, range_sync: bool = None):
        import os

        self.cuda = torch.cuda.is_available() and (device is None or torch.device(device).type == "cuda")
        self.sync = sync and self.cuda
        # profiling mode (RAGTL_PHASE_SYNC=1): each phase's roctx range closes only after the device
        # has finished the phase's kernels, and the next opens on an idle device, so a trace
        # attributes every kernel to the phase that enqueued it (without it the host runs ahead and
        # e.g. the reference forward's GEMMs execute after its range has closed)
        if range_sync is None:
            range_sync = os.environ.get("RAGTL_PHASE_SYNC", "0") == "1"
        self.range_sync = bool(range_sync) and self.cuda
        self.totals = defaultdict(float)
        self._pending = []

    @contextlib.contextmanager
    def phase(self, name: str):
        if self.sync or self.range_sync:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0 = None
        if self.cuda:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record()
        with range_(name):
            yield
            if self.cuda:
                ev1 = torch.cuda.Event(enable_timing=True)
                ev1.record()
                if self.range_sync:
                    ev1.synchronize()  # inside the range: its kernels are all within it
        if self.cuda:
            if self.sync:
                torch.cuda.synchronize()
            self._pending.append((name, ev0, ev1))
        else:
            self.totals[name] += time.perf_counter() - t0

    def _resolve(self):
        for name, e0, e1 in self._pending:
            e1.synchronize()
            self.totals[name] += e0.elapsed_time(e1) / 1e3
        self._pending.clear()

    def reset(self):
        self._pending.clear()
        self.totals.clear()

    def as_dict(self, prefix: str = "time/"):
        self._resolve()
        return {prefix + k: v for k, v in self.totals.items()}


class StreamPair:
    """A main stream and a side stream (e.g. rollout generation vs reward scoring)."""

    def __init__(self, device=None):
        self.enabled = torch.cuda.is_available() and (device is None or torch.device(device).type == "cuda")
        self.main = torch.cuda.current_stream() if self.enabled else None
        # the side stream is created at the highest priority: HIP maps streams onto a few hardware
        # queues (GPU_MAX_HW_QUEUES), round-robin by creation order among streams of one priority,
        # so a normal-priority side stream can land on the main stream's queue and then waits
        # behind every kernel queued there (no overlap at all); high-priority streams get queues
        # of their own, and the small reward / scoring kernels are the latency-critical ones
        self.side = None
        if self.enabled:
            hi = torch.cuda.Stream.priority_range()[1] if hasattr(torch.cuda.Stream, "priority_range") else -1
            self.side = torch.cuda.Stream(priority=min(hi, 0))

    @contextlib.contextmanager
    def on_side(self, wait: bool = False):
        """Run on the side stream. ``wait=True`` orders it after everything already enqueued on the
        main stream; leave it False when the side work only consumes host-produced inputs (then it
        truly overlaps the main stream's queued kernels)."""
        if not self.enabled:
            yield
            return
        if wait:
            self.side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.side):
            yield

    def join(self):
        if self.enabled:
            torch.cuda.current_stream().wait_stream(self.side)


# ---------------------------------------------------------------------------------------------
# hipGraph capture / replay
# ---------------------------------------------------------------------------------------------
_GRAPH_POOL = {}


def graph_pool(device=None):
    """One graph memory pool per device, shared by every ``GraphRunner`` of the process: the
    rollout decode graph (batch 256) and the RAG-answer decode graph (batch 1) then draw their
    captured intermediates from one reservation instead of one each. Graphs of a shared pool must
    not replay concurrently (they are replayed from one stream here)."""
    dev = torch.device(device or "cuda")
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if idx not in _GRAPH_POOL:
        handle = torch.cuda.graph_pool_handle()
        # a pool lives while some graph captured into it lives: an anchor graph (one tiny kernel)
        # keeps it valid after every generator that used it has been freed
        with torch.cuda.device(idx):
            x = torch.zeros(1, device=f"cuda:{idx}")
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                x.add_(1)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=handle):
                x.add_(1)
        _GRAPH_POOL[idx] = (handle, g, x)
    return _GRAPH_POOL[idx][0]


class GraphRunner:
    """Capture a device-only step once as a hipGraph and replay it (SURVEY T1 ``GraphRunner``).

    ``capture(fn, key, keep, restore)``:
      * runs ``fn`` once eagerly on a side stream first, so lazy allocations (workspaces, folded
        weights, library handles) happen outside the capture;
      * snapshots the tensors in ``restore`` before that warm-up and restores them after the
        warm-up and after the capture (a step that mutates device state must not advance it);
      * captures ``fn`` into a graph on ``pool`` (default: the process-wide ``graph_pool``);
      * keeps a reference to every tensor in ``keep``: a graph reads its inputs through the
        addresses it captured, so a tensor created per call (e.g. an EOS-id list) must live as long
        as the graph, not as long as the call that captured it.
    ``replay()`` launches the graph; ``needs(key)`` says whether a capture with ``key`` is current.
    """

    def __init__(self, pool=None):
        self.pool = pool
        self.graph = None
        self.key = None
        self._keep = ()

    def needs(self, key) -> bool:
        return self.graph is None or self.key != key

    def reset(self):
        self.graph, self.key, self._keep = None, None, ()

    def capture(self, fn, key=None, keep=(), restore=()):
        saved = [t.clone() for t in restore]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()  # warm-up: lazy allocations and caches outside the capture
        torch.cuda.current_stream().wait_stream(s)
        for t, v in zip(restore, saved):
            t.copy_(v)
        g = torch.cuda.CUDAGraph()
        pool = self.pool if self.pool is not None else graph_pool()
        with torch.cuda.graph(g, pool=pool):
            fn()
        for t, v in zip(restore, saved):
            t.copy_(v)
        torch.cuda.synchronize()
        self.graph, self.key, self._keep = g, key, tuple(keep)

    def replay(self):
        self.graph.replay()
