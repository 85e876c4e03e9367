"""Data-parallel gradient synchronisation over a flat gradient buffer.

Trainable parameters live in one flat fp32 buffer (:class:`ops.FlatParams`; bf16 + fp32 buffers
for full-parameter training, :class:`ops.MixedFlatParams`), ordered as the model
runs forward, so backward produces gradients from the END of the buffer towards its start. The
buffer is cut into contiguous buckets; a post-accumulate-grad hook counts ready parameters and, as
soon as a bucket is complete, launches an asynchronous all-reduce (RCCL over xGMI on GPU) of that
slice while backward keeps computing earlier layers. ``finish()`` waits for the outstanding
buckets and averages.

Bucket sizing for xGMI: a ring all-reduce moves 2(N-1)/N x bytes through each link; LoRA grads are
latency-bound (tens to ~170 MB), so a few large buckets (default 64 MB) amortise the per-collective
latency while still leaving the last buckets to overlap with the tail of backward.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from .dist import info


class GradSync:
    def __init__(self, flat, bucket_bytes: int = 64 << 20, overlap: bool = True):
        self.flat = flat
        self.world = info().world
        self.enabled = info().enabled
        self.gloo = self.enabled and dist.get_backend() == "gloo"
        self.overlap = overlap and self.enabled
        n = flat.numel
        per = max(1, bucket_bytes // 4)
        # buckets aligned to parameter boundaries, built from the END of the buffer (the order in
        # which backward produces gradients); bucket 0 = last parameters
        offs = list(flat.offsets) + [n]
        self.param_bucket = [0] * len(flat.params)
        bounds = []
        cur_end = None
        cur_start = None
        for idx in reversed(range(len(flat.params))):
            s_, e_ = offs[idx], offs[idx + 1]
            if cur_end is None:
                cur_end = e_
            cur_start = s_
            self.param_bucket[idx] = len(bounds)
            if cur_end - cur_start >= per:
                bounds.append((cur_start, cur_end))
                cur_end = None
        if cur_end is not None:
            bounds.append((cur_start, cur_end))
        self.buckets = bounds
        self.need = [0] * len(bounds)
        for bi in self.param_bucket:
            self.need[bi] += 1
        self._ready = [0] * len(bounds)
        self._handles: List[Optional[object]] = [None] * len(bounds)
        self._hooks = []
        self.sync_enabled = True
        self.wait_s = 0.0  # host time blocked in finish() (exposed all-reduce tail), reset by the caller
        if self.overlap:
            for p, bi in zip(flat.params, self.param_bucket):
                self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(bi)))

    def _make_hook(self, bi):
        def hook(_p):
            if not self.sync_enabled:
                return
            self._ready[bi] += 1
            if self._ready[bi] == self.need[bi] and self._handles[bi] is None:
                self._launch(bi)
        return hook

    def _launch(self, bi):
        s, e = self.buckets[bi]
        hs = []
        # one slice per gradient buffer the bucket touches (fp32, or bf16 + fp32 under full-parameter
        # training: ops.MixedFlatParams); RCCL reduces bf16 in place, 2 B per weight over xGMI
        for t in self.flat.grad_slices(s, e):
            if t.dtype == torch.bfloat16 and (not t.is_cuda or self.gloo):
                # gloo (CPU runs, and the one-GPU multi-rank rehearsal): reduce an fp32 copy of a
                # bf16 slice. RCCL reduces bf16 in place (2 B per weight over xGMI); its ring sums
                # in bf16, which the full-fine-tuning DP tests bound (docs/DESIGN.md)
                f = t.float()
                dist.all_reduce(f)
                t.copy_(f)
            else:
                hs.append(dist.all_reduce(t, async_op=True))
        self._handles[bi] = hs

    def no_sync(self):
        """Context manager: accumulate gradients locally (micro-batches before the last one)."""
        import contextlib

        @contextlib.contextmanager
        def cm():
            prev = self.sync_enabled
            self.sync_enabled = False
            try:
                yield
            finally:
                self.sync_enabled = prev
        return cm()

    def start(self):
        self._ready = [0] * len(self.buckets)
        self._handles = [None] * len(self.buckets)

    def finish(self):
        """Complete all buckets (launch the ones whose hooks did not fire) and average."""
        if not self.enabled:
            return
        import time

        t0 = time.perf_counter()
        self.flat.relink_grads()
        for bi in range(len(self.buckets)):
            if self._handles[bi] is None:
                self._launch(bi)
        for hs in self._handles:
            for h in hs:
                h.wait()
        self.flat.div_grads(self.world)
        self.wait_s += time.perf_counter() - t0
        self._handles = [None] * len(self.buckets)
        self._ready = [0] * len(self.buckets)

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
