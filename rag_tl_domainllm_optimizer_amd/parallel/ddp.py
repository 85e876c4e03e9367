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

bf16 gradient slices (full-parameter training, ``ops.MixedFlatParams``) are NOT summed in bf16: a
ring all-reduce rounds the running sum to 8 significant bits at every hop (about 3 bits lost at
world 8). Mode ``"rs32"`` (default): the slice is widened to an fp32 staging buffer and
reduce-scattered in fp32 (overlapped with backward, (N-1)/N x 4 B per weight), each rank rounds its
summed shard to bf16 once, and a bf16 all-gather ((N-1)/N x 2 B) completes it in ``finish()`` —
6 B of link traffic per weight against 4 B for a bf16 all-reduce and 8 B for an fp32 one, with a
single rounding. ``"bf16"`` keeps the in-place bf16 all-reduce (RAGTL_BF16_REDUCE=bf16). Memory: each
bucket in flight holds a padded fp32 staging copy plus its fp32 shard (~(1 + 1/N) x 4 B per weight
of the bucket); at most ``rs32_inflight`` (default 2, RAGTL_RS32_INFLIGHT) are alive at once.
"""
from __future__ import annotations

from typing import List, Optional

import os

import torch
import torch.distributed as dist

from .dist import info


class GradSync:
    def __init__(self, flat, bucket_bytes: int = 64 << 20, overlap: bool = True, bf16_reduce: str = None):
        self.flat = flat
        self.bf16_reduce = bf16_reduce or os.environ.get("RAGTL_BF16_REDUCE", "rs32")
        assert self.bf16_reduce in ("rs32", "bf16"), self.bf16_reduce
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
        self.comm_bytes = 0  # payload bytes handed to collectives (per rank), reset by the caller
        self._stage1 = []    # rs32 buckets in flight: (bf16 slice, fp32 shard out, handle, fp32 staging buffer)
        self._stage2 = []    # rs32 buckets reduced and rounded: (bf16 slice, bf16 summed shard)
        # at most this many fp32 staging buffers stay alive: launching another first retires the
        # oldest (wait, round its shard to bf16, drop both fp32 buffers), so full-parameter DP holds
        # ~2 buckets of fp32 staging at the end of backward instead of 2x the whole bf16 gradient
        # (~28 GB for a 7B model)
        self.rs32_inflight = max(1, int(os.environ.get("RAGTL_RS32_INFLIGHT", "2")))
        if self.overlap:
            for p, bi in zip(flat.params, self.param_bucket):
                # also fires when a backward accumulated straight into .grad and returned None
                # (the LoRA epilogue, ops.linear._linear_bwd): AccumulateGrad still runs
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
        # training: ops.MixedFlatParams)
        for t in self.flat.grad_slices(s, e):
            if t.dtype == torch.bfloat16 and (self.bf16_reduce == "rs32" or not t.is_cuda or self.gloo):
                hs.append(self._rs32(t))
            else:
                self.comm_bytes += t.numel() * t.element_size()
                hs.append(dist.all_reduce(t, async_op=True))
        self._handles[bi] = hs

    def _rs32(self, t: torch.Tensor):
        """Stage 1 of the fp32 reduction of a bf16 slice: widen into a padded fp32 buffer and
        reduce-scatter it (async). Stage 2 (round the shard once, bf16 all-gather) runs in finish()."""
        while len(self._stage1) >= self.rs32_inflight:
            self._retire_oldest()
        w = self.world
        n = t.numel()
        shard = (n + w - 1) // w
        buf = torch.zeros(shard * w, dtype=torch.float32, device=t.device)
        buf[:n].copy_(t)
        out = torch.empty(shard, dtype=torch.float32, device=t.device)
        self.comm_bytes += buf.numel() * 4
        h = dist.reduce_scatter_tensor(out, buf, async_op=True)
        self._stage1.append((t, out, h, buf))
        return _Done()

    def _retire_oldest(self):
        t, out, h, _buf = self._stage1.pop(0)
        h.wait()  # on RCCL a stream dependency, not a host wait
        self._stage2.append((t, out.to(torch.bfloat16)))  # the ONE rounding of the fp32 sum

    def _finish_rs32(self):
        while self._stage1:
            self._retire_oldest()
        if not self._stage2:
            return
        w = self.world
        gathers = []
        for t, shard16 in self._stage2:
            full = torch.empty(shard16.numel() * w, dtype=torch.bfloat16, device=t.device)
            self.comm_bytes += full.numel() * 2
            gathers.append((t, full, dist.all_gather_into_tensor(full, shard16, async_op=True)))
        for t, full, h in gathers:
            h.wait()
            t.copy_(full[:t.numel()])
        self._stage2 = []

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
        self._finish_rs32()
        self.flat.div_grads(self.world)
        self.wait_s += time.perf_counter() - t0
        self._handles = [None] * len(self.buckets)
        self._ready = [0] * len(self.buckets)

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []


class _Done:
    """Handle of a collective whose completion finish() tracks elsewhere (rs32 stage 2)."""

    def wait(self):
        return True
