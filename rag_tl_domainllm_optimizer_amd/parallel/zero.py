"""ZeRO-1: sharded fp32 optimizer state for full-parameter training under data parallelism.

The reference trains every policy weight with AdamW (reinforcement_learning_optimization_after_rag.py
:153-156, 228-232). Replicated over N data-parallel ranks that is 16 B of training state per weight
on every rank (bf16 weight + bf16 gradient + fp32 master + two fp32 moments: ~116 GB for
Mistral-7B) and N copies of the same optimizer pass. Here each rank owns 1/N of every gradient
bucket:

* backward: as soon as a bucket's gradients are final (post-accumulate hooks, buckets launched
  strictly in order), its bf16 slice is widened into an fp32 staging buffer and reduce-scattered
  IN FP32 (RCCL over xGMI; no bf16 rounding of the sum, unlike ``GradSync``'s rs32 path, which
  rounds the shard before its all-gather). The rank keeps only its fp32 shard of the sum.
* step: the rank's shards are one compact fp32 vector; one kernel pass gives its sum of squares, a
  1024-float all-reduce gives the global norm (clip as torch ``clip_grad_norm_``), one fused AdamW
  launch updates the fp32 master / moments of the shard and writes its bf16 weights, and a bf16
  all-gather per bucket rebuilds the full compute copy on every rank.

Link bytes per weight and step: 4 (fp32 reduce-scatter) + 2 (bf16 all-gather), the same as
``GradSync``'s rs32 + replicated AdamW, but the bf16 gradient is never re-gathered and the
optimizer runs on 1/N of the weights.

Memory per rank (bytes per weight): bf16 weights 2 + bf16 gradients 2 + (fp32 master 4 + moments
8) / N = 5.5 at N = 8 (39.8 GB for Mistral-7B's 7.24 B weights; replicated: 16 B, 116 GB). The
compact fp32 gradient shard (4/N B) and, from N = 3, the bf16 update shard (2/N B) live INSIDE the
bf16 gradient buffer, in bytes whose gradients have already been consumed: bucket b (counted from
the end of the layout, the order backward finishes them) writes its shard to bytes
[2 n16 - 4 (n16 - s_b) / N, ...) >= 2 s_b, i.e. only over buckets 0..b, whose bf16 inputs were
widened into staging before their collectives started. Launching buckets strictly in index order
keeps that invariant when backward finishes parameters out of order.

The fp32 tail of the layout (the value head, 4097 weights) stays replicated: all-reduced and
updated by every rank with the same clip coefficient.

Parameters must come from ``ops.flat_params(..., align=16 * world, keep_master=False)`` so that
every bucket splits into N equal, 16-element-aligned shards.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist

from .dist import info

_NPART = 1024  # grad-norm partials (the fused AdamW kernel reduces up to 1024)


class _Bucket:
    __slots__ = ("s", "e", "sh", "j0", "params")

    def __init__(self, s, e, sh, j0):
        self.s, self.e, self.sh, self.j0 = s, e, sh, j0
        self.params = 0


class ZeroAdamW:
    """FusedAdamW-compatible optimizer (``step``, ``zero_grad``, ``last_norm``, ``skipped``,
    ``step_count``) whose ``sync`` attribute is the GradSync-compatible gradient reducer
    (``start`` / ``finish`` / ``no_sync`` / ``wait_s`` / ``comm_bytes``)."""

    sharded = True

    def __init__(self, flat, lr=5e-5, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01, max_grad_norm=0.0,
                 bucket_bytes: int = 256 << 20, inflight: int = 2):
        from ..ops.optim import MixedFlatParams

        di = info()
        self.world, self.rank = di.world, di.rank
        w = self.world
        if not isinstance(flat, MixedFlatParams) or flat.master_base != flat.n16:
            raise TypeError("ZeroAdamW: needs ops.flat_params(..., keep_master=False) (bf16 members)")
        if flat.align % (16 * w):
            raise ValueError(f"ZeroAdamW: members must be aligned to 16 x world = {16 * w} elements "
                             f"(got {flat.align})")
        self.flat = flat
        self.lr, (self.b1, self.b2), self.eps, self.wd = lr, betas, eps, weight_decay
        self.max_grad_norm = max_grad_norm
        self.step_count = 0
        self.inflight = max(1, inflight)
        n16 = flat.n16
        dev = flat.data16.device
        self.device = dev
        self.cuda = dev.type == "cuda"
        # buckets over the bf16 members, from the END of the layout (backward order), aligned to
        # member boundaries; bucket b holds layout [s, e), rank r owns [s + r sh, s + (r + 1) sh)
        per = max(16 * w, bucket_bytes // 4)
        offs = [o for o, p in zip(flat.offsets, flat.params) if p.dtype == torch.bfloat16] + [n16]
        nb16 = flat.n_params16
        bounds, cur_end = [], None
        self.param_bucket = {}
        for idx in reversed(range(nb16)):
            s_, e_ = offs[idx], offs[idx + 1]
            if cur_end is None:
                cur_end = e_
            self.param_bucket[idx] = len(bounds)
            if cur_end - s_ >= per:
                bounds.append((s_, cur_end))
                cur_end = None
        if cur_end is not None:
            bounds.append((offs[0], cur_end))
        self.ns = n16 // w  # compact shard length
        self.buckets: List[_Bucket] = []
        c = 0
        for s_, e_ in bounds:
            sh = (e_ - s_) // w
            assert sh * w == e_ - s_ and sh % 16 == 0, (s_, e_, w)
            c += sh
            self.buckets.append(_Bucket(s_, e_, sh, self.ns - c))  # compact index: ascending layout order
        for idx, bi in self.param_bucket.items():
            self.buckets[bi].params += 1
        # compact fp32 gradient shard (and bf16 update shard) inside the bf16 gradient bytes
        gb = flat.grad16.view(torch.uint8)
        self.gshard = gb[2 * n16 - 4 * self.ns:2 * n16].view(torch.float32)
        if 6 * self.ns <= 2 * n16:
            self.pshard16 = gb[2 * n16 - 6 * self.ns:2 * n16 - 4 * self.ns].view(torch.bfloat16)
        else:  # N = 2: no room left below the gradient shard
            self.pshard16 = torch.empty(self.ns, dtype=torch.bfloat16, device=dev)
        # fp32 master / moments of this rank's shards (the starting bf16 weights, exactly)
        self.master = torch.empty(self.ns, dtype=torch.float32, device=dev)
        for b in self.buckets:
            o = b.s + self.rank * b.sh
            self.master[b.j0:b.j0 + b.sh].copy_(flat.data16[o:o + b.sh])
        self.exp_avg = torch.zeros_like(self.master)
        self.exp_avg_sq = torch.zeros_like(self.master)
        # replicated fp32 tail (value head): master = flat.data
        self.m32 = torch.zeros_like(flat.data)
        self.v32 = torch.zeros_like(flat.data)
        self.partials = torch.zeros(_NPART if self.cuda else 2, dtype=torch.float32, device=dev)
        self.last_norm = torch.zeros((), dtype=torch.float32, device=dev)
        self._norm_tail = torch.zeros((), dtype=torch.float32, device=dev)
        self.skipped = torch.zeros((), dtype=torch.int32, device=dev)
        self._skipped_tail = torch.zeros((), dtype=torch.int32, device=dev)
        self.sync = _ZeroSync(self)

    # ---------------------------------------------------------------- memory accounting
    def state_bytes(self) -> dict:
        """Per-rank bytes of training state (tests / bench JSON)."""
        f = self.flat
        d = {"weights_bf16": f.data16.numel() * 2, "grads_bf16": f.grad16.numel() * 2,
             "master_fp32": self.master.numel() * 4, "moments_fp32": 2 * self.exp_avg.numel() * 4,
             "tail_fp32": f.data.numel() * 4 * 4,
             "update_shard_bf16": 0 if self._scratch_pshard() else self.pshard16.numel() * 2}
        d["total"] = sum(d.values())
        return d

    def _scratch_pshard(self) -> bool:
        return self.pshard16.untyped_storage().data_ptr() == self.flat.grad16.untyped_storage().data_ptr()

    # ---------------------------------------------------------------- optimizer interface
    def zero_grad(self):
        self.flat.zero_grad()

    def step(self, lr=None):
        lr = self.lr if lr is None else lr
        self.flat.relink_grads()
        self.step_count += 1
        w = self.world
        gs = self.gshard
        gs.div_(w)  # sum -> mean over ranks
        tail_g = self.flat.grad32
        # the bf16 update shard lives in gradient scratch on N >= 3: seed it with the current
        # weights so a skipped (non-finite) step all-gathers them unchanged
        self.pshard16.copy_(self.master)
        if self.cuda:
            from ..ops import native

            C = native()
            half = _NPART // 2
            C.grad_sumsq(gs, self.partials[:half])
            self.partials[half:].zero_()
            dist.all_reduce(self.partials)
            if tail_g.numel():  # replicated: added after the cross-rank sum
                C.grad_sumsq(tail_g, self.partials[half:])
            C.adamw_apply(self.master, gs, self.exp_avg, self.exp_avg_sq, self.pshard16, lr, self.b1, self.b2,
                          self.eps, self.wd, self.step_count, self.max_grad_norm, self.partials, self.last_norm,
                          self.skipped)
            if tail_g.numel():
                C.adamw_apply(self.flat.data, tail_g, self.m32, self.v32, None, lr, self.b1, self.b2, self.eps,
                              self.wd, self.step_count, self.max_grad_norm, self.partials, self._norm_tail,
                              self._skipped_tail)
        else:
            ss = torch.stack([gs.double().pow(2).sum(), torch.zeros((), dtype=torch.float64)])
            dist.all_reduce(ss)
            tot = float(ss[0]) + float(tail_g.double().pow(2).sum())
            norm = tot ** 0.5
            self.last_norm.fill_(norm)
            if not torch.isfinite(torch.tensor(norm)):
                self.skipped += 1
            else:
                clip = min(1.0, self.max_grad_norm / (norm + 1e-6)) if self.max_grad_norm > 0 else 1.0
                t = self.step_count - int(self.skipped)
                _adamw_eager(self.master, gs, self.exp_avg, self.exp_avg_sq, lr, self.b1, self.b2, self.eps,
                             self.wd, t, clip)
                if tail_g.numel():
                    _adamw_eager(self.flat.data, tail_g, self.m32, self.v32, lr, self.b1, self.b2, self.eps,
                                 self.wd, t, clip)
                self.pshard16.copy_(self.master)
        # every rank's updated bf16 shards -> the full compute copy
        hs = [dist.all_gather_into_tensor(self.flat.data16[b.s:b.e], self.pshard16[b.j0:b.j0 + b.sh],
                                          async_op=True) for b in self.buckets]
        self.sync.comm_bytes += self.flat.n16 * 2
        for h in hs:
            h.wait()
        self.flat.bump_versions()

    # ---------------------------------------------------------------- checkpoints
    def state_dict(self):
        """Metadata only: the tensors of a sharded state are written per rank (``save_shard``)."""
        return {"step": self.step_count, "lr": self.lr, "betas": (self.b1, self.b2), "eps": self.eps,
                "weight_decay": self.wd, "max_grad_norm": self.max_grad_norm, "skipped": self.skipped,
                "zero_world": self.world}

    def load_state_dict(self, sd):
        if int(sd.get("zero_world", self.world)) != self.world:
            raise ValueError(f"ZeRO checkpoint written at world {sd.get('zero_world')}, loading at {self.world}")
        self.step_count = int(sd["step"])
        self.lr = sd.get("lr", self.lr)
        if "skipped" in sd:
            self.skipped.copy_(torch.as_tensor(sd["skipped"]))
            self._skipped_tail.copy_(torch.as_tensor(sd["skipped"]))

    def shard_file(self, d: str) -> str:
        return os.path.join(d, f"optimizer_zero{self.world}_rank{self.rank}.safetensors")

    def save_shard(self, d: str):
        from safetensors.torch import save_file

        f = self.shard_file(d)
        save_file({"master": self.master.cpu(), "exp_avg": self.exp_avg.cpu(), "exp_avg_sq": self.exp_avg_sq.cpu(),
                   "tail": self.flat.data.cpu().contiguous(), "m32": self.m32.cpu(), "v32": self.v32.cpu()},
                  f + ".tmp")
        os.replace(f + ".tmp", f)

    def load_shard(self, d: str):
        """Every rank: its own shard, then the bf16 compute copy rebuilt from the masters."""
        from safetensors.torch import load_file

        t = load_file(self.shard_file(d))
        with torch.no_grad():
            self.master.copy_(t["master"])
            self.exp_avg.copy_(t["exp_avg"])
            self.exp_avg_sq.copy_(t["exp_avg_sq"])
            self.flat.data.copy_(t["tail"])
            self.m32.copy_(t["m32"])
            self.v32.copy_(t["v32"])
            self.pshard16.copy_(self.master)
        hs = [dist.all_gather_into_tensor(self.flat.data16[b.s:b.e], self.pshard16[b.j0:b.j0 + b.sh],
                                          async_op=True) for b in self.buckets]
        for h in hs:
            h.wait()
        self.flat.bump_versions()


def _adamw_eager(p, g, m, v, lr, b1, b2, eps, wd, step, clip):
    """torch.optim.AdamW on a given clip coefficient (CPU path; the GPU path is the fused kernel)."""
    gr = g * clip
    m.mul_(b1).add_(gr, alpha=1 - b1)
    v.mul_(b2).addcmul_(gr, gr, value=1 - b2)
    p.mul_(1 - lr * wd)
    denom = (v / (1 - b2 ** step)).sqrt().add_(eps)
    p.addcdiv_(m, denom, value=-lr / (1 - b1 ** step))


class _ZeroSync:
    """Gradient side of ZeroAdamW: in-order bucketed fp32 reduce-scatter overlapped with backward."""

    def __init__(self, opt: ZeroAdamW):
        self.opt = opt
        self.flat = opt.flat
        self.world = opt.world
        self.buckets = opt.buckets
        self.sync_enabled = True
        self.wait_s = 0.0
        self.comm_bytes = 0
        self._ready = [0] * len(self.buckets)
        self._next = 0        # next bucket to launch (strict order: see the module doc)
        self._inflight = []   # (handle, staging buffer)
        self._hooks = []
        if info().enabled:
            for idx, bi in opt.param_bucket.items():
                p = self.flat.params[idx]
                self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(bi)))

    def _make_hook(self, bi):
        def hook(_p):
            if not self.sync_enabled:
                return
            self._ready[bi] += 1
            self._launch_ready()
        return hook

    def _launch_ready(self):
        while self._next < len(self.buckets) and self._ready[self._next] >= self.buckets[self._next].params:
            self._launch(self._next)
            self._next += 1

    def _launch(self, bi):
        b = self.buckets[bi]
        while len(self._inflight) >= self.opt.inflight:
            h, _buf = self._inflight.pop(0)
            h.wait()
        buf = torch.empty(b.e - b.s, dtype=torch.float32, device=self.flat.grad16.device)
        buf.copy_(self.flat.grad16[b.s:b.e])
        out = self.opt.gshard[b.j0:b.j0 + b.sh]
        self.comm_bytes += buf.numel() * 4
        self._inflight.append((dist.reduce_scatter_tensor(out, buf, async_op=True), buf))

    def no_sync(self):
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
        self._next = 0

    def finish(self):
        if not info().enabled:
            return
        import time

        t0 = time.perf_counter()
        self.flat.relink_grads()
        for bi in range(self._next, len(self.buckets)):
            self._launch(bi)
        self._next = len(self.buckets)
        g32 = self.flat.grad32
        h32 = None
        if g32.numel():
            self.comm_bytes += g32.numel() * 4
            h32 = dist.all_reduce(g32, async_op=True)
        while self._inflight:
            h, _buf = self._inflight.pop(0)
            h.wait()
        if h32 is not None:
            h32.wait()
            g32.div_(self.world)
        self.wait_s += time.perf_counter() - t0
        self._ready = [0] * len(self.buckets)

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []


def zero_enabled(full_finetune: bool, requested: Optional[bool] = None) -> bool:
    """ZeRO-1 applies to full-parameter training at world > 1 (default on; ``requested=False`` keeps
    the replicated optimizer)."""
    if not full_finetune or info().world <= 1:
        return False
    return True if requested is None else bool(requested)


def per_rank_state_bytes(n16: int, n32: int, world: int) -> int:
    """Training-state bytes per rank for n16 bf16 weights and n32 fp32 weights: replicated mixed
    AdamW at world 1 (2 + 2 + 4 + 8 B per bf16 weight), ZeRO-1 above (bf16 weights and gradients
    whole, fp32 master and moments 1/N; the fp32 gradient shard lives in the gradient buffer, and
    so does the bf16 update shard from N = 3 on). The fp32 tail is replicated: 16 B per weight."""
    if world <= 1:
        return 16 * n16 + 16 * n32
    upd = 0 if world >= 3 else 2 * n16 // world
    return 4 * n16 + 12 * n16 // world + upd + 16 * n32
