"""Flat-buffer fused AdamW with on-device grad-norm clipping.

All trainable parameters are re-homed into one contiguous fp32 buffer (``FlatParams``), their
``.grad`` into a second; the optimizer state lives in two more flat buffers. One optimizer step is
two kernel launches (grad sum-of-squares partials, fused clip + AdamW) with no host sync; the
data-parallel all-reduce works on the same flat grad buffer in a few large buckets.
Full-parameter training of a bf16 model uses ``MixedFlatParams`` instead: bf16 compute copies and
bf16 gradients beside an fp32 master; one fused pass reads the bf16 gradients and rewrites both.
Semantics = torch.optim.AdamW (decoupled weight decay, bias correction) + clip_grad_norm_.
"""
from __future__ import annotations

from typing import Iterable, List

import torch

from . import reference as ref
from ._ext import native, on_gpu


def _round(n: int, align: int) -> int:
    return (n + align - 1) // align * align


class FlatParams:
    """Packs parameters into one fp32 buffer; parameters become views into it."""

    def __init__(self, params: Iterable[torch.nn.Parameter], align: int = 16):
        self.params: List[torch.nn.Parameter] = [p for p in params]
        if not self.params:
            raise ValueError("FlatParams: no parameters")
        dev = self.params[0].device
        self.offsets = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            off += _round(p.numel(), align)
        self.numel = off
        self.data = torch.zeros(off, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(off, dtype=torch.float32, device=dev)
        for p, o in zip(self.params, self.offsets):
            n = p.numel()
            self.data[o:o + n].copy_(p.detach().reshape(-1).float())
            p.data = self.data[o:o + n].view(p.shape)
            p.grad = self.grad[o:o + n].view(p.shape)

    def zero_grad(self):
        self.grad.zero_()
        for p, o in zip(self.params, self.offsets):
            n = p.numel()
            if p.grad is None or p.grad.data_ptr() != self.grad[o:o + n].data_ptr():
                p.grad = self.grad[o:o + n].view(p.shape)

    def relink_grads(self):
        """Autograd may replace .grad (e.g. when it was None); fold any foreign grads back in."""
        for p, o in zip(self.params, self.offsets):
            n = p.numel()
            view = self.grad[o:o + n]
            if p.grad is None:
                p.grad = view.view(p.shape)
            elif p.grad.data_ptr() != view.data_ptr():
                view.copy_(p.grad.reshape(-1).float())
                p.grad = view.view(p.shape)

    # gradient-buffer interface shared with MixedFlatParams (parallel.GradSync)
    def grad_slices(self, s: int, e: int) -> List[torch.Tensor]:
        return [self.grad[s:e]]

    def div_grads(self, d: float):
        self.grad.div_(d)


class MixedFlatParams:
    """Full-parameter training of a bf16 model — the reference's mode: AdamW over every policy
    weight and the value head (reinforcement_learning_optimization_after_rag.py:153-156,228-232).

    * bf16 parameters stay the compute copy the MFMA kernels read. They become views into ONE flat
      bf16 buffer (``data16``), so the kernels and captured hipGraphs keep their addresses, and the
      optimizer rewrites them in its own pass.
    * Their gradients are views into one flat bf16 buffer (``grad16``): the DP all-reduce moves
      2 B per weight over xGMI.
    * The optimizer owns the fp32 master copy (``data``) and the fp32 moments.
    * fp32 parameters (the value head) are views into the master's tail, with fp32 gradients
      (``grad32``).

    Layout in elements: [0, n16) bf16 members | [n16, numel) fp32 members. Per bf16 weight
    2 + 2 + 4 + 8 = 16 B of training state: Mistral-7B full fine-tuning holds 116 GB, which fits
    one 288 GB MI355X beside a frozen reference copy, the KV cache and the activations.
    """

    def __init__(self, params: Iterable[torch.nn.Parameter], align: int = 16, keep_master: bool = True):
        """``keep_master=False`` (ZeRO-1, :class:`parallel.zero.ZeroAdamW`): no fp32 master of the
        bf16 members here — each rank's optimizer keeps the master of its own shard — and ``data``
        holds only the fp32 tail (``master_base = n16``). ``align``: element alignment of every
        member; ZeRO passes 16 x world so every bucket splits into equal 16-element shards."""
        params = list(params)
        if not params:
            raise ValueError("MixedFlatParams: no parameters")
        p16 = [p for p in params if p.dtype == torch.bfloat16]
        p32 = [p for p in params if p.dtype == torch.float32]
        if len(p16) + len(p32) != len(params):
            raise TypeError("MixedFlatParams: parameters must be bfloat16 or float32")
        self.params: List[torch.nn.Parameter] = p16 + p32
        self.n_params16 = len(p16)
        dev = self.params[0].device
        self.offsets, off = [], 0
        for p in p16:
            self.offsets.append(off)
            off += _round(p.numel(), align)
        self.n16 = off
        for p in p32:
            self.offsets.append(off)
            off += _round(p.numel(), align)
        self.numel = off
        self.align = align
        self.master_base = 0 if keep_master else self.n16
        self.data = torch.zeros(off - self.master_base, dtype=torch.float32, device=dev)
        self.data16 = torch.zeros(self.n16, dtype=torch.bfloat16, device=dev)
        self.grad16 = torch.zeros(self.n16, dtype=torch.bfloat16, device=dev)
        self.grad32 = torch.zeros(off - self.n16, dtype=torch.float32, device=dev)
        with torch.no_grad():
            for p, o in zip(self.params, self.offsets):
                n = p.numel()
                if o >= self.master_base:
                    self.data[o - self.master_base:o - self.master_base + n].copy_(p.detach().reshape(-1))
                if p.dtype == torch.bfloat16:
                    self.data16[o:o + n].copy_(p.detach().reshape(-1))
                p.data = self._param_view(p, o)
                p.grad = self._grad_view(p, o)

    def _param_view(self, p, o):
        if p.dtype == torch.bfloat16:
            return self.data16[o:o + p.numel()].view(p.shape)
        o -= self.master_base
        return self.data[o:o + p.numel()].view(p.shape)

    def _grad_view(self, p, o):
        n = p.numel()
        if p.dtype == torch.bfloat16:
            return self.grad16[o:o + n].view(p.shape)
        return self.grad32[o - self.n16:o - self.n16 + n].view(p.shape)

    # gradient-buffer interface shared with FlatParams (parallel.GradSync)
    def grad_slices(self, s: int, e: int) -> List[torch.Tensor]:
        out = []
        if s < self.n16:
            out.append(self.grad16[s:min(e, self.n16)])
        if e > self.n16:
            out.append(self.grad32[max(s, self.n16) - self.n16:e - self.n16])
        return out

    def div_grads(self, d: float):
        self.grad16.div_(d)
        self.grad32.div_(d)

    def full_grad(self) -> torch.Tensor:
        """fp32 gradient over the whole layout (CPU optimizer path, tests)."""
        return torch.cat([self.grad16.float(), self.grad32])

    def zero_grad(self):
        self.grad16.zero_()
        self.grad32.zero_()
        for p, o in zip(self.params, self.offsets):
            view = self._grad_view(p, o)
            if p.grad is None or p.grad.data_ptr() != view.data_ptr():
                p.grad = view

    def relink_grads(self):
        for p, o in zip(self.params, self.offsets):
            view = self._grad_view(p, o)
            if p.grad is None:
                p.grad = view
            elif p.grad.data_ptr() != view.data_ptr():
                view.copy_(p.grad.reshape(view.shape))
                p.grad = view

    def refresh_shadow(self):
        """bf16 compute copies <- fp32 master (after a checkpoint load or a CPU optimizer step)."""
        if self.master_base:
            raise RuntimeError("MixedFlatParams(keep_master=False): the master lives in the ZeRO shards")
        with torch.no_grad():
            self.data16.copy_(self.data[:self.n16])
        self.bump_versions()

    def bump_versions(self):
        """The optimizer rewrote the bf16 compute copies behind autograd's back: advance their
        version counters so version-keyed derived images (norm-folded decode weights, fp8
        images) are rebuilt before the next use."""
        if self.n_params16:
            torch.autograd.graph.increment_version(self.params[:self.n_params16])


def flat_params(params: Iterable[torch.nn.Parameter], align: int = 16, keep_master: bool = True):
    """FlatParams for fp32 trainables (LoRA adapters, value head, fp32 CPU models);
    MixedFlatParams as soon as a bf16 weight trains (full-parameter fine-tuning on the GPU)."""
    params = list(params)
    if any(p.dtype == torch.bfloat16 for p in params):
        return MixedFlatParams(params, align, keep_master)
    return FlatParams(params, align)


class FusedAdamW:
    def __init__(self, flat, lr=5e-5, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01,
                 max_grad_norm: float = 0.0):
        self.flat = flat
        self.lr = lr
        self.b1, self.b2 = betas
        self.eps = eps
        self.wd = weight_decay
        self.max_grad_norm = max_grad_norm
        self.step_count = 0
        dev = flat.data.device
        self.exp_avg = torch.zeros_like(flat.data)
        self.exp_avg_sq = torch.zeros_like(flat.data)
        self.partials = torch.zeros(1024 if dev.type == "cuda" else 1, dtype=torch.float32, device=dev)
        self.last_norm = torch.zeros((), dtype=torch.float32, device=dev)
        self.skipped = torch.zeros((), dtype=torch.int32, device=dev)

    def step(self, lr=None):
        lr = self.lr if lr is None else lr
        self.flat.relink_grads()
        self.step_count += 1
        mixed = isinstance(self.flat, MixedFlatParams)
        if on_gpu(self.flat.data):
            if mixed:
                native().adamw_mixed(self.flat.data, self.flat.grad16, self.flat.grad32, self.exp_avg,
                                     self.exp_avg_sq, self.flat.data16, lr, self.b1, self.b2, self.eps, self.wd,
                                     self.step_count, self.max_grad_norm, self.partials, self.last_norm,
                                     self.skipped)
            else:
                native().adamw(self.flat.data, self.flat.grad, self.exp_avg, self.exp_avg_sq, None, lr, self.b1,
                               self.b2, self.eps, self.wd, self.step_count, self.max_grad_norm, self.partials,
                               self.last_norm, self.skipped)
        else:
            g = self.flat.full_grad() if mixed else self.flat.grad
            # bias correction over APPLIED steps (calls - skipped), as the GPU kernel derives it
            norm, skipped = ref.adamw_(self.flat.data, g, self.exp_avg, self.exp_avg_sq, lr, self.b1,
                                       self.b2, self.eps, self.wd, self.step_count - int(self.skipped),
                                       self.max_grad_norm)
            self.last_norm.fill_(float(norm))
            if skipped:
                self.skipped += 1
            elif mixed:
                with torch.no_grad():
                    self.flat.data16.copy_(self.flat.data[:self.flat.n16])
        if mixed:
            self.flat.bump_versions()

    def zero_grad(self):
        self.flat.zero_grad()

    def state_dict(self):
        return {"step": self.step_count, "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq, "lr": self.lr,
                "betas": (self.b1, self.b2), "eps": self.eps, "weight_decay": self.wd,
                "max_grad_norm": self.max_grad_norm, "skipped": self.skipped}

    def load_state_dict(self, sd):
        self.step_count = int(sd["step"])
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        self.lr = sd.get("lr", self.lr)
        if "skipped" in sd:
            self.skipped.copy_(sd["skipped"])
