"""Flat-buffer fused AdamW with on-device grad-norm clipping.

All trainable parameters are re-homed into one contiguous fp32 buffer (``FlatParams``), their
``.grad`` into a second; the optimizer state lives in two more flat buffers. One optimizer step is
two kernel launches (grad sum-of-squares partials, fused clip + AdamW) with no host sync; the
data-parallel all-reduce works on the same flat grad buffer in a few large buckets.
Semantics = torch.optim.AdamW (decoupled weight decay, bias correction) + clip_grad_norm_.
"""
from __future__ import annotations

from typing import Iterable, List

import torch

from . import reference as ref
from ._ext import native, on_gpu


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
            off += (p.numel() + align - 1) // align * align
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


class FusedAdamW:
    def __init__(self, flat: FlatParams, lr=5e-5, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01,
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
        if on_gpu(self.flat.data):
            native().adamw(self.flat.data, self.flat.grad, self.exp_avg, self.exp_avg_sq, None, lr, self.b1, self.b2,
                           self.eps, self.wd, self.step_count, self.max_grad_norm, self.partials, self.last_norm,
                           self.skipped)
        else:
            norm, skipped = ref.adamw_(self.flat.data, self.flat.grad, self.exp_avg, self.exp_avg_sq, lr, self.b1,
                                       self.b2, self.eps, self.wd, self.step_count, self.max_grad_norm)
            self.last_norm.fill_(float(norm))
            if skipped:
                self.skipped += 1
                self.step_count -= 1

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
