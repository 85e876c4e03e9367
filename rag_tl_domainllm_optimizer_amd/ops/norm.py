"""Fused residual-add + RMSNorm / LayerNorm with autograd.

``rms_norm(x, w, eps, residual)`` returns ``(y, h)`` where ``h = x + residual`` is the updated
residual stream (the vLLM-style fused_add_rms_norm pattern: the residual add of the previous
sub-layer costs no separate pass). Backward accepts gradients for both outputs.
"""
from __future__ import annotations

import torch

from . import reference as ref
from ._ext import native, on_gpu


class _NormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, w, b, eps, layernorm):
        xs = x.contiguous()
        rs = residual.contiguous() if residual is not None else None
        if on_gpu(x):
            y, h, rstd, mean = native().norm_fwd(layernorm, xs, rs, w, b, eps)
        else:
            y, h, rstd, mean = ref.norm(xs, w, b, eps, rs, layernorm)
        hh = h if residual is not None else xs
        ctx.layernorm = layernorm
        ctx.eps = eps
        ctx.has_res = residual is not None
        ctx.has_b = b is not None
        ctx.save_for_backward(hh, w, rstd, mean if mean is not None else torch.empty(0))
        if residual is not None:
            return y, h
        return y

    @staticmethod
    def backward(ctx, dy, dh=None):
        h, w, rstd, mean = ctx.saved_tensors
        dy = dy.contiguous()
        need_dw = ctx.needs_input_grad[2]
        need_db = ctx.has_b and ctx.needs_input_grad[3]
        dh_res = dh.contiguous() if (dh is not None and ctx.has_res) else None
        if on_gpu(dy):
            dx, dw, db = native().norm_bwd(ctx.layernorm, dy, h, w, rstd, mean if ctx.layernorm else None, dh_res,
                                           need_dw, need_db)
        else:
            with torch.enable_grad():
                hh = h.detach().float().requires_grad_(True)
                ww = w.detach().float().requires_grad_(need_dw)
                if ctx.layernorm:
                    y = torch.nn.functional.layer_norm(hh, (hh.shape[-1],), ww, None, ctx.eps)
                else:
                    y = hh * torch.rsqrt(hh.pow(2).mean(-1, keepdim=True) + ctx.eps) * ww
                grads = torch.autograd.grad(y, [hh] + ([ww] if need_dw else []), dy.float())
            dx = grads[0]
            if dh_res is not None:
                dx = dx + dh_res.float()
            dx = dx.to(dy.dtype)
            dw = grads[1] if need_dw else None
            db = dy.float().reshape(-1, dy.shape[-1]).sum(0) if need_db else None
        dw = dw.to(w.dtype) if (need_dw and dw is not None) else None
        if need_db and db is not None:
            db = db.to(w.dtype)
        else:
            db = None
        dres = dx if ctx.has_res else None
        return dx, dres, dw, db, None, None


def _norm(x, w, b, eps, residual, layernorm):
    from .linear import SplitK

    if isinstance(x, SplitK):  # the producing GEMM's split-K reduce fused into this pass
        if residual is None:
            x = x.reduce()
        else:
            return tuple(native().norm_fwd_slabs(layernorm, x.slabs, x.nsplit, x.M, x.N, residual.contiguous(), w, b,
                                                 eps))
    grad = torch.is_grad_enabled() and (x.requires_grad or w.requires_grad or (residual is not None and residual.requires_grad))
    if not grad:
        xs = x.contiguous()
        rs = residual.contiguous() if residual is not None else None
        if on_gpu(x):
            y, h, _, _ = native().norm_fwd(layernorm, xs, rs, w, b, eps)
        else:
            y, h, _, _ = ref.norm(xs, w, b, eps, rs, layernorm)
        return y, (h if residual is not None else xs)
    if residual is None:
        return _NormFn.apply(x, None, w, b, eps, layernorm), x
    return _NormFn.apply(x, residual, w, b, eps, layernorm)


def rms_norm(x, w, eps=1e-6, residual=None):
    """(y, h): h = x + residual (or x), y = RMSNorm(h) * w."""
    return _norm(x, w, None, eps, residual, False)


def layer_norm(x, w, b=None, eps=1e-5, residual=None):
    """(y, h): h = x + residual (or x), y = LayerNorm(h) * w + b."""
    return _norm(x, w, b, eps, residual, True)
