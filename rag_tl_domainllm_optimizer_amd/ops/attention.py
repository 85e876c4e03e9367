"""RoPE (+ KV-cache append), flash attention (fwd/bwd) and KV-cache decode attention."""
from __future__ import annotations

import math
from typing import Optional

import torch

from . import reference as ref
from ._ext import native, on_gpu


# ------------------------------------------------------------------------------------------ RoPE
def rope_qkv_(qkv: torch.Tensor, pos: torch.Tensor, cos, sin, Hq: int, Hkv: int, D: int, *, S: int = 1,
              k_cache=None, v_cache=None, slot_base=None, rope_q: bool = True, sign: float = 1.0):
    """In-place rotary embedding of the q/k heads of fused qkv rows; optionally appends the
    (rotated) k and v rows to a KV cache [B, Hkv, Smax, D] at slot ``slot_base[b] + s`` for token
    ``t = b*S + s``. ``cos``/``sin`` may be None (no rotation: learned-position models)."""
    if on_gpu(qkv):
        native().rope_qkv(qkv, pos, cos, sin, S, Hq, Hkv, D, sign, k_cache, v_cache, slot_base, rope_q)
        return qkv
    if cos is not None:
        qkv.copy_(ref.rope_qkv(qkv, pos, cos, sin, Hq, Hkv, D, sign, rope_q))
    if k_cache is not None:
        T = qkv.shape[0]
        B = T // S
        base = slot_base.long() if slot_base is not None else torch.zeros(B, dtype=torch.long)
        k = qkv[:, Hq * D:(Hq + Hkv) * D].reshape(B, S, Hkv, D).transpose(1, 2)
        v = qkv[:, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D].reshape(B, S, Hkv, D).transpose(1, 2)
        for b in range(B):
            s0 = int(base[b])
            k_cache[b, :, s0:s0 + S] = k[b]
            v_cache[b, :, s0:s0 + S] = v[b]
    return qkv


class _RopeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, pos, cos, sin, Hq, Hkv, D, rope_q):
        rope_qkv_(qkv, pos, cos, sin, Hq, Hkv, D, rope_q=rope_q)
        ctx.mark_dirty(qkv)
        ctx.save_for_backward(pos, cos, sin)
        ctx.cfg = (Hq, Hkv, D, rope_q)
        return qkv

    @staticmethod
    def backward(ctx, g):
        pos, cos, sin = ctx.saved_tensors
        Hq, Hkv, D, rope_q = ctx.cfg
        g = g.contiguous().clone()
        rope_qkv_(g, pos, cos, sin, Hq, Hkv, D, rope_q=rope_q, sign=-1.0)
        return g, None, None, None, None, None, None, None


def rope_qkv(qkv, pos, cos, sin, Hq, Hkv, D, rope_q=True):
    """Autograd-aware RoPE on fused qkv rows (in place when no grad is needed)."""
    if torch.is_grad_enabled() and qkv.requires_grad:
        if not on_gpu(qkv):
            return ref.rope_qkv(qkv, pos, cos, sin, Hq, Hkv, D, 1.0, rope_q)
        return _RopeFn.apply(qkv, pos, cos, sin, Hq, Hkv, D, rope_q)
    return rope_qkv_(qkv, pos, cos, sin, Hq, Hkv, D, rope_q=rope_q)


# ----------------------------------------------------------------------------- flash attention
class _FlashFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, B, S, Hq, Hkv, D, causal, window, scale, kv_start):
        q = qkv[:, : Hq * D]
        k = qkv[:, Hq * D:(Hq + Hkv) * D]
        v = qkv[:, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D]
        o, lse = native().attn_fwd(q, k, v, B, S, S, Hq, Hkv, D, causal, window, scale, kv_start, None, None, 0, True)
        ctx.save_for_backward(qkv, o, lse, kv_start if kv_start is not None else torch.empty(0))
        ctx.cfg = (B, S, Hq, Hkv, D, causal, window, scale, kv_start is not None)
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse, kv_start = ctx.saved_tensors
        B, S, Hq, Hkv, D, causal, window, scale, has_start = ctx.cfg
        do = do.contiguous()
        dqkv = torch.zeros_like(qkv)
        q = qkv[:, : Hq * D]
        k = qkv[:, Hq * D:(Hq + Hkv) * D]
        v = qkv[:, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D]
        native().attn_bwd(q, k, v, o, do, lse, dqkv[:, : Hq * D], dqkv[:, Hq * D:(Hq + Hkv) * D],
                          dqkv[:, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D], B, S, Hq, Hkv, D, causal, window, scale,
                          kv_start if has_start else None)
        return dqkv, None, None, None, None, None, None, None, None, None


def flash_attention_qkv(qkv, B, S, Hq, Hkv, D, causal=True, window=0, scale=None, kv_start=None):
    """Self-attention over fused qkv rows [B*S, (Hq+2Hkv)*D] -> o [B*S, Hq*D]."""
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if not on_gpu(qkv):
        q = qkv[:, : Hq * D]
        k = qkv[:, Hq * D:(Hq + Hkv) * D]
        v = qkv[:, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D]
        return ref.attention(q, k, v, B, S, S, Hq, Hkv, D, causal, window, scale, kv_start)[0]
    if torch.is_grad_enabled() and qkv.requires_grad:
        return _FlashFn.apply(qkv, B, S, Hq, Hkv, D, causal, window, scale, kv_start)
    q = qkv[:, : Hq * D]
    k = qkv[:, Hq * D:(Hq + Hkv) * D]
    v = qkv[:, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D]
    return native().attn_fwd(q, k, v, B, S, S, Hq, Hkv, D, causal, window, scale, kv_start, None, None, 0, False)[0]


def attention(q, k, v, B, Sq, Sk, Hq, Hkv, D, causal=False, window=0, scale=None, kv_start=None, kv_len=None,
              rel_bias_lut: Optional[torch.Tensor] = None, rb_L: int = 0):
    """Inference attention on separate (strided) q/k/v row views; used by the encoders
    (bidirectional, key-length mask, MPNet relative-position bias LUT in log2 units)."""
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if on_gpu(q):
        return native().attn_fwd(q, k, v, B, Sq, Sk, Hq, Hkv, D, causal, window, scale, kv_start, kv_len,
                                 rel_bias_lut, rb_L, False)[0]
    return ref.attention(q, k, v, B, Sq, Sk, Hq, Hkv, D, causal, window, scale, kv_start, kv_len, rel_bias_lut,
                         rb_L)[0]


# ------------------------------------------------------------------------------ decode attention
def decode_partition(batch_heads: int) -> int:
    """Keys per split-K partition: small partitions when few (batch, kv-head) pairs exist."""
    return 64 if batch_heads < 128 else 256


def decode_workspace(B, Hq, Hkv, D, Smax, device, PS=None):
    PS = PS or decode_partition(B * Hkv)
    NP = (Smax + PS - 1) // PS
    return torch.empty(B * Hkv * NP * (Hq // Hkv) * (D + 2), dtype=torch.float32, device=device), PS


def decode_attention(q, k_cache, v_cache, kv_len, Hq, kv_start=None, window=0, scale=None, workspace=None, out=None):
    """One query token per sequence against a KV cache [B, Hkv, Smax, D] -> [B, Hq*D]."""
    B, Hkv, Smax, D = k_cache.shape
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if not on_gpu(q):
        o = ref.decode_attention(q, k_cache, v_cache, kv_len, Hq, kv_start, window, scale)
        if out is not None:
            out.copy_(o)
            return out
        return o
    if workspace is None:
        workspace = decode_workspace(B, Hq, Hkv, D, Smax, q.device)
    part, PS = workspace
    if out is None:
        out = torch.empty(B, Hq * D, dtype=q.dtype, device=q.device)
    native().attn_decode(q, k_cache, v_cache, kv_len, kv_start, window, scale, Hq, part, PS, out)
    return out
