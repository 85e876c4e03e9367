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
# the RoPE backward inside the attention backward's dQ / dK stores (A/B switch for the tests: off =
# the separate inverse-rotation pass over d_qkv; bitwise the same result)
ROPE_BWD_FUSED = True


class _FlashFn(torch.autograd.Function):
    """Flash attention over fused qkv rows, optionally with RoPE applied in place first.

    With ``rope`` = (pos, cos, sin) the rotation runs inside this Function: forward rotates q/k in
    the (otherwise unused) projection output and attends; backward inverse-rotates dq/dk in the
    gradient buffer the attention kernel just wrote. Versus a separate in-place RoPE autograd node
    this saves the CopySlices copy and the gradient clone of the whole qkv tensor per layer."""

    @staticmethod
    def forward(ctx, qkv, B, S, Hq, Hkv, D, causal, window, scale, kv_start, rope=None, rope_done=False):
        if rope is not None and not rope_done:
            # in place on the projection output: nothing else holds it (the linear saved its input)
            rope_qkv_(qkv, rope[0], rope[1], rope[2], Hq, Hkv, D)
        ctx.rope = rope
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
        # the backward kernels write every row of dq / dk / dv (masked rows as zeros): no zero fill
        # unless the rows carry columns beyond q | k | v
        dqkv = torch.empty_like(qkv) if qkv.shape[1] == (Hq + 2 * Hkv) * D else torch.zeros_like(qkv)
        q = qkv[:, : Hq * D]
        k = qkv[:, Hq * D:(Hq + Hkv) * D]
        v = qkv[:, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D]
        rope = ctx.rope
        fused = rope is not None and ROPE_BWD_FUSED and rope[0].dtype == torch.int32
        native().attn_bwd(q, k, v, o, do, lse, dqkv[:, : Hq * D], dqkv[:, Hq * D:(Hq + Hkv) * D],
                          dqkv[:, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D], B, S, Hq, Hkv, D, causal, window, scale,
                          kv_start if has_start else None, *(rope if fused else (None, None, None)))
        if rope is not None and not fused:
            pos, cos, sin = rope
            rope_qkv_(dqkv, pos, cos, sin, Hq, Hkv, D, sign=-1.0)
        return dqkv, None, None, None, None, None, None, None, None, None, None, None


def flash_attention_qkv(qkv, B, S, Hq, Hkv, D, causal=True, window=0, scale=None, kv_start=None, rope=None,
                        rope_done=False):
    """Self-attention over fused qkv rows [B*S, (Hq+2Hkv)*D] -> o [B*S, Hq*D]. ``rope`` =
    (pos, cos, sin) rotates q/k first (in place on ``qkv``, which must not be needed elsewhere).
    ``rope_done``: the projection already rotated q / k in its GEMM epilogue (ops.linear_rope);
    the rotation's gradient (inverse rotation of dq / dk) still runs here."""
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    grad_gpu = on_gpu(qkv) and torch.is_grad_enabled() and qkv.requires_grad
    if rope_done and not grad_gpu:
        rope = None
    if rope is not None and not grad_gpu:
        qkv = rope_qkv(qkv, rope[0], rope[1], rope[2], Hq, Hkv, D)
        rope = None
    if not on_gpu(qkv):
        q = qkv[:, : Hq * D]
        k = qkv[:, Hq * D:(Hq + Hkv) * D]
        v = qkv[:, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D]
        return ref.attention(q, k, v, B, S, S, Hq, Hkv, D, causal, window, scale, kv_start)[0]
    if torch.is_grad_enabled() and qkv.requires_grad:
        return _FlashFn.apply(qkv, B, S, Hq, Hkv, D, causal, window, scale, kv_start, rope, rope_done)
    q = qkv[:, : Hq * D]
    k = qkv[:, Hq * D:(Hq + Hkv) * D]
    v = qkv[:, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D]
    return native().attn_fwd(q, k, v, B, S, S, Hq, Hkv, D, causal, window, scale, kv_start, None, None, 0, False)[0]


def packed_inverse(idx: torch.Tensor, R: int) -> torch.Tensor:
    """int32 [R]: the packed row of every grid row (-1 for pad rows) — the scatter's index."""
    inv = torch.full((R,), -1, dtype=torch.int32, device=idx.device)
    inv[idx] = torch.arange(idx.numel(), dtype=torch.int32, device=idx.device)
    return inv


def _scatter_rows_raw(src, idx, inv, R):
    if on_gpu(src) and src.dtype == torch.bfloat16:
        return native().rows_scatter(src, inv, R)
    return src.new_zeros(R, src.shape[1]).index_copy(0, idx, src)


def _gather_rows_raw(src, idx):
    if on_gpu(src) and src.dtype == torch.bfloat16:
        return native().embed(src.contiguous(), idx, None, None)
    return src.index_select(0, idx)


class _ScatterRows(torch.autograd.Function):
    """[N, W] packed rows -> [R, W] grid (zeros on pad rows) in one native pass; backward gathers."""

    @staticmethod
    def forward(ctx, src, idx, inv, R):
        ctx.save_for_backward(idx)
        return _scatter_rows_raw(src, idx, inv, R)

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        return _gather_rows_raw(g, idx), None, None, None


class _GatherRows(torch.autograd.Function):
    """[R, W] grid -> its [N, W] real rows (native gather); backward scatters with zero pads."""

    @staticmethod
    def forward(ctx, src, idx, inv):
        ctx.save_for_backward(idx, inv)
        ctx.R = src.shape[0]
        return _gather_rows_raw(src, idx)

    @staticmethod
    def backward(ctx, g):
        idx, inv = ctx.saved_tensors
        return _scatter_rows_raw(g.contiguous(), idx, inv, ctx.R), None, None


def scatter_rows(src, idx, inv, R):
    return _ScatterRows.apply(src, idx, inv, R)


def gather_rows(src, idx, inv):
    return _GatherRows.apply(src, idx, inv)


def flash_attention_packed(qkv_p, idx, B, S, Hq, Hkv, D, causal=True, window=0, scale=None, kv_start=None,
                           rope=None, inv=None, rope_done=False):
    """Varlen self-attention over PACKED token rows (no pad rows in the GEMMs around it).

    ``qkv_p`` [N, W] holds only real tokens; ``idx`` [N] (int64) is each row's position b*S + s in
    the [B, S] grid the attention kernels tile. The rows are scattered into a zeroed grid (pad
    keys stay zero: left pads are masked by ``kv_start``, right pads lie after every real query of
    their row under the causal mask), attended with the usual kernels, and the real output rows
    gathered back. Scatter / gather move ~40 KB per token per layer against ~0.4 GFLOP of
    projection GEMMs per token per layer that no longer run on pads (both differentiable, one
    native pass each: ``inv`` = packed_inverse(idx, B*S), computed once per forward)."""
    if inv is None:
        inv = packed_inverse(idx, B * S)
    grid = scatter_rows(qkv_p, idx, inv, B * S)
    o = flash_attention_qkv(grid, B, S, Hq, Hkv, D, causal, window, scale, kv_start, rope, rope_done)
    return gather_rows(o, idx, inv)


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
def decode_partition(batch_heads: int, D: int = 128, Smax: int = 4096) -> int:
    """Keys per split-K partition of the fused decode kernel. A partition is a whole number of
    key chunks (4 waves x 64/(D/8) keys x 4 keys per lane). With >= 256 (batch, kv-head) pairs the
    grid already fills the chip: one partition per pair (no cross-block combine); with fewer pairs
    the keys are split so that ~256 workgroups run (at most 8 partitions of at least 2 chunks each:
    the in-launch combine costs more than a third partition of a short cache saves), merged
    in-launch by the last arriver. Batch 1 (MI355X, profiles/kernels_attn_fused_b1_partition_sweep.log):
    456 keys -> 2-chunk partitions (15.4 vs 16.5 us at 1 chunk), 2048 keys -> 4 chunks (22.2 vs 34.7)."""
    chunk = 4 * (64 // (D // 8)) * 4
    nchunks = (Smax + chunk - 1) // chunk
    if batch_heads >= 256:
        return nchunks * chunk
    want_np = min(8, max(1, -(-256 // batch_heads)))
    per = max(2, -(-nchunks // want_np))
    return min(per, nchunks) * chunk


class DecodeWorkspace(tuple):
    """(partials fp32, keys per partition, tickets int32) — static buffers reused by graph replays.
    Tickets are zero between launches (the merging partition re-arms them)."""

    @property
    def part(self):
        return self[0]

    @property
    def PS(self):
        return self[1]

    @property
    def tickets(self):
        return self[2]


def decode_workspace(B, Hq, Hkv, D, Smax, device, PS=None):
    PS = PS or decode_partition(B * Hkv, D, Smax)
    NP = (Smax + PS - 1) // PS
    # records of D + 2 floats (o | m | l) per (batch, kv head, partition, query head)
    part = torch.empty(B * (D + 2) * Hkv * NP * (Hq // Hkv), dtype=torch.float32, device=device)
    tickets = torch.zeros(B * Hkv, dtype=torch.int32, device=device)
    return DecodeWorkspace((part, PS, tickets))


# ----------------------------------------------------------------------------- fp8 K/V cache
# Config 5 keeps the rollout KV cache in OCP e4m3fn with one fp32 scale per
# (batch row, kv head, slot): absmax / 448 of the rotated head row. K rows are stored
# k-permuted so that one lane of the MFMA decode kernel reads its four 8-element K chunks as 32
# contiguous bytes: element d = 32 s + 8 g + e lives at byte 32 g + 8 s + e (D = 128). V rows are
# stored in order. Half the cache bytes of bf16: the decode attention of the 13B MHA model is a
# pure K/V stream (csrc/kernels/attention.hip, attn_decode_mfma_kernel<KV8>).
FP8_KV_D = 128


def fp8_kv_perm(D: int = FP8_KV_D) -> torch.Tensor:
    """byte position of element d in a stored K row."""
    d = torch.arange(D)
    return 32 * ((d % 32) // 8) + 8 * (d // 32) + d % 8


def kv_quantize_rows(x: torch.Tensor, permute: bool):
    """[..., D] -> (e4m3fn bytes [..., D] (k-permuted if ``permute``), fp32 scales [...]) — the
    same rounding as the kernels (scale = amax / 448, x / scale rounded to nearest even)."""
    xf = x.float()
    amax = xf.abs().amax(-1)
    sc = torch.where(amax > 0, amax / 448.0, torch.ones_like(amax))
    q = (xf * (1.0 / sc)[..., None]).to(torch.float8_e4m3fn).view(torch.uint8)
    if permute:
        out = torch.empty_like(q)
        out[..., fp8_kv_perm(x.shape[-1]).to(q.device)] = q
        q = out
    return q, sc


def kv_dequantize(q: torch.Tensor, sc: torch.Tensor, permute: bool) -> torch.Tensor:
    """inverse of ``kv_quantize_rows`` -> fp32 [..., D]"""
    if permute:
        q = q[..., fp8_kv_perm(q.shape[-1]).to(q.device)]
    return q.view(torch.float8_e4m3fn).float() * sc[..., None]


def kv_store_fp8(qkv: torch.Tensor, k_cache, v_cache, k_scale, v_scale, B: int, S: int, Hq: int):
    """rotated prompt rows qkv [B*S, ...] -> fp8 cache slots [0, S) of [B, Hkv, Smax, D] (+ scales)."""
    _, Hkv, Smax, D = k_cache.shape
    if on_gpu(qkv):
        native().kv_store_fp8(qkv, k_cache, v_cache, k_scale, v_scale, B, S, Hq)
        return
    k = qkv[:, Hq * D:(Hq + Hkv) * D].reshape(B, S, Hkv, D).transpose(1, 2)
    v = qkv[:, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D].reshape(B, S, Hkv, D).transpose(1, 2)
    kq, ks = kv_quantize_rows(k, True)
    vq, vs = kv_quantize_rows(v, False)
    k_cache[:, :, :S] = kq
    v_cache[:, :, :S] = vq
    k_scale[:, :, :S] = ks
    v_scale[:, :, :S] = vs


def _decode_step_fp8kv_cpu(qkv, k_cache, v_cache, k_scale, v_scale, slot, attn_len, Hq, pos, cos, sin, kv_start,
                           window, scale, out, sign):
    B, Hkv, Smax, D = k_cache.shape
    q = rope_qkv_(qkv.clone(), pos, cos, sin, Hq, Hkv, D, S=1, sign=sign)
    kq, ks = kv_quantize_rows(q[:, Hq * D:(Hq + Hkv) * D].reshape(B, Hkv, D), True)
    vq, vs = kv_quantize_rows(q[:, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D].reshape(B, Hkv, D), False)
    for b in range(B):
        s = int(slot[b])
        k_cache[b, :, s], v_cache[b, :, s] = kq[b], vq[b]
        k_scale[b, :, s], v_scale[b, :, s] = ks[b], vs[b]
    kd = kv_dequantize(k_cache, k_scale[..., :Smax], True).to(qkv.dtype)
    vd = kv_dequantize(v_cache, v_scale[..., :Smax], False).to(qkv.dtype)
    return decode_attention(q, kd, vd, attn_len, Hq, kv_start, window, scale, out=out)


def decode_step_attention(qkv, k_cache, v_cache, slot, attn_len, Hq, pos=None, cos=None, sin=None, kv_start=None,
                          window=0, scale=None, workspace=None, out=None, sign: float = 1.0, k_scale=None,
                          v_scale=None, stamps=None):
    """One decode step of a layer, fused: rotate q / k_new (if ``cos`` is given), append k_new and
    v_new at cache slot ``slot[b]``, attend over ``attn_len[b]`` keys -> [B, Hq*D].
    ``qkv`` [B, (Hq + 2 Hkv) D] is left unrotated (the fused kernel rotates in registers).
    ``k_scale`` / ``v_scale`` [B, Hkv, SmaxP]: the caches are fp8 (uint8) — see ``kv_store_fp8``.
    ``stamps``: debug int64 buffer for the 8-wave kernel's per-block phase stamps (tools/)."""
    from .linear import SplitK

    B, Hkv, Smax, D = k_cache.shape
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    fp8kv = k_scale is not None
    if isinstance(qkv, SplitK):
        # the qkv GEMM's split-K partials: summed in the MFMA kernel's prologue when it applies
        if workspace is None or len(workspace) < 3:
            workspace = decode_workspace(B, Hq, Hkv, D, Smax, k_cache.device)
        if out is None:
            out = torch.empty(B, Hq * D, dtype=qkv.dtype, device=qkv.device)
        if native().attn_decode_fused_slabs(qkv.slabs, qkv.nsplit, k_cache, v_cache, slot, attn_len, kv_start, pos,
                                            cos, sin, sign, window, scale, Hq, workspace[0], workspace[2],
                                            workspace[1], out, k_scale, v_scale):
            return out
        qkv = qkv.reduce()
    if not on_gpu(qkv):
        if fp8kv:
            return _decode_step_fp8kv_cpu(qkv, k_cache, v_cache, k_scale, v_scale, slot, attn_len, Hq, pos, cos, sin,
                                          kv_start, window, scale, out, sign)
        q = rope_qkv_(qkv.clone(), pos, cos, sin, Hq, Hkv, D, S=1, k_cache=k_cache, v_cache=v_cache,
                      slot_base=slot, sign=sign)
        return decode_attention(q, k_cache, v_cache, attn_len, Hq, kv_start, window, scale, out=out)
    if workspace is None or len(workspace) < 3:
        workspace = decode_workspace(B, Hq, Hkv, D, Smax, qkv.device)
    part, PS, tickets = workspace[0], workspace[1], workspace[2]
    if out is None:
        out = torch.empty(B, Hq * D, dtype=qkv.dtype, device=qkv.device)
    native().attn_decode_fused(qkv, k_cache, v_cache, slot, attn_len, kv_start, pos, cos, sin, sign, window, scale,
                               Hq, part, tickets, PS, out, k_scale, v_scale, stamps)
    return out


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
    part, PS = workspace[0], workspace[1]
    if out is None:
        out = torch.empty(B, Hq * D, dtype=q.dtype, device=q.device)
    native().attn_decode(q, k_cache, v_cache, kv_len, kv_start, window, scale, Hq, part, PS, out)
    return out
