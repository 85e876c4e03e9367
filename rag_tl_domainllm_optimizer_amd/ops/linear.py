"""Linear projections: frozen/trainable base weight + fused LoRA adapters + bias/activation.

Every GPU GEMM is a hand-written MFMA kernel; dispatch is by shape only (no library backend):
  * M <= 64 (decode, small batch): the weight-streaming kernels of gemm_bf16.hip (split-K,
    in-GEMM RMS-norm, SwiGLU / residual epilogues);
  * M > 64 (prefill, reference scoring, training): the 256x256 MFMA family of gemm_big.hip in
    three operand layouts — NT forward, NN input gradient (W read transposed in-kernel), TN weight
    / LoRA gradients (split-K, fp32).

LoRA: ``Y = act(X W^T + U UB^T + b)`` with ``U = X A_pad^T`` (A_pad = scaling x A,
zero-padded to a multiple of 64 rows). U is a narrow split-K pass; ``U UB^T`` then rides on the
base GEMM's accumulators as extra K-steps (the K-extension operands of gemm_big), so the adapter
product needs no output pass and no concatenated copy. Several adapters on one fused projection
(q|k|v, gate|up) share one padded rank dimension, with UB block-diagonal.
Backward: dX = dY W + dU A_pad (one NN GEMM with the same K-extension), dU = dY UB,
dA = s dU^T X, dB = dY^T U (TN, fp32), dW = dY^T X (full fine-tuning).
The reference runs these products through HF/PyTorch (reinforcement_learning_optimization_after_rag
.py:200-209 forward, :229 backward).
"""
from __future__ import annotations

import contextlib
import threading
from dataclasses import dataclass, field
from typing import List, Optional

import torch

from . import reference as ref
from ._ext import native, on_gpu

ACT_IDS = {None: 0, "none": 0, "relu": 1, "gelu": 2, "gelu_tanh": 3, "gelu_new": 3, "silu": 4, "swiglu": 5}
ACT_SWIGLU = 5  # w = [gate; up] (2F rows) -> silu(x gate^T) * (x up^T), [.., F]
ACT_DSWIGLU = 6  # gemm_big NN epilogue: d[gate | up] from dF and the [gate | up] pre-activation


def splitk_plan(M: int, N: int, K: int, act: int = 0):
    """(nsplit, bn) for a token-parallel NT GEMM. Up to 512 rows (decode at batch 65..512, small
    prefills) the 256x128 tile doubles the workgroups over the 256x256 one, and the K split fills
    the rest of the chip (qkv 48 tiles x 5, o / down 32 x 8, gate_up 224 x 1 with the SwiGLU in the
    epilogue, lm_head 250 x 1). Larger M: one launch planned by rt_gemm_big (bn 0: 256x256 tiles,
    the last partial wave on 256x128 tiles)."""
    if M > 512:
        return 1, 0
    bn = 128 if act in (0, ACT_SWIGLU) else 256
    tiles = ((M + 255) // 256) * (N // bn if act == ACT_SWIGLU else (N + bn - 1) // bn)
    if tiles >= 128:
        return 1, bn
    nk = (K + 63) // 64
    return max(1, min(nk // 8, (256 + tiles // 2) // tiles)), bn


_BI = threading.local()  # per-thread nesting depth of batch_invariant() (a serving thread keeps its plans)


def _batch_invariant_on() -> bool:
    return getattr(_BI, "depth", 0) > 0


@contextlib.contextmanager
def batch_invariant(on: bool = True):
    """Row-invariant GEMM numerics inside the block: every token-parallel GEMM (``gemm``) runs the
    gemm_big kernel without a K split whatever M is, so a row's output bits do not depend on how
    many other rows share the launch (no M-dependent split-K / skinny-kernel choice; gemm_big's
    256- and 128-column tiles accumulate every element in the same K order). The PPO scoring
    forwards (``train.common.score_sequences``) run under it: reference log-probs, the optional
    theta_old recompute and the update forward then agree bitwise across minibatch sizes,
    padding and packing. Costs nothing at scoring sizes (M in the thousands never splits)."""
    d = int(bool(on))
    _BI.depth = getattr(_BI, "depth", 0) + d
    try:
        yield
    finally:
        _BI.depth -= d


def gemm(x: torch.Tensor, w: torch.Tensor, u=None, ub=None, bias=None, act=0, out_f32=False, out=None,
         residual=None, nsplit: int = 0):
    """Raw (non-autograd) fused GEMM on 2-D row-major operands: act(x w^T + u ub^T + bias) (+ residual).
    M <= 64: weight-streaming kernels; small M with few output tiles: split-K fp32 slabs + fused
    reduce epilogue (``nsplit`` overrides the plan); otherwise the 256x256 MFMA kernel. Under
    :func:`batch_invariant` always the 256x256-family kernel without a split."""
    if on_gpu(x):
        M, K = x.shape
        N = w.shape[0]
        if _batch_invariant_on() and K % 8 == 0 and (act != ACT_SWIGLU or N % 256 == 0) \
                and (residual is None or not out_f32):
            return native().gemm_big(x, w, ROW, ROW, u, ub, bias, act, 1 if out_f32 else 0, 1, out, None, residual, 0)
        # 32 <= M <= 64 on narrow weights (qkv / o): the 256x128-tile split-K form beats the ring
        # kernel by 2-4 us (profiles/gemm_r2_m32_m64_ring_vs_splitk.log), and the 256-row wide kernel
        # beats both where it applies (N % 256 == 0: qkv 22.4 -> 19.0, o 18.2 -> 15.4 us at M = 64,
        # profiles/r6/m64_wide_probe.log); wide / deep weights and M < 32 stay on the native kernels
        narrow_split = 32 <= M <= 64 and N <= 8192 and K <= 8192 and N % 16 == 0 and act == 0 and u is None \
            and not out_f32 and bias is None and residual is None and nsplit == 0 and (N % 256 or K % 64)
        if M <= 64 and residual is None and N % 8 == 0 and not narrow_split:
            return native().gemm(x, w, u, ub, bias, act, out_f32, out)
        s, bn = splitk_plan(M, N, K, act)
        if narrow_split:
            s, bn = max(s, 2), 128
        if nsplit:
            s = nsplit
        if u is not None or out_f32 or N % 16:
            s = 1
        if s > 1:
            slabs = torch.empty(s * M * N, dtype=torch.float32, device=x.device)
            return native().gemm_splitk(x, w, s, slabs, bias, act, out, residual, bn or 256)
        return native().gemm_big(x, w, ROW, ROW, u, ub, bias, act, 1 if out_f32 else 0, 1, out, None, residual, bn)
    y = ref.gemm(x, w, u, ub, bias, act, out_f32)
    if residual is not None:
        y = (y.float() + residual.float()).to(y.dtype)
    if out is not None:
        out.copy_(y)
        return out
    return y


ROW, KMAJ = 0, 1  # operand layouts of the token-parallel GEMM family (csrc/kernels/gemm_big.hip)


def _op(t: torch.Tensor, layout: int, trans_for_a: bool) -> torch.Tensor:
    """Logical operand of the CPU oracle: A as [M, K] / B as [K, N]."""
    if trans_for_a:
        return t if layout == ROW else t.t()
    return t.t() if layout == ROW else t


def gemm_big(a, b, la: int, lb: int, a2=None, b2=None, bias=None, act: int = 0, out_mode: int = 0,
             nsplit: int = 1, out=None, out2=None, residual=None, bn: int = 0):
    """C = epi(A·B + A2·B2) with per-operand layouts (ROW: K contiguous, KMAJ: M / N contiguous).
    GPU: one hand-written MFMA kernel (gemm_big_kernel); CPU: fp32 oracle (tests, plumbing).
    out_mode 0 bf16 / 1 fp32 / 2 fp32 accumulate into ``out``; act 5 = SwiGLU over [gate; up].
    bn: 256 / 128 output columns per tile, 0 = planned (256, the last partial wave on 128)."""
    if on_gpu(a):
        return native().gemm_big(a, b, la, lb, a2, b2, bias, act, out_mode, nsplit, out, out2, residual, bn)
    A = _op(a, la, True).float()
    B = _op(b, lb, False).float()
    y = A @ B
    if a2 is not None:
        y = y + _op(a2, la, True).float() @ _op(b2, lb, False).float()
    if act == ACT_DSWIGLU:  # out = d[gate | up] from dF = y (rounded like the GEMM output) and residual
        from .misc import _swiglu_grad

        out.copy_(_swiglu_grad(residual, y.to(a.dtype)))
        return out
    if act == ACT_SWIGLU:
        F = y.shape[1] // 2
        pre = y.to(a.dtype)
        if out2 is not None:
            out2.copy_(pre)
        g, u = pre[:, :F].float(), pre[:, F:].float()
        y = torch.nn.functional.silu(g) * u
    else:
        if bias is not None:
            y = y + bias.float()
        y = ref.apply_act(y, act)
        if residual is not None:
            y = y.to(a.dtype).float() + residual.float()
    if out_mode == 2:
        out.add_(y)
        return out
    y = y.to(a.dtype if out_mode == 0 else torch.float32)
    if out is not None:
        out.copy_(y)
        return out
    return y


def gemm_nn(dy: torch.Tensor, w: torch.Tensor, du=None, a_pad=None) -> torch.Tensor:
    """dX = dY W (+ dU A_pad): W [N, K] is read K-contiguous-transposed in-kernel (no W^T copy)."""
    return gemm_big(dy, w, ROW, KMAJ, du, a_pad)


def gemm_tn(a: torch.Tensor, b: torch.Tensor, nsplit: int = 0, out=None, zeroed: bool = False) -> torch.Tensor:
    """a^T b in fp32 (weight / LoRA gradients): a [T, P], b [T, Q] -> [P, Q]; the token reduction
    is split over ``nsplit`` workgroup rows (0 = fill the chip) with fp32 atomic accumulation.
    Narrow outputs (a LoRA rank side of 64) run on the 64x64-tile kernel, wide ones on gemm_big.
    ``zeroed``: ``out`` is already zero (one fill shared by several products)."""
    T, P = a.shape
    Q = b.shape[1]
    if out is None:
        out = torch.zeros(P, Q, dtype=torch.float32, device=a.device)
    elif not zeroed:
        out.zero_()
    if not on_gpu(a):
        out.add_(a.float().t() @ b.float())
        return out
    if min(P, Q) <= 128:
        # 128x64 tiles when the wide side is A and very wide (dB of gate_up, P = 28672: 152 -> 121
        # us at 9632 tokens, profiles/r3/small_bm_probe.log); narrower products lose parallelism
        bm = 128 if P >= 16384 else 64
        tiles = ((P + bm - 1) // bm) * ((Q + 63) // 64)
        # token split: 4 ways on 64 tiles, 8 above (fewer fp32 atomic partials than filling the chip
        # 4x over: dA / dB at 9632 tokens 32.7 -> 27.1 us (K / N = 4096), 46.0 -> 39.9 us (N =
        # 6144), profiles/r5/lora_narrow_split_sweep.log)
        ns = nsplit or max(1, min(T // 256, 4 if tiles <= 64 else 8))
        return native().gemm_small(a, b, KMAJ, KMAJ, 2, ns, out, bm)
    tiles = ((P + 255) // 256) * ((Q + 255) // 256)
    ns = nsplit or max(1, min(64, 256 // max(tiles, 1), T // 512))
    return gemm_big(a, b, KMAJ, KMAJ, out_mode=2, nsplit=ns, out=out)


@dataclass
class LoRAGroup:
    """Adapters attached to one (possibly fused) projection.

    ``a[i]`` [r_i, K] and ``b[i]`` [n_i, r_i] are the trainable fp32 parameters of adapter i,
    which writes output columns ``[col0[i], col0[i] + n_i)`` with scale ``scale[i]``.
    ``a_pad`` [Rp, K] and ``ub`` [N, Rp] are the bf16 compute images (rebuilt by ``refresh``).
    """

    names: List[str]
    a: List[torch.nn.Parameter]
    b: List[torch.nn.Parameter]
    col0: List[int]
    scale: List[float]
    n_out: int
    a_pad: Optional[torch.Tensor] = None
    ub: Optional[torch.Tensor] = None
    r0: List[int] = field(default_factory=list)
    enabled: bool = True
    # inference mode: W' = W + UB A_pad materialised once per adapter update (decode / prefill of
    # rollouts read one merged weight stream instead of running the rank-Rp K-extension)
    use_merged: bool = False
    merged: Optional[torch.Tensor] = None
    merged_dirty: bool = True
    # PEFT lora_dropout on the adapter input (training forwards only)
    dropout: float = 0.0

    @property
    def rank_total(self) -> int:
        return sum(int(a.shape[0]) for a in self.a)

    @property
    def rp(self) -> int:
        return max(64, (self.rank_total + 63) // 64 * 64)

    @torch.no_grad()
    def refresh(self, dtype=torch.bfloat16):
        """Rebuild the padded bf16 images from the fp32 parameters (after each optimizer step)."""
        K = self.a[0].shape[1]
        dev = self.a[0].device
        rp = self.rp
        if self.a_pad is None or self.a_pad.shape != (rp, K) or self.a_pad.device != dev:
            self.a_pad = torch.zeros(rp, K, dtype=dtype, device=dev)
            self.ub = torch.zeros(self.n_out, rp, dtype=dtype, device=dev)
        self.r0 = []
        r = 0
        for a, b, c0, s in zip(self.a, self.b, self.col0, self.scale):
            ri = a.shape[0]
            self.r0.append(r)
            self.a_pad[r:r + ri].copy_(a.detach() * s)
            self.ub[c0:c0 + b.shape[0], r:r + ri].copy_(b.detach())
            r += ri
        self.merged_dirty = True

    @torch.no_grad()
    def merged_weight(self, w: torch.Tensor, rows_per_chunk: int = 4096) -> torch.Tensor:
        """W + UB A_pad, updated IN PLACE so captured graphs that read it stay valid across adapter
        updates. On the GPU one NN GEMM (K = Rp) with W as the residual input of its epilogue: 4 B
        of traffic per weight element. Rounding: UB A_pad is accumulated in fp32 and rounded to
        bf16, then W is added in fp32 and the sum rounded again — two bf16 roundings, bitwise what
        a GEMM followed by a separate add kernel gives (the CPU path rounds once)."""
        if self.merged is None or self.merged.shape != w.shape or self.merged.device != w.device:
            self.merged = torch.empty(w.shape, dtype=w.dtype, device=w.device)
            self.merged_dirty = True
        if self.merged_dirty:
            if on_gpu(w) and w.dtype == torch.bfloat16:
                native().gemm_big(self.ub, self.a_pad, ROW, KMAJ, None, None, None, 0, 0, 1, self.merged, None, w)
                # a native write leaves the version counter alone: bump it so the caches derived
                # from the merged weight (norm fold, fp8, shuffled decode image) see the update
                torch.autograd.graph.increment_version(self.merged)
            else:
                for r0 in range(0, w.shape[0], rows_per_chunk):
                    r1 = min(w.shape[0], r0 + rows_per_chunk)
                    self.merged[r0:r1].copy_(torch.addmm(w[r0:r1].float(), self.ub[r0:r1].float(),
                                                         self.a_pad.float()))
            self.merged_dirty = False
        return self.merged


_SCATTER_TABLES: dict = {}


def refresh_lora_batched(groups: List["LoRAGroup"], dtype=torch.bfloat16) -> bool:
    """Rebuild the bf16 compute images (``a_pad`` = scaled A rows, ``ub`` = B blocks) of many LoRA
    groups in ONE native launch (``scatter_scaled``) instead of ``LoRAGroup.refresh``'s two torch
    copies and a scale per adapter — after every optimizer step that was ~7 x 3 launches per layer.
    The descriptor table (device int64) is cached per set of buffer addresses. Returns False when
    the groups are not fp32-parameter / bf16-image GPU groups (the caller refreshes eagerly)."""
    import struct

    if not groups or dtype != torch.bfloat16 or not on_gpu(groups[0].a[0]):
        return False
    rows, key = [], []
    for g in groups:
        K = g.a[0].shape[1]
        if g.a_pad is None or g.a_pad.shape != (g.rp, K) or g.a_pad.dtype != dtype or g.a_pad.device != g.a[0].device:
            g.refresh(dtype=dtype)  # allocates the images (and fills them this once)
        if not g.r0:
            r = 0
            for a in g.a:
                g.r0.append(r)
                r += a.shape[0]
        rp = g.ub.shape[1]
        for a, b, r0, c0, sc in zip(g.a, g.b, g.r0, g.col0, g.scale):
            if a.dtype != torch.float32 or b.dtype != torch.float32 or a.stride(1) != 1 or b.stride(1) != 1:
                return False
            ri, ni = a.shape[0], b.shape[0]
            bits = struct.unpack("<i", struct.pack("<f", float(sc)))[0]
            rows.append((a.data_ptr(), a.stride(0), g.a_pad.data_ptr() + 2 * r0 * g.a_pad.stride(0),
                         g.a_pad.stride(0), ri, K, bits))
            rows.append((b.data_ptr(), b.stride(0), g.ub.data_ptr() + 2 * (c0 * rp + r0), rp, ni, ri,
                         struct.unpack("<i", struct.pack("<f", 1.0))[0]))
        g.merged_dirty = True
    key = (groups[0].a[0].device, tuple(rows))
    ent = _SCATTER_TABLES.get(key)
    if ent is None:
        if len(_SCATTER_TABLES) > 8:
            _SCATTER_TABLES.clear()
        tab = torch.tensor(rows, dtype=torch.int64).to(groups[0].a[0].device)
        ent = _SCATTER_TABLES[key] = (tab, max(r[4] * r[5] for r in rows))
    native().scatter_scaled(ent[0], ent[1])
    return True


_WS: dict = {}


def _workspace(key, n: int, device) -> torch.Tensor:
    """A cached fp32 buffer of >= n elements (split-K slabs of the LoRA backward products: fully
    overwritten by every producer, consumed in stream order before the next one reuses it)."""
    k = (key, str(device))
    t = _WS.get(k)
    if t is None or t.numel() < n:
        t = _WS[k] = torch.empty(max(n, 1), dtype=torch.float32, device=device)
    return t[:n]


def _tn_slabs(a: torch.Tensor, b: torch.Tensor, key):
    """Narrow a^T b (a [T, P], b [T, Q], min(P, Q) <= 128: the LoRA dA / dB products) as fp32
    split-K slabs [ns, P, Q] in a cached workspace: every token split stores its partial tile with
    plain stores and the consumer sums the ns slabs in a fixed order — bitwise reproducible, unlike
    the fp32 atomics of gemm_tn (partials added in arrival order). Same tiles and token splits as
    gemm_tn's tiles. Returns (slabs [ns * P, Q], ns)."""
    T, P = a.shape
    Q = b.shape[1]
    bm = 128 if P >= 16384 else 64
    # token splits re-swept with slabs (no atomic cost; profiles/r6/lora_narrow_sweep.log, 9632
    # tokens): 8 on the 64x64-tile products (dA at K = 4096, dB of o / down: 19.4 -> 17.8 us), 2 on
    # the 128x64-tile dB of gate_up (130.9 -> 118.5 us: its 224 tiles fill the chip; 8 slabs of
    # 7.3 MB each were the cost). Whole PPO step: same within noise (update 2.137-2.140 vs 2.138-2.145
    # s, same box, profiles/r6/bench_lora_slab_splits_ab.log)
    ns = max(1, min(T // 256, 2 if bm == 128 else 8))
    ws = _workspace(key, ns * P * Q, a.device).view(ns * P, Q)
    native().gemm_small(a, b, KMAJ, KMAJ, 3, ns, ws, bm)
    return ws, ns


def _narrow(a: torch.Tensor, b: torch.Tensor, lb: int, nsplit: int = 0) -> torch.Tensor:
    """a [M, K] (ROW) times a narrow operand b (ROW [R, K] or KMAJ [K, R]; R = padded LoRA rank) ->
    [M, R] bf16 on the 64x64-tile kernel (U = X A_pad^T forward, dU = dY UB backward). One
    workgroup per 64 tokens leaves most CUs idle at a few thousand tokens (151 workgroups at 9632
    tokens, each over a K of up to 28672), so the reduction is split until ~3 workgroups per CU
    are in flight: fp32 split-K slabs summed in a fixed order and rounded to bf16 once."""
    if not on_gpu(a):
        B = b.float().t() if lb == ROW else b.float()
        return (a.float() @ B).to(a.dtype)
    M, K = a.shape
    R = b.shape[0] if lb == ROW else b.shape[1]
    # 128x64 tiles over the deepest reductions (dU of gate_up, K = 28672: 125 -> 116 us)
    bm = 128 if K >= 24576 else 64
    tiles = ((M + bm - 1) // bm) * ((R + 63) // 64)
    # (measured at 9632 tokens: dU 383 -> 172 us at K = 28672, profiles/lora_narrow_r2.log). The
    # forward U (ROW adapter image) runs 3 ways split from cold activations: K = 4096 31.3 -> 28.7
    # us, K = 14336 78.0 -> 73.8 us (profiles/r5/lora_narrow_split_sweep.log)
    # The forward U (ROW adapter image) splits 3 ways into fp32 SLABS summed in a fixed order (fp32
    # atomics land in arrival order: not bitwise reproducible, nor batch-invariant — the PPO ratio
    # and reference KL need the scoring forward to be, ops.batch_invariant): K = 4096 31.3 -> 28.7
    # us, K = 14336 78.0 -> 73.8 us at 9632 tokens (profiles/r5/lora_narrow_split_sweep.log, atomic
    # form). The backward dU (KMAJ adapter image) splits the same way into slabs.
    auto = min(3, max(1, K // 512)) if lb == ROW else max(1, min(K // 512, (768 + tiles - 1) // tiles))
    if lb == KMAJ and bm == 128:
        auto = min(auto, 6)  # dU of gate_up (K = 28672): 6 slabs 115 vs 11 at 127-129 us (lora_narrow_sweep.log)
    ns = nsplit or auto
    if ns == 1:
        return native().gemm_small(a, b, ROW, lb, 0, 1, None, bm)
    if R % 8 == 0:
        slabs = native().gemm_small(a, b, ROW, lb, 3, ns, None, bm)
        return native().splitk_reduce(slabs, ns, M, R, torch.empty(M, R, dtype=a.dtype, device=a.device))
    out = torch.zeros(M, R, dtype=torch.float32, device=a.device)
    native().gemm_small(a, b, ROW, lb, 2, ns, out, bm)
    return out.to(a.dtype)


def _dropout_mask(x: torch.Tensor, p: float) -> torch.Tensor:
    """Inverted-dropout multiplier (0 or 1/(1-p)) of the adapter input."""
    keep = torch.empty_like(x, dtype=torch.float32).bernoulli_(1.0 - p)
    return (keep / (1.0 - p)).to(x.dtype)


def _fp8_train_ok(f8, x2, w, bias, act, lora) -> bool:
    """The config-5 fp8 training forward applies: a frozen base weight under LoRA (no dropout),
    W8A8-compatible shapes, no bias, plain or SwiGLU epilogue, M > 64, on the GPU."""
    if f8 is None or lora is None or lora.dropout > 0 or bias is not None or w.requires_grad or not on_gpu(x2) \
            or x2.shape[0] <= 64:
        return False
    from .fp8 import fp8_supported

    return fp8_supported(w) and x2.shape[1] % 128 == 0 and (act == 0 or (act == ACT_SWIGLU and w.shape[0] % 256 == 0))


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x2, w, bias, act, lora: Optional[LoRAGroup], f8, rope, *lora_params):
        u = ub = xd = None
        mask = None
        if lora is not None:
            xd = x2
            if lora.dropout > 0:
                mask = _dropout_mask(x2, lora.dropout)
                xd = x2 * mask
            u = _narrow(xd, lora.a_pad, ROW)  # [M, Rp] = drop(X) (s A)^T
            ub = lora.ub
        ctx.act = act
        ctx.lora = lora
        ctx.has_bias = bias is not None
        pre = None
        if _fp8_train_ok(f8, x2, w, bias, act, lora):
            # config 5: the frozen base product on the fp8 MFMA (W8A8: per-token x, per-channel W
            # scales), the adapter term as a bf16 K-extension of the same accumulators — its
            # operands pre-divided by the scales the epilogue applies. The backward stays bf16.
            from .fp8 import quantize_fp8

            wq, sw = f8.get(w)
            xq, sx = quantize_fp8(x2)
            u8 = (u.float() / sx[:, None]).to(x2.dtype)
            ub8 = (ub.float() / sw[:, None]).to(x2.dtype)
            if act == ACT_SWIGLU:
                pre = torch.empty(x2.shape[0], w.shape[0], dtype=x2.dtype, device=x2.device)
                y = native().gemm_fp8_lora(xq, sx, wq, sw, u8, ub8, ACT_SWIGLU, pre)
            else:
                y = native().gemm_fp8_lora(xq, sx, wq, sw, u8, ub8, 0, None)
        elif act == ACT_SWIGLU:
            # w = [gate; up]: ONE GEMM writes silu(g) * u and the [M, 2F] pre-activation (kept for
            # the SwiGLU backward) from its epilogue — no separate SwiGLU pass over the activations
            pre = torch.empty(x2.shape[0], w.shape[0], dtype=x2.dtype, device=x2.device)
            y = gemm_big(x2, w, ROW, ROW, u, ub, None, ACT_SWIGLU, out2=pre)
        elif rope is not None:
            # q / k rotated in the epilogue; the rotation's backward is the attention node's
            # (ops.flash_attention_qkv(..., rope_done=True) inverse-rotates dq / dk), so this node's
            # backward is the plain projection's
            y = gemm_rope(x2, w, u, ub, bias, rope)
        else:
            y = gemm(x2, w, u, ub, bias, act)
        # other activation epilogues: the pre-activation is recomputed in backward (no extra
        # activation-sized tensor is kept alive). The SwiGLU pre-activation and the dropout mask go
        # through save_for_backward like everything else, so non-reentrant activation
        # checkpointing frees them between forward and backward (and recomputes them)
        e = torch.empty(0)
        ctx.save_for_backward(x2, w, u if u is not None else e, bias if bias is not None else e,
                              pre if pre is not None else e, mask if mask is not None else e)
        return y

    @staticmethod
    def backward(ctx, dy):
        x2, w, u, bias, pre, mask = ctx.saved_tensors
        mask = mask if mask.numel() else None
        lora = ctx.lora
        dy = dy.contiguous()
        if ctx.act == ACT_SWIGLU:
            from .misc import _swiglu_grad

            dy = _swiglu_grad(pre, dy)  # d[gate | up]
        elif ctx.act != 0:
            # recompute pre-activation and apply the activation derivative
            ub = lora.ub if lora is not None else None
            pre = gemm(x2, w, u if lora is not None else None, ub, bias if ctx.has_bias else None, 0, out_f32=True)
            with torch.enable_grad():
                p = pre.detach().requires_grad_(True)
                yact = ref.apply_act(p, ctx.act)
                (g,) = torch.autograd.grad(yact, p, dy.float())
            dy = g.to(dy.dtype)
        needs = ctx.needs_input_grad
        db = None
        if ctx.has_bias and needs[2]:
            db = dy.float().sum(0).to(bias.dtype)
        dx, dw, lora_grads = _linear_bwd(dy, x2, w, u, lora, mask, needs[0], needs[1])
        return (dx, dw, db, None, None, None, None, *lora_grads)


# the LoRA backward's direct-to-.grad epilogue (A/B switch for tests)
DIRECT_LORA_GRADS = True


def _direct_grads_ok(lora: "LoRAGroup") -> bool:
    """The adapter gradients can be accumulated straight into the parameters' .grad buffers (fp32
    contiguous tensors already allocated on the device, e.g. views of a flat gradient buffer,
    ops.FlatParams) instead of being returned to autograd for an accumulate-add each."""
    if not DIRECT_LORA_GRADS or torch.is_grad_enabled():  # create_graph: gradients stay differentiable
        return False
    for p in lora.a + lora.b:
        g = p.grad
        if g is None or g.dtype != torch.float32 or not g.is_contiguous() or g.device != p.device:
            return False
    return True


def _grad_table(lora: "LoRAGroup", ga: torch.Tensor, nsa: int, gb: torch.Tensor, nsb: int):
    """Device descriptor table of lora_grad_accum for this group's slab workspaces and .grad
    buffers (cached per address set): each adapter's dA rows (scaled, summed over the nsa slabs of
    dA_all [Rp, K]) -> a.grad and its dB block (its own output rows and rank columns of the nsb slabs
    of dB_all [N, Rp]) -> b.grad. Entry: src, src row stride, dst, dst row stride, rows, cols,
    scale bits, slabs, slab stride (elements)."""
    import struct

    Rp, K = lora.a_pad.shape
    N = lora.ub.shape[0]
    key = (ga.data_ptr(), nsa, gb.data_ptr(), nsb, tuple(p.grad.data_ptr() for p in lora.a + lora.b),
           tuple(lora.scale))
    ent = getattr(lora, "_grad_tab", None)
    if ent is not None and ent[0] == key:
        return ent[1], ent[2]
    rows = []
    f = lambda x: struct.unpack("<i", struct.pack("<f", float(x)))[0]  # noqa: E731
    for a, b, r0, c0, sc in zip(lora.a, lora.b, lora.r0, lora.col0, lora.scale):
        ri, ni = a.shape[0], b.shape[0]
        rows.append((ga.data_ptr() + 4 * r0 * K, K, a.grad.data_ptr(), K, ri, K, f(sc), nsa, Rp * K))
        rows.append((gb.data_ptr() + 4 * (c0 * Rp + r0), Rp, b.grad.data_ptr(), ri, ni, ri, f(1.0), nsb, N * Rp))
    tab = torch.tensor(rows, dtype=torch.int64).to(ga.device)
    mx = max(rw[4] * rw[5] for rw in rows)
    lora._grad_tab = (key, tab, mx)
    return tab, mx


def _linear_bwd(dy, x2, w, u, lora, mask, need_x: bool, need_w: bool, dx_act: int = 0, dx_aux=None, dx_out=None):
    """Gradients of y = x W^T (+ s (drop(x) A^T) B^T) given dL/dy: (dX, dW, [dA_i, dB_i, ...]).
    ``dx_act`` = ACT_DSWIGLU: dX is the down projection's input gradient dF and goes through the
    SwiGLU backward in the dX GEMM's epilogue (``dx_aux`` = the [gate | up] pre-activation,
    ``dx_out`` = the d[gate | up] buffer it writes). On the GPU with .grad buffers in place
    (:func:`_direct_grads_ok`) the adapter gradients are accumulated into them by one native
    epilogue and returned as None."""
    dx = dw = None
    gpu = on_gpu(dy)
    direct = gpu and lora is not None and _direct_grads_ok(lora)
    # dU = dY UB [M, Rp]: split over N into fp32 slabs, summed in a fixed order and rounded once
    du = _narrow(dy, lora.ub, KMAJ) if lora is not None else None
    if need_x:
        if dx_act == ACT_DSWIGLU:
            assert mask is None
            dx = gemm_big(dy, w, ROW, KMAJ, du, lora.a_pad if lora is not None else None, act=ACT_DSWIGLU,
                          out=dx_out, residual=dx_aux)
        elif lora is not None and mask is None:
            # dX = dY W + dU A_pad in ONE NN GEMM (the adapter term as K-extension steps)
            dx = gemm_big(dy, w, ROW, KMAJ, du, lora.a_pad)
        else:
            dx = gemm_big(dy, w, ROW, KMAJ)
            if lora is not None:  # dropout: the adapter gradient flows through the mask
                dx = dx + gemm_big(du, lora.a_pad, ROW, KMAJ) * mask
    if need_w:
        # full fine-tuning: dW = dY^T X [N, K] (TN; bf16 compute-copy gradient)
        dw = gemm_big(dy, x2, KMAJ, KMAJ) if (gpu and w.dtype == torch.bfloat16) else \
            (dy.float().t() @ x2.float()).to(w.dtype)
    lora_grads = []
    if lora is not None:
        # all adapters of the projection in two TN GEMMs with fp32 output (bf16 in, fp32
        # accumulate): dA_all = dU^T drop(X) [Rp, K]; dB_all = dY^T U [N, Rp] (adapter i uses
        # its diagonal block)
        xd = x2 * mask if mask is not None else x2
        Rp, Kr, Nr = lora.ub.shape[1], x2.shape[1], dy.shape[1]
        if gpu and Rp <= 128:
            # token-split fp32 slabs (bitwise reproducible): summed by lora_grad_accum straight into
            # .grad (direct), else by one torch reduction each
            ga_s, nsa = _tn_slabs(du, xd, ("lora_ga", Rp, Kr))
            gb_s, nsb = _tn_slabs(dy, u, ("lora_gb", Nr, Rp))
            if not direct:
                ga_all, gb_all = ga_s.view(nsa, Rp, Kr).sum(0), gb_s.view(nsb, Nr, Rp).sum(0)
        else:
            ga_s, nsa, gb_s, nsb = gemm_tn(du, xd), 1, gemm_tn(dy, u), 1
            ga_all, gb_all = ga_s, gb_s
        if direct:
            tab, mx = _grad_table(lora, ga_s, nsa, gb_s, nsb)
            native().lora_grad_accum(tab, mx)
            # None to autograd: the parameters' AccumulateGrad nodes still run (with no gradient)
            # and fire their post-accumulate hooks after this backward returns, i.e. behind the
            # epilogue on the stream — parallel.GradSync's bucket readiness needs nothing else
            # (tests/test_zz_dist_gpu.py: ranks hold the same reduced gradient)
            return dx, dw, [None] * (2 * len(lora.a))
        one_scale = len(set(lora.scale)) == 1
        if one_scale:
            ga_all.mul_(lora.scale[0])  # one launch for every adapter of the projection
        for a, b, r0, c0, s in zip(lora.a, lora.b, lora.r0, lora.col0, lora.scale):
            ri, ni = a.shape[0], b.shape[0]
            ga = ga_all[r0:r0 + ri]
            lora_grads.append((ga if one_scale else ga * s).to(a.dtype))
            lora_grads.append(gb_all[c0:c0 + ni, r0:r0 + ri].to(b.dtype))
        # parameter order in forward(*lora_params) is a0, b0, a1, b1, ...
    return dx, dw, lora_grads


class _SwiGLUMLPFn(torch.autograd.Function):
    """The Llama / Mistral MLP as one autograd node: f = silu(x Wg^T) * (x Wu^T) (gate / up in one
    GEMM with the SwiGLU epilogue, LoRA as K-extension), d = f Wd^T (+ LoRA). Backward runs the down
    projection's dX GEMM with the SwiGLU backward in its epilogue (ACT_DSWIGLU): d[gate | up] comes
    straight out of that GEMM, so dF never goes to memory and there is no separate SwiGLU-backward
    pass (two [M, F] bf16 streams per layer and minibatch; the [gate | up] streams are read / written
    once either way). Numerics are bitwise those of the two-node form (dF is rounded to bf16 before
    the epilogue's arithmetic, which is swiglu_bwd_kernel's). LoRA without dropout, bf16 weights."""

    @staticmethod
    def forward(ctx, x2, w_gu, w_d, lora_gu, lora_d, n_gu: int, *lora_params):
        u_gu = _narrow(x2, lora_gu.a_pad, ROW) if lora_gu is not None else None
        pre = torch.empty(x2.shape[0], w_gu.shape[0], dtype=x2.dtype, device=x2.device)
        f = gemm_big(x2, w_gu, ROW, ROW, u_gu, lora_gu.ub if lora_gu is not None else None, None, ACT_SWIGLU,
                     out2=pre)
        u_d = _narrow(f, lora_d.a_pad, ROW) if lora_d is not None else None
        d = gemm(f, w_d, u_d, lora_d.ub if lora_d is not None else None, None, 0)
        e = torch.empty(0)
        ctx.lora_gu, ctx.lora_d, ctx.n_gu = lora_gu, lora_d, n_gu
        ctx.save_for_backward(x2, w_gu, w_d, u_gu if u_gu is not None else e, pre, f, u_d if u_d is not None else e)
        return d

    @staticmethod
    def backward(ctx, dd):
        x2, w_gu, w_d, u_gu, pre, f, u_d = ctx.saved_tensors
        needs = ctx.needs_input_grad
        dd = dd.contiguous()
        dpre = torch.empty_like(pre)
        _, dw_d, g_d = _linear_bwd(dd, f, w_d, u_d if ctx.lora_d is not None else None, ctx.lora_d, None, True,
                                   needs[2], dx_act=ACT_DSWIGLU, dx_aux=pre, dx_out=dpre)
        dx, dw_gu, g_gu = _linear_bwd(dpre, x2, w_gu, u_gu if ctx.lora_gu is not None else None, ctx.lora_gu, None,
                                      needs[0], needs[1])
        return (dx, dw_gu, dw_d, None, None, None, *g_gu, *g_d)


def swiglu_mlp(x: torch.Tensor, w_gu: torch.Tensor, w_d: torch.Tensor, lora_gu: Optional[LoRAGroup] = None,
               lora_d: Optional[LoRAGroup] = None, cpu: bool = False) -> Optional[torch.Tensor]:
    """Training-forward MLP through :class:`_SwiGLUMLPFn` when it applies (GPU, bf16, autograd on,
    LoRA without dropout, [gate; up] rows % 256); returns None otherwise (the caller runs the two
    ``linear`` calls). ``cpu``: also on CPU tensors (the fp32 oracles of every step; tests)."""
    shp = x.shape
    x2 = x.reshape(-1, shp[-1])
    lg = lora_gu if (lora_gu is not None and lora_gu.enabled) else None
    ld = lora_d if (lora_d is not None and lora_d.enabled) else None
    if not (on_gpu(x2) or cpu) or not torch.is_grad_enabled() or w_gu.shape[0] % 256 \
            or (on_gpu(x2) and w_gu.dtype != torch.bfloat16) \
            or w_d.shape[1] % 8 or any(g is not None and (g.dropout > 0 or g.use_merged) for g in (lg, ld)):
        return None
    params = []
    for g in (lg, ld):
        if g is not None:
            if g.a_pad is None or g.a_pad.device != x.device:
                g.refresh(dtype=w_gu.dtype)
            for a, b in zip(g.a, g.b):
                params += [a, b]
    if not (x2.requires_grad or w_gu.requires_grad or w_d.requires_grad or any(p.requires_grad for p in params)):
        return None
    n_gu = 2 * len(lg.a) if lg is not None else 0
    y = _SwiGLUMLPFn.apply(x2.contiguous(), w_gu, w_d, lg, ld, n_gu, *params)
    return y.reshape(*shp[:-1], w_d.shape[0])


def linear(x: torch.Tensor, w: torch.Tensor, bias=None, act=None, lora: Optional[LoRAGroup] = None, fp8=None):
    """y = act(x W^T (+ LoRA) + b) over the last dim of x. ``fp8`` (an ``ops.fp8.Fp8Cache``)
    enables the fp8 inference path for this weight (no-grad only; LoRA merged first)."""
    act_id = ACT_IDS[act] if not isinstance(act, int) else act
    shp = x.shape
    x2 = x.reshape(-1, shp[-1])
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    use_lora = lora is not None and lora.enabled
    if use_lora and (lora.a_pad is None or lora.a_pad.device != x.device):
        lora.refresh(dtype=w.dtype)
    grad_needed = torch.is_grad_enabled() and (
        x2.requires_grad or w.requires_grad or (bias is not None and bias.requires_grad)
        or (use_lora and any(p.requires_grad for p in lora.a + lora.b)))
    if act_id == ACT_SWIGLU:
        # SwiGLU is the GEMM epilogue. no-grad: skinny kernels for decode, gemm_big otherwise;
        # training (_LinearFn): gemm_big also writes the [gate | up] pre-activation for backward
        if on_gpu(x2) and grad_needed and bias is None and w.shape[0] % 256 == 0 \
                and x2.shape[1] % 8 == 0 and x2.shape[0] > 64 and w.dtype == torch.bfloat16 \
                and not (use_lora and lora.use_merged):
            params = []
            if use_lora:
                for a, b in zip(lora.a, lora.b):
                    params += [a, b]
            f8 = fp8.train_cache() if (fp8 is not None and fp8.train) else None
            y = _LinearFn.apply(x2, w, None, ACT_SWIGLU, lora if use_lora else None, f8, None, *params)
            return y.reshape(*shp[:-1], w.shape[0] // 2)
        if on_gpu(x2) and not grad_needed and bias is None and w.shape[0] % 256 == 0 and x2.shape[1] % 8 == 0 \
                and w.dtype == torch.bfloat16 and use_lora and not lora.use_merged and fp8 is None \
                and (x2.shape[0] > 64 or _batch_invariant_on()):
            # unmerged adapters without grad (reference / theta_old scoring): the training forward's
            # exact product — U = X A_pad^T as K-extension steps of the [gate; up] GEMM with the
            # SwiGLU epilogue — not the merged bf16 W + s B A (a second rounding of every weight)
            y = gemm_big(x2, w, ROW, ROW, _narrow(x2, lora.a_pad, ROW), lora.ub, None, ACT_SWIGLU)
            return y.reshape(*shp[:-1], w.shape[0] // 2)
        if on_gpu(x2) and not grad_needed and bias is None and w.shape[0] % 64 == 0 and x2.shape[1] % 64 == 0 \
                and (x2.shape[0] <= 64 or w.shape[0] % 256 == 0):
            w_eff = lora.merged_weight(w) if use_lora else w
            if fp8 is not None:
                from .fp8 import fp8_supported, gemm_fp8

                if fp8_supported(w_eff):
                    if x2.shape[0] <= 64:
                        shuf = fp8.shuf_ok(w_eff, x2.shape[0], ACT_SWIGLU)
                        q, sc = fp8.shuf(w_eff) if shuf else fp8.get(w_eff)
                        y = native().gemm_fp8(x2, None, q, sc, None, ACT_SWIGLU, None, None, 0.0, shuf)
                    else:
                        # prefill / reference scoring: W8A8 [gate | up] on the fp8 MFMA (2x the bf16
                        # rate) with SwiGLU paired in the GEMM epilogue
                        q, sc = fp8.get(w_eff)
                        y = gemm_fp8(x2, q, sc, act=ACT_SWIGLU)
                    return y.reshape(*shp[:-1], w.shape[0] // 2)
            y = gemm(x2, w_eff, None, None, None, ACT_SWIGLU)
            return y.reshape(*shp[:-1], w.shape[0] // 2)
        from .misc import swiglu

        return swiglu(linear(x, w, bias, None, lora, fp8))
    if fp8 is not None and not torch.is_grad_enabled():
        from .fp8 import fp8_supported, gemm_fp8

        w_eff = lora.merged_weight(w) if use_lora else w
        if fp8_supported(w_eff) and (x2.shape[0] > 64 or x2.shape[1] % 64 == 0):
            if on_gpu(x2) and fp8.shuf_ok(w_eff, x2.shape[0], act_id):
                qs, s = fp8.shuf(w_eff)
                y = native().gemm_fp8(x2, None, qs, s, bias, act_id, None, None, 0.0, True)
            else:
                q, s = fp8.get(w_eff)
                y = gemm_fp8(x2, q, s, bias, act_id)
            return y.reshape(*shp[:-1], w.shape[0])
    if use_lora and lora.use_merged and not torch.is_grad_enabled():
        y = gemm(x2, lora.merged_weight(w), None, None, bias, act_id)
        return y.reshape(*shp[:-1], w.shape[0])
    if not grad_needed:
        u = _narrow(x2, lora.a_pad, ROW) if use_lora else None
        y = gemm(x2, w, u, lora.ub if use_lora else None, bias, act_id)
    else:
        params = []
        if use_lora:
            for a, b in zip(lora.a, lora.b):
                params += [a, b]
        f8 = fp8.train_cache() if (fp8 is not None and fp8.train) else None
        y = _LinearFn.apply(x2, w, bias, act_id, lora if use_lora else None, f8, None, *params)
    return y.reshape(*shp[:-1], w.shape[0])


def gemm_rope(x2: torch.Tensor, w: torch.Tensor, u=None, ub=None, bias=None, rope=None) -> torch.Tensor:
    """y = rope(x2 w^T (+ u ub^T) + bias) with ``rope`` = (pos int32 [M], cos, sin [positions, D/2] fp32,
    rope_cols, D): output columns [0, rope_cols) are D-wide heads rotated at pos[row] (the q / k heads
    of a fused qkv projection); GPU: one gemm_big launch with the rotary epilogue (E_ROPE)."""
    pos, cos, sin, cols, D = rope
    if on_gpu(x2):
        return native().gemm_rope(x2, w, u, ub, bias, pos, cos, sin, cols, D)
    y = ref.gemm(x2, w, u, ub, bias, 0, False)
    return ref.rope_qkv(y, pos, cos, sin, cols // D, 0, D)


# model-level A/B switch of the rotary epilogue (tests compare both forms; no native state)
ROPE_EPILOGUE = True


def rope_fusable(x2: torch.Tensor, w: torch.Tensor, lora: Optional[LoRAGroup], fp8) -> bool:
    """The qkv projection takes the rotary epilogue: token-parallel bf16 GEMM on the GPU (M > 256,
    the gemm_big planner's regime; no fp8 form for this projection; LoRA unmerged or merged)."""
    M = x2.shape[0]
    return (ROPE_EPILOGUE and on_gpu(x2) and x2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and M > 256 and
            w.shape[0] % 8 == 0 and x2.shape[1] % 8 == 0 and fp8 is None and splitk_plan(M, w.shape[0], x2.shape[1], 0)[0] <= 1)


def linear_rope(x: torch.Tensor, w: torch.Tensor, bias=None, lora: Optional[LoRAGroup] = None, fp8=None, rope=None):
    """``linear`` of a fused qkv projection with its rotary embedding in the GEMM epilogue when that
    applies (``rope_fusable``). Returns (y, rotated): rotated = False leaves the rotation to the
    attention call as before (``rope`` = (pos, cos, sin, rope_cols, D), pos per row of x)."""
    shp = x.shape
    x2 = x.reshape(-1, shp[-1])
    if rope is None or not rope_fusable(x2, w, lora, fp8):
        return linear(x, w, bias, None, lora, fp8), False
    x2 = x2.contiguous()
    use_lora = lora is not None and lora.enabled
    if use_lora and (lora.a_pad is None or lora.a_pad.device != x.device):
        lora.refresh(dtype=w.dtype)
    grad_needed = torch.is_grad_enabled() and (
        x2.requires_grad or w.requires_grad or (bias is not None and bias.requires_grad)
        or (use_lora and any(p.requires_grad for p in lora.a + lora.b)))
    if grad_needed:
        params = []
        if use_lora:
            for a, b in zip(lora.a, lora.b):
                params += [a, b]
        y = _LinearFn.apply(x2, w, bias, 0, lora if use_lora else None, None, rope, *params)
    elif use_lora and lora.use_merged:
        y = gemm_rope(x2, lora.merged_weight(w), None, None, bias, rope)
    else:
        u = _narrow(x2, lora.a_pad, ROW) if use_lora else None
        y = gemm_rope(x2, w, u, lora.ub if use_lora else None, bias, rope)
    return y.reshape(*shp[:-1], w.shape[0]), True


class SplitK:
    """Unreduced split-K partial sums of an NT GEMM, ``slabs`` [nsplit, M, N] fp32: the reduce is
    left to the consumer (``ops.rms_norm`` with a residual, ``ops.decode_step_attention``), which
    sums the slabs in its own pass (decode at batch 65..512: no reduce launch, no bf16 round trip)."""

    __slots__ = ("slabs", "nsplit", "M", "N", "dtype", "device")

    def __init__(self, slabs, nsplit, M, N, dtype):
        self.slabs, self.nsplit, self.M, self.N, self.dtype = slabs, nsplit, M, N, dtype
        self.device = slabs.device

    @property
    def shape(self):
        return torch.Size((self.M, self.N))

    def reduce(self) -> torch.Tensor:
        out = torch.empty(self.M, self.N, dtype=self.dtype, device=self.device)
        return native().splitk_reduce(self.slabs, self.nsplit, self.M, self.N, out)


def linear_deferred(x: torch.Tensor, w: torch.Tensor, bias=None, lora: Optional[LoRAGroup] = None, fp8=None):
    """``linear`` for no-grad decode steps that may return a :class:`SplitK` (unreduced) when the
    plan splits K (no bias / activation, merged or absent LoRA); else a tensor. ``fp8`` (config 5):
    the W8A8 split-K form — per-token fp8 activations, each split's partial scaled in its epilogue,
    the same slab consumers (the o / down projections of a 13B layer are 40 output tiles: without
    the split they ran on 40 of 256 CUs)."""
    x2 = x.reshape(-1, x.shape[-1])
    use_lora = lora is not None and lora.enabled
    if (not on_gpu(x2) or torch.is_grad_enabled() or bias is not None or w.dtype != torch.bfloat16
            or x2.dtype != torch.bfloat16 or (use_lora and not lora.use_merged) or x2.shape[0] <= 64
            or w.shape[0] % 16 or x2.shape[1] % 8):
        return linear(x, w, bias, None, lora, fp8)
    w_eff = lora.merged_weight(w) if use_lora else w
    M, K = x2.shape
    N = w_eff.shape[0]
    if fp8 is not None:
        from .fp8 import fp8_supported, quantize_fp8

        if not fp8_supported(w_eff) or K % 128:
            return linear(x, w, bias, None, lora, fp8)
        s, bn = splitk_plan(M, N, K // 2, 0)  # an fp8 K-step is 128 bytes: half the bf16 steps
        if s <= 1:
            return linear(x, w, bias, None, lora, fp8)
        q, sc = fp8.get(w_eff)
        xq, sx = quantize_fp8(x2)
        slabs = torch.empty(s * M * N, dtype=torch.float32, device=x2.device)
        native().gemm_fp8_splitk_raw(xq, sx, q, sc, s, slabs, bn or 256)
        return SplitK(slabs, s, M, N, x2.dtype)
    s, bn = splitk_plan(M, N, K, 0)
    if s <= 1:
        return gemm(x2.contiguous(), w_eff).reshape(*x.shape[:-1], N)
    slabs = torch.empty(s * M * N, dtype=torch.float32, device=x2.device)
    native().gemm_splitk_raw(x2.contiguous(), w_eff, s, slabs, bn or 256)
    return SplitK(slabs, s, M, N, x2.dtype)


def gemm_decode(x: torch.Tensor, w: torch.Tensor, act: int = 0, residual=None, norm_eps: float = 0.0, fp8=None,
                shuf=None):
    """Decode-step GEMM (M <= 64) with the fused prologue/epilogue of the skinny kernels:
    ``C = act(rstd(x) * x w^T) + residual`` where ``rstd`` (``norm_eps > 0``) is the RMS-norm of
    each input row computed inside the GEMM (the norm weight must already be folded into ``w``)
    and ``act`` may be ACT_SWIGLU (w = [gate; up]). ``fp8`` (Fp8Cache) streams e4m3fn weights;
    ``shuf`` (ShufCache, M <= 16) streams the tile-ordered image of ``w`` instead."""
    if on_gpu(x):
        x = x.contiguous()
        if fp8 is not None:
            from .fp8 import fp8_supported

            if fp8_supported(w):
                if fp8.shuf_ok(w, x.shape[0], act):
                    qs, sc = fp8.shuf(w)
                    return native().gemm_fp8(x, None, qs, sc, None, act, None, residual, norm_eps, True)
                q, sc = fp8.get(w)
                return native().gemm_fp8(x, None, q, sc, None, act, None, residual, norm_eps)
        if shuf is not None and x.shape[0] <= 16 and w.shape[0] % 16 == 0:
            return native().gemm(x, shuf.get(w), None, None, None, act, False, None, residual, norm_eps, True)
        return native().gemm(x, w, None, None, None, act, False, None, residual, norm_eps)
    y = x.float() @ w.float().t()
    if norm_eps > 0:
        y = y * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + norm_eps)
    if act == ACT_SWIGLU:
        F = w.shape[0] // 2
        y = torch.nn.functional.silu(y[:, :F]) * y[:, F:]
    else:
        y = ref.apply_act(y, act)
    if residual is not None:
        y = y + residual.float()
    return y.to(x.dtype)


class ShufCache(dict):
    """Tile-ordered image of a decode weight (native ``shuffle_decode_weight``: each 16-row x 64-k
    MFMA tile 2 KiB contiguous, so every load instruction of the M <= 16 kernel reads one 1-KiB
    run), rebuilt in place when the source's data pointer or version changes (graph-safe
    address). Pays on the split-K projections (down 28.5 -> 21.9 us at M = 1)."""

    @torch.no_grad()
    def get(self, w: torch.Tensor) -> torch.Tensor:
        key = (w.data_ptr(), w._version)
        if dict.get(self, "key") != key:
            buf = dict.get(self, "w")
            if buf is None or buf.shape != w.shape or buf.device != w.device:
                buf = torch.empty_like(w, memory_format=torch.contiguous_format)
                self["w"] = buf
            native().shuffle_decode_weight(w.contiguous(), buf)
            self["key"] = key
        return self["w"]


class FoldCache(dict):
    """W diag(norm_w): the RMS-norm weight folded into the following projection for the fused
    decode path, recomputed in place when either source changes (graph-safe addresses)."""

    @torch.no_grad()
    def get(self, w: torch.Tensor, norm_w: torch.Tensor) -> torch.Tensor:
        key = (w.data_ptr(), w._version, norm_w.data_ptr(), norm_w._version)
        if dict.get(self, "key") != key:
            buf = dict.get(self, "w")
            if buf is None or buf.shape != w.shape or buf.device != w.device:
                buf = torch.empty_like(w)
                self["w"] = buf
            torch.mul(w, norm_w.to(w.dtype)[None, :], out=buf)
            self["key"] = key
        return self["w"]
