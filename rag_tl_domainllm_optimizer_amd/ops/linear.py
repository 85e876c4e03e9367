"""Linear projections: frozen/trainable base weight + fused LoRA adapters + bias/activation.

GPU forward is one MFMA GEMM in which the LoRA term rides on the same accumulators as extra
K-steps:  ``Y = act(X W^T + U UB^T + b)`` with ``U = X A_pad^T`` (A_pad = scaling * A, zero-padded
to a multiple of 64 rows) computed by a small GEMM first. Several adapters on one fused projection
(q|k|v, gate|up) share one padded rank dimension, with UB block-diagonal.

Extended-weight layout (``LoRAGroup.attach_ext``): a frozen base weight that carries adapters is
stored ONCE as ``ext = [W | UB]`` ([N, K + Rp], the parameter becomes the strided view
``ext[:, :K]`` and ``UB`` the view ``ext[:, K:]``), so the token-parallel (M > 64) LoRA forward is
ONE plain GEMM ``[X | U] @ ext^T`` on hipBLASLt — measured 1.2-1.5 PF/s on the PPO-update shapes
against 0.7-1.05 PF/s for the hand-written fused kernel (tools/update_gemm_probe.py,
profiles/update_gemm_probe.log). Decode / skinny shapes keep the hand-written kernels.

Backward (training): dX = dY W + dU A_pad, dA = s dU^T X, dB = dY^T U, dW = dY^T X (full FT) are
plain library GEMMs (torch.matmul -> hipBLASLt); only the forward carries fused epilogues.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import List, Optional

import torch

from . import reference as ref
from ._ext import native, on_gpu

ACT_IDS = {None: 0, "none": 0, "relu": 1, "gelu": 2, "gelu_tanh": 3, "gelu_new": 3, "silu": 4, "swiglu": 5}
ACT_SWIGLU = 5  # w = [gate; up] (2F rows) -> silu(x gate^T) * (x up^T), [.., F]


# Plain GEMMs (no LoRA K-extension, bias or activation epilogue, bf16 out) pick a backend by M:
#   M <= 16      SKINNY_BACKEND, default "native": split-K MFMA weight-streaming kernel, measured
#                faster than hipBLASLt on cold (HBM-streamed) decode weights at batch 1-8
#                (profiles/kernels_skinny_cold.log: qkv 16.5 vs 19.5 us, o 11.4 vs 19.0 us,
#                gate_up 46.9 vs 56.0 us, lm_head 47.8 vs 57.4 us)
#   16 < M <= 64 MID_BACKEND, default "auto": the LDS-DMA ring kernel for deep weights (K >= 8192:
#                down 36.6 vs 39.8 us), hipBLASLt for the rest (qkv 18 vs 26, o 15 vs 21, gate_up
#                49-52 vs 58, lm_head 54-58 vs 58 us) — hipGraph replay over distinct weights at
#                M = 64, profiles/kernels_decode_split_sweep.log
#   M > 64       PLAIN_BACKEND, default "lib" (hipBLASLt ~1.5 PF/s vs ~1.2 PF/s for the 256x256
#                8-phase kernel on plain GEMMs)
# Everything with a fused epilogue or a LoRA term always runs on the hand-written kernels.
PLAIN_BACKEND = os.environ.get("RAGTL_PLAIN_GEMM", "lib")
MID_BACKEND = os.environ.get("RAGTL_MID_GEMM", "auto")
SKINNY_BACKEND = os.environ.get("RAGTL_SKINNY", "native")


def set_gemm_backend(plain: Optional[str] = None, skinny: Optional[str] = None, mid: Optional[str] = None):
    """Select "lib" (hipBLASLt) or "native" (hand-written kernels) for plain GEMMs by M range;
    returns the previous (plain, skinny, mid) triple."""
    global PLAIN_BACKEND, SKINNY_BACKEND, MID_BACKEND
    prev = (PLAIN_BACKEND, SKINNY_BACKEND, MID_BACKEND)
    for name, val in (("PLAIN_BACKEND", plain), ("SKINNY_BACKEND", skinny), ("MID_BACKEND", mid)):
        if val is not None:
            assert val in ("lib", "native", "auto")
            globals()[name] = val
    return prev


def gemm(x: torch.Tensor, w: torch.Tensor, u=None, ub=None, bias=None, act=0, out_f32=False, out=None):
    """Raw (non-autograd) fused GEMM on 2-D row-major operands."""
    if on_gpu(x):
        if u is None and bias is None and act == 0 and not out_f32:
            M = x.shape[0]
            backend = SKINNY_BACKEND if M <= 16 else (MID_BACKEND if M <= 64 else PLAIN_BACKEND)
            if backend == "auto":
                backend = "native" if w.shape[1] >= 8192 else "lib"
            # the hand-written kernels store 8-column vectors: an output width that is not a multiple
            # of 8 (e.g. OpenChat's 32002-token vocabulary) takes the library GEMM
            if backend == "lib" or w.shape[0] % 8:
                return torch.matmul(x, w.t(), out=out)
        return native().gemm(x, w, u, ub, bias, act, out_f32, out)
    y = ref.gemm(x, w, u, ub, bias, act, out_f32)
    if out is not None:
        out.copy_(y)
        return out
    return y


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
    # [W | UB] storage of the base weight (attach_ext); None = W stored on its own
    ext: Optional[torch.Tensor] = None

    @property
    def rank_total(self) -> int:
        return sum(int(a.shape[0]) for a in self.a)

    @property
    def rp(self) -> int:
        return max(64, (self.rank_total + 63) // 64 * 64)

    @torch.no_grad()
    def attach_ext(self, w: torch.nn.Parameter) -> bool:
        """Re-home the base weight ``w`` [N, K] into ``ext = [W | UB]`` (one copy, then W's old
        storage is released); ``w.data`` becomes the strided view ``ext[:, :K]``. GPU bf16 only."""
        if not (w.is_cuda and w.dtype == torch.bfloat16 and w.dim() == 2 and w.shape[0] == self.n_out):
            return False
        N, K = w.shape
        rp = self.rp
        # deep K (down_proj, K = 14336): pad so K + Rp is a multiple of 256 — hipBLASLt runs K = 14400
        # 1.65x slower than K = 14336 or 14592 (profiles/lora_fwd_probe.log); shallow K keeps Rp = 64
        # (K = 4160 is within 0-6 % of the adapter-free GEMM)
        rp_ext = rp if K < 8192 or K % 256 else (rp + 255) // 256 * 256
        if self.ext is not None and self.ext.shape == (N, K + rp_ext) and self.ext_linked(w):
            return True
        ext = torch.empty(N, K + rp_ext, dtype=w.dtype, device=w.device)
        ext[:, :K].copy_(w.data)
        ext[:, K:].zero_()
        w.data = ext[:, :K]
        self.ext = ext
        self.a_pad = None  # rebuilt by refresh() with ub as a view of ext
        self.refresh(dtype=w.dtype)
        return True

    def ext_linked(self, w: torch.Tensor) -> bool:
        """True if ``w`` still is the W-view of ``ext`` (something may have replaced w.data)."""
        e = self.ext
        return (e is not None and w.data_ptr() == e.data_ptr() and w.shape[0] == e.shape[0]
                and w.stride(0) == e.stride(0) and w.device == e.device)

    @torch.no_grad()
    def refresh(self, dtype=torch.bfloat16):
        """Rebuild the padded bf16 images from the fp32 parameters (after each optimizer step)."""
        K = self.a[0].shape[1]
        dev = self.a[0].device
        rp = self.rp
        if self.a_pad is None or self.a_pad.shape != (rp, K) or self.a_pad.device != dev:
            self.a_pad = torch.zeros(rp, K, dtype=dtype, device=dev)
            if self.ext is not None and self.ext.device == dev and self.ext.shape[1] - K >= rp:
                self.ub = self.ext[:, K:K + rp]
                self.ext[:, K:].zero_()
            else:
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
        """W + UB A_pad (fp32 accumulate, one bf16 rounding), updated IN PLACE so captured graphs
        that read it stay valid across adapter updates. On the GPU: copy W, then one bf16 GEMM with
        beta = 1 (4 B of traffic per weight element instead of the 20 B of an fp32 round trip)."""
        if self.merged is None or self.merged.shape != w.shape or self.merged.device != w.device:
            self.merged = torch.empty(w.shape, dtype=w.dtype, device=w.device)
            self.merged_dirty = True
        if self.merged_dirty:
            if on_gpu(w) and w.dtype == torch.bfloat16:
                self.merged.copy_(w)
                self.merged.addmm_(self.ub, self.a_pad)
            else:
                for r0 in range(0, w.shape[0], rows_per_chunk):
                    r1 = min(w.shape[0], r0 + rows_per_chunk)
                    self.merged[r0:r1].copy_(torch.addmm(w[r0:r1].float(), self.ub[r0:r1].float(),
                                                         self.a_pad.float()))
            self.merged_dirty = False
        return self.merged


def _mm_tn_f32(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a^T @ b in fp32 for the LoRA weight gradients: a [M, P], b [M, Q] with M = tokens (thousands)
    and a small output (P or Q = the padded rank). As one GEMM the library tiles only the small
    output (64-128 workgroups for [64, 4096]: a quarter of the chip); split over M into a batched
    GEMM of ~512 tiles and summed (the [c, P, Q] partials are a few MB)."""
    if not (a.is_cuda and a.dtype in (torch.bfloat16, torch.float16) and b.dtype == a.dtype):
        return a.float().t() @ b.float()
    M, P = a.shape
    Q = b.shape[1]
    tiles = max(1, ((P + 63) // 64) * ((Q + 63) // 64))
    c = 1
    while c * tiles < 512 and M % (2 * c) == 0 and M // (2 * c) >= 256:
        c *= 2
    if c == 1:
        return torch.mm(a.t(), b, out_dtype=torch.float32)
    part = torch.bmm(a.view(c, M // c, P).transpose(1, 2), b.view(c, M // c, Q), out_dtype=torch.float32)
    return part.sum(0)


def _mm_splitk(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a @ b for the LoRA rank-sized products (a [M, K] tokens x features, b [K, Rp], a view is fine):
    a deep reduction (K up to 28672) into a narrow [M, Rp] output, which one library GEMM tiles into
    only M/64 workgroups. Split K into a batched GEMM of ~512 tiles (fp32 partials [c, M, Rp], a
    few MB, summed). Used for U = X A^T (forward) and dU = dY UB (backward)."""
    M, K = a.shape
    N = b.shape[1]
    if not (a.is_cuda and a.dtype in (torch.bfloat16, torch.float16) and b.dtype == a.dtype):
        return a @ b
    tiles = max(1, ((M + 63) // 64) * ((N + 63) // 64))
    c = 1
    while c * tiles < 512 and K % (2 * c) == 0 and K // (2 * c) >= 512:
        c *= 2
    if c == 1:
        return a @ b
    Kc = K // c
    part = torch.bmm(a.unflatten(1, (c, Kc)).transpose(0, 1), b.unflatten(0, (c, Kc)), out_dtype=torch.float32)
    return part.sum(0).to(a.dtype)


EXT_MIN_M = 65  # token-parallel shapes take the [X | U] @ [W | UB]^T library GEMM


def _use_ext(x2, w, bias, act, lora) -> bool:
    return (lora is not None and lora.ext is not None and bias is None and act == 0 and on_gpu(x2)
            and x2.shape[0] >= EXT_MIN_M and lora.ext_linked(w))


def _ext_forward(x2: torch.Tensor, lora: LoRAGroup):
    """y = [X | U] @ ext^T with U = X A_pad^T written next to X: returns (y, x view, u view)."""
    M, K = x2.shape
    rp = lora.a_pad.shape[0]
    xe = torch.empty(M, lora.ext.shape[1], dtype=x2.dtype, device=x2.device)
    xv, uv = xe[:, :K], xe[:, K:K + rp]
    if xe.shape[1] > K + rp:
        xe[:, K + rp:].zero_()
    xv.copy_(x2)
    uv.copy_(_mm_splitk(x2, lora.a_pad.t()))
    return torch.matmul(xe, lora.ext.t()), xv, uv


def _mm_nn_deep(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a [M, K] @ b [K, N] for a deep reduction into a narrow output (dX of gate_up: K = 28672 into
    N = 4096): one GEMM tiles only ceil(M/256) x 16 = 304 tiles at M = 4800 (1.2 waves on 256 CUs);
    split K four ways into a batched GEMM with fp32 partials, summed: 1448 -> 1116 us at M = 4800,
    1758 -> 1432 us at M = 7168 (profiles/splitk_probe.log). Shallow reductions lose with the split
    (dX of qkv / o), so only K >= 16384 takes it."""
    M, K = a.shape
    N = b.shape[1]
    tiles = ((M + 255) // 256) * ((N + 255) // 256)
    if not (a.is_cuda and a.dtype == torch.bfloat16 and K >= 16384 and K % 4 == 0 and tiles < 1024
            and b.stride(1) == 1):
        return a @ b
    c = 4
    kc = K // c
    part = torch.bmm(a.unflatten(1, (c, kc)).transpose(0, 1), b.unflatten(0, (c, kc)), out_dtype=torch.float32)
    return part.sum(0).to(a.dtype)


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x2, w, bias, act, lora: Optional[LoRAGroup], *lora_params):
        u = ub = None
        if _use_ext(x2, w, bias, act, lora):
            y, x2, u = _ext_forward(x2, lora)
        else:
            if lora is not None:
                u = _mm_splitk(x2, lora.a_pad.t()) if x2.shape[0] > 64 else gemm(x2, lora.a_pad)  # [M, Rp] = X (sA)^T
                ub = lora.ub
            y = gemm(x2, w, u, ub, bias, act)
        ctx.act = act
        ctx.lora = lora
        ctx.has_bias = bias is not None
        # with an activation epilogue the pre-activation is recomputed in backward (no extra
        # activation-sized tensor is kept alive)
        ctx.save_for_backward(x2, w, u if u is not None else torch.empty(0), bias if bias is not None else torch.empty(0))
        return y

    @staticmethod
    def backward(ctx, dy):
        x2, w, u, bias = ctx.saved_tensors
        lora = ctx.lora
        dy = dy.contiguous()
        if ctx.act != 0:
            # recompute pre-activation and apply the activation derivative
            ub = lora.ub if lora is not None else None
            pre = gemm(x2, w, u if lora is not None else None, ub, bias if ctx.has_bias else None, 0, out_f32=True)
            with torch.enable_grad():
                p = pre.detach().requires_grad_(True)
                yact = ref.apply_act(p, ctx.act)
                (g,) = torch.autograd.grad(yact, p, dy.float())
            dy = g.to(dy.dtype)
        needs = ctx.needs_input_grad
        dx = dw = db = None
        du = _mm_splitk(dy, lora.ub) if lora is not None else None  # [M, Rp] (= dL/dU)
        if needs[0]:
            dx = _mm_nn_deep(dy, w) if on_gpu(dy) else dy @ w
            if lora is not None:
                # dX += dU A_pad as a separate K = Rp pass: measured cheaper than seeding dX with it and
                # letting the big GEMM accumulate (beta = 1 slowed the big GEMM by more)
                dx.addmm_(du, lora.a_pad)
        if needs[1]:
            dw = (dy.t() @ x2).to(w.dtype)
        if ctx.has_bias and needs[2]:
            db = dy.float().sum(0).to(bias.dtype)
        lora_grads = []
        if lora is not None:
            # all adapters of the projection in two GEMMs with fp32 output (bf16 in, fp32 accumulate):
            # dA_all = dU^T X [Rp, K]; dB_all = dY^T U [N, Rp] (adapter i uses its diagonal block)
            ga_all = _mm_tn_f32(du, x2)
            gb_all = _mm_tn_f32(dy, u)
            for a, b, r0, c0, s in zip(lora.a, lora.b, lora.r0, lora.col0, lora.scale):
                ri, ni = a.shape[0], b.shape[0]
                lora_grads.append((ga_all[r0:r0 + ri] * s).to(a.dtype))
                lora_grads.append(gb_all[c0:c0 + ni, r0:r0 + ri].to(b.dtype))
            # parameter order in forward(*lora_params) is a0, b0, a1, b1, ...
        return (dx, dw, db, None, None, *lora_grads)


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
    if act_id == ACT_SWIGLU:
        # fused into the skinny gate/up GEMM when it can run there (no-grad decode on the GPU)
        if (on_gpu(x2) and not torch.is_grad_enabled() and x2.shape[0] <= 64 and bias is None
                and w.shape[0] % 64 == 0 and x2.shape[1] % 64 == 0):
            w_eff = lora.merged_weight(w) if use_lora else w
            if fp8 is not None:
                from .fp8 import fp8_supported

                if fp8_supported(w_eff):
                    q, sc = fp8.get(w_eff)
                    y = native().gemm_fp8(x2, None, q, sc, None, ACT_SWIGLU, None)
                    return y.reshape(*shp[:-1], w.shape[0] // 2)
            y = native().gemm(x2, w_eff, None, None, None, ACT_SWIGLU, False, None)
            return y.reshape(*shp[:-1], w.shape[0] // 2)
        from .misc import swiglu

        return swiglu(linear(x, w, bias, None, lora, fp8))
    if fp8 is not None and not torch.is_grad_enabled():
        from .fp8 import fp8_supported, gemm_fp8

        w_eff = lora.merged_weight(w) if use_lora else w
        if fp8_supported(w_eff) and (x2.shape[0] > 64 or x2.shape[1] % 64 == 0):
            q, s = fp8.get(w_eff)
            y = gemm_fp8(x2, q, s, bias, act_id)
            return y.reshape(*shp[:-1], w.shape[0])
    if use_lora and lora.use_merged and not torch.is_grad_enabled():
        y = gemm(x2, lora.merged_weight(w), None, None, bias, act_id)
        return y.reshape(*shp[:-1], w.shape[0])
    grad_needed = torch.is_grad_enabled() and (
        x2.requires_grad or w.requires_grad or (bias is not None and bias.requires_grad)
        or (use_lora and any(p.requires_grad for p in lora.a + lora.b)))
    if not grad_needed:
        if use_lora and _use_ext(x2, w, bias, act_id, lora):
            y = _ext_forward(x2, lora)[0]
            return y.reshape(*shp[:-1], w.shape[0])
        u = None
        if use_lora:
            u = _mm_splitk(x2, lora.a_pad.t()) if x2.shape[0] > 64 else gemm(x2, lora.a_pad)
        y = gemm(x2, w, u, lora.ub if use_lora else None, bias, act_id)
    else:
        params = []
        if use_lora:
            for a, b in zip(lora.a, lora.b):
                params += [a, b]
        y = _LinearFn.apply(x2, w, bias, act_id, lora if use_lora else None, *params)
    return y.reshape(*shp[:-1], w.shape[0])


def gemm_decode(x: torch.Tensor, w: torch.Tensor, act: int = 0, residual=None, norm_eps: float = 0.0, fp8=None):
    """Decode-step GEMM (M <= 64) with the fused prologue/epilogue of the skinny kernels:
    ``C = act(rstd(x) * x w^T) + residual`` where ``rstd`` (``norm_eps > 0``) is the RMS-norm of
    each input row computed inside the GEMM (the norm weight must already be folded into ``w``)
    and ``act`` may be ACT_SWIGLU (w = [gate; up]). ``fp8`` (Fp8Cache) streams e4m3fn weights."""
    if on_gpu(x):
        x = x.contiguous()
        if fp8 is not None:
            from .fp8 import fp8_supported

            if fp8_supported(w):
                q, sc = fp8.get(w)
                return native().gemm_fp8(x, None, q, sc, None, act, None, residual, norm_eps)
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
