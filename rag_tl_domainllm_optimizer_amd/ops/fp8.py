"""fp8 (OCP e4m3fn) inference path for frozen weights (BASELINE config 5).

* weights: per-output-channel absmax scale, quantised once per adapter update (LoRA merged first);
* M > 64 (prefill / reference-model scoring): W8A8 — activations quantised per token, one
  MX-scaled ``mfma_f32_16x16x128_f8f6f4`` 256x256 GEMM (2x the bf16 MFMA rate), scales in the
  epilogue;
* M <= 64 (decode): W8A16 — bf16 activations, fp8 weights widened to bf16 in registers: half the
  weight bytes streamed per token, from a tile-ordered fp8 image (``Fp8Cache.shuf``): one
  workgroup per 16 weight rows (no split-K) up to M = 16, the LDS-DMA ring above.
gfx950 uses OCP e4m3fn (max 448), not the MI300 fnuz variant (cdna_hip_programming.md §3).
"""
from __future__ import annotations

from typing import Optional

import torch

from . import reference as ref
from ._ext import native, on_gpu

E4M3_MAX = 448.0


def quantize_fp8(x: torch.Tensor):
    """Per-row absmax quantisation -> (uint8 e4m3fn bits [R, C], fp32 scale [R])."""
    if on_gpu(x):
        q, s = native().quant_fp8(x.contiguous())
        return q, s
    xf = x.float()
    amax = xf.abs().amax(1)
    s = torch.where(amax > 0, amax / E4M3_MAX, torch.ones_like(amax))
    q = (xf / s[:, None]).to(torch.float8_e4m3fn).view(torch.uint8)
    return q, s


def dequantize_fp8(q: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    return q.view(torch.float8_e4m3fn).float() * s[:, None]


def gemm_fp8(x: torch.Tensor, wq: torch.Tensor, sw: torch.Tensor, bias=None, act=0, out=None) -> torch.Tensor:
    """y = act(x W^T + b) with W given as fp8 (wq, sw). W8A16 for M <= 64, W8A8 above (the
    gemm_big schedule on the MX fp8 MFMA). ``act`` 5 = SwiGLU over W = [gate; up] -> [M, N / 2]."""
    M, K = x.shape
    if on_gpu(x):
        C = native()
        if M <= 64:
            return C.gemm_fp8(x, None, wq, sw, bias, act, out)
        xq, sx = quantize_fp8(x)
        if act in (0, 5):
            return C.gemm_fp8(xq, sx, wq, sw, bias, act, out)
        # W8A8 kernels fuse bias and SwiGLU only (the decoder presets use nothing else): other
        # activations run on the bf16 GEMM output
        y = ref.apply_act(C.gemm_fp8(xq, sx, wq, sw, bias, 0, None).float(), act).to(x.dtype)
        if out is not None:
            out.copy_(y)
            return out
        return y
    xf = x.float() if M <= 64 else dequantize_fp8(*quantize_fp8(x))
    y = xf @ dequantize_fp8(wq, sw).t()
    if bias is not None:
        y = y + bias.float()
    if act == 5:  # SwiGLU pair: weight rows [gate; up]
        F = y.shape[1] // 2
        y = (torch.nn.functional.silu(y[:, :F]) * y[:, F:]).to(x.dtype)
    else:
        y = ref.apply_act(y, act).to(x.dtype)
    if out is not None:
        out.copy_(y)
        return out
    return y


def fp8_supported(w: torch.Tensor) -> bool:
    return w.dim() == 2 and w.shape[1] % 128 == 0 and w.shape[0] % 8 == 0


class Fp8Cache(dict):
    """fp8 image of one weight, refreshed in place when the source tensor changes (address or
    in-place version, e.g. a re-merged LoRA weight) so graph-captured decode steps stay valid.
    ``shuf`` adds the tile-ordered decode image (built on first use, then kept in step).
    ``train`` (config 5, ``model.fp8_train``): training forwards of the frozen base run W8A8 too,
    from ``train_cache()`` — a second image of the UNMERGED base weight, so rollouts (merged
    weights) and updates (base weights) do not re-quantise each other's image every step."""

    train = False

    def train_cache(self) -> "Fp8Cache":
        tc = getattr(self, "_train_cache", None)
        if tc is None:
            tc = Fp8Cache()
            self._train_cache = tc
        return tc

    @torch.no_grad()
    def get(self, w: torch.Tensor):
        key = (w.data_ptr(), w._version)
        if self.get_key() != key:
            q, s = quantize_fp8(w)
            if "q" in self and self["q"].shape == q.shape and self["q"].device == q.device:
                self["q"].copy_(q)
                self["s"].copy_(s)
            else:
                self["q"], self["s"] = q, s
            self["key"] = key
            if "qs" in self:
                self._shuffle()
        return self["q"], self["s"]

    def _shuffle(self):
        q = self["q"]
        qs = dict.get(self, "qs")
        if qs is None or qs.shape != q.shape or qs.device != q.device:
            qs = torch.empty_like(q)
            self["qs"] = qs
        native().shuffle_decode_weight_fp8(q, qs)

    @torch.no_grad()
    def shuf(self, w: torch.Tensor):
        """(tile-ordered fp8 image, scales) for the M <= 16 W8A16 kernel."""
        self.get(w)
        if "qs" not in self:
            self._shuffle()
        return self["qs"], self["s"]

    @staticmethod
    def shuf_ok(w: torch.Tensor, m: int, act: int = 0) -> bool:
        """The tile-ordered fp8 image serves every W8A16 decode GEMM (M <= 64) of these shapes."""
        return m <= 64 and w.shape[1] % 128 == 0 and w.shape[0] % (64 if act == 5 else 16) == 0

    def get_key(self):
        return dict.get(self, "key")
