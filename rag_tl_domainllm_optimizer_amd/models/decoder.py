"""Causal decoder LMs: Llama-2 / Mistral (RMSNorm, RoPE, GQA, SwiGLU, sliding window) and OPT
(pre-LN, learned positions, biases, ReLU MLP, tied head), in one module with three entry points:

* ``forward``  — full-sequence forward (training / scoring), flash attention, autograd-ready,
  LoRA adapters fused into the projection GEMMs;
* ``prefill``  — prompt forward that also appends K/V to a static cache;
* ``decode``   — one token per sequence against the cache (graph-capturable: no host sync, no
  allocation-dependent control flow).

Parameters use a fused layout (``qkv_proj`` = q|k|v rows, ``gate_up_proj`` = gate|up rows) so each
sub-layer is one GEMM; :mod:`.io` maps to/from the HF per-projection names. The reference loads
the same architectures through ``AutoModelForCausalLM`` (reinforcement_learning_optimization_after_rag.py:23,140,171).
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn as nn

from .. import ops
from ..ops import reference as ref
from .config import ModelConfig

LLAMA_LORA_TARGETS = ("q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj", "down_proj")
OPT_LORA_TARGETS = ("q_proj", "k_proj", "v_proj", "out_proj", "fc1", "fc2")


class DecoderLayer(nn.Module):
    def __init__(self, cfg: ModelConfig, device=None, dtype=torch.bfloat16):
        super().__init__()
        H, F = cfg.hidden_size, cfg.intermediate_size
        kw = dict(device=device, dtype=dtype)
        self.cfg = cfg
        self.ln1_w = nn.Parameter(torch.ones(H, **kw))
        self.ln2_w = nn.Parameter(torch.ones(H, **kw))
        self.qkv_w = nn.Parameter(torch.empty(cfg.qkv_dim, H, **kw))
        self.o_w = nn.Parameter(torch.empty(H, cfg.num_heads * cfg.head_dim, **kw))
        if cfg.arch == "opt":
            self.ln1_b = nn.Parameter(torch.zeros(H, **kw))
            self.ln2_b = nn.Parameter(torch.zeros(H, **kw))
            self.qkv_b = nn.Parameter(torch.zeros(cfg.qkv_dim, **kw))
            self.o_b = nn.Parameter(torch.zeros(H, **kw))
            self.fc1_w = nn.Parameter(torch.empty(F, H, **kw))
            self.fc1_b = nn.Parameter(torch.zeros(F, **kw))
            self.fc2_w = nn.Parameter(torch.empty(H, F, **kw))
            self.fc2_b = nn.Parameter(torch.zeros(H, **kw))
        else:
            self.gate_up_w = nn.Parameter(torch.empty(2 * F, H, **kw))
            self.down_w = nn.Parameter(torch.empty(H, F, **kw))
        # LoRA: projection name -> LoRAGroup ; parameters registered in lora_params for state tracking
        self.lora: Dict[str, ops.LoRAGroup] = {}
        self.lora_params = nn.ParameterDict()
        self.lora_enabled = True
        # fp8 inference images of the projection weights (CausalLM.set_fp8)
        self.fp8_enabled = False
        self.fp8_train = False  # W8A8 frozen-base product in LoRA training forwards (config 5)
        self._fp8: Dict[str, ops.Fp8Cache] = {}
        # norm-folded weights of the fused decode path (Llama/Mistral)
        self._fold: Dict[str, ops.FoldCache] = {}
        # tile-ordered images of the split-K decode projections (qkv, o, down) for batch <= 16
        self._shufc: Dict[str, ops.ShufCache] = {}

    # ---------------------------------------------------------------- helpers
    def _lg(self, name):
        g = self.lora.get(name)
        return g if (g is not None and self.lora_enabled) else None

    def _b(self, name):
        return getattr(self, name, None)

    def _f8(self, name):
        if not self.fp8_enabled:
            return None
        c = self._fp8.setdefault(name, ops.Fp8Cache())
        c.train = self.fp8_train  # config 5: W8A8 training forwards of the frozen base too
        return c

    def _dec_caches(self, f8name: str, shufname: str, w: torch.Tensor, m: int):
        """(Fp8Cache, ShufCache) for one decode projection at batch ``m``: the fp8 image except
        where the bf16 GEMV is faster — 2 <= m <= 16 on projections of <= 2^24 weights (Mistral
        o_proj), where the fp8 16-row GEMV reads twice its weight bytes of activations per row
        group (profiles/r3/fp8_decode_table_v6.log: o 8.1-8.8 us bf16 vs 10.1-10.9 us fp8)."""
        if self.fp8_enabled and not (2 <= m <= 16 and w.numel() <= (1 << 24)):
            return self._f8(f8name), None
        if not shuffle_enabled(m):
            return None, None
        return None, self._shufc.setdefault(shufname, ops.ShufCache())

    # ---------------------------------------------------------------- fused decode step (M <= 64)
    def _w_eff(self, wname: str, gname: str):
        w = getattr(self, wname)
        g = self._lg(gname)
        if g is None:
            return w
        if g.a_pad is None or g.a_pad.device != w.device:
            g.refresh(dtype=w.dtype)
        return g.merged_weight(w)

    @torch.no_grad()
    def refresh_decode_weights(self):
        """Bring the merged / folded / fp8 decode weights up to date eagerly (graph replays of a
        captured decode step only read them)."""
        if self.cfg.arch == "opt":
            return
        wq = self._fold.setdefault("qkv", ops.FoldCache()).get(self._w_eff("qkv_w", "qkv"), self.ln1_w)
        wgu = self._fold.setdefault("gate_up", ops.FoldCache()).get(self._w_eff("gate_up_w", "gate_up"), self.ln2_w)
        wo, wd = self._w_eff("o_w", "o"), self._w_eff("down_w", "down")
        for name, w in (("qkv_folded", wq), ("gate_up_folded", wgu), ("o", wo), ("down", wd)):
            c = self._f8(name)
            if c is not None:
                c.get(w)
        for name, w in (("qkv", wq), ("o", wo), ("gate_up", wgu), ("down", wd)):
            if name in self._shufc:  # images exist once a batch <= 16 decode ran
                self._shufc[name].get(w)

    def decode_fused(self, h, attend):
        """One Llama/Mistral layer of a decode step in four kernels: [RMSNorm folded into the qkv
        GEMM] -> attention (RoPE + append + split-K) -> [o GEMM + residual] -> [RMSNorm folded into
        the gate/up GEMM + SwiGLU] -> [down GEMM + residual]. ``h`` is the bf16 residual stream."""
        cfg = self.cfg
        eps = cfg.norm_eps
        m = h.shape[0]
        wq = self._fold.setdefault("qkv", ops.FoldCache()).get(self._w_eff("qkv_w", "qkv"), self.ln1_w)
        f8, sh = self._dec_caches("qkv_folded", "qkv", wq, m)
        qkv = ops.gemm_decode(h, wq, norm_eps=eps, fp8=f8, shuf=sh)
        wo = self._w_eff("o_w", "o")
        f8, sh = self._dec_caches("o", "o", wo, m)
        h = ops.gemm_decode(attend(qkv), wo, residual=h, fp8=f8, shuf=sh)
        wgu = self._fold.setdefault("gate_up", ops.FoldCache()).get(self._w_eff("gate_up_w", "gate_up"), self.ln2_w)
        f8, sh = self._dec_caches("gate_up_folded", "gate_up", wgu, m)
        f = ops.gemm_decode(h, wgu, act=ops.ACT_SWIGLU, norm_eps=eps, fp8=f8, shuf=sh)
        wd = self._w_eff("down_w", "down")
        f8, sh = self._dec_caches("down", "down", wd, m)
        return ops.gemm_decode(f, wd, residual=h, fp8=f8, shuf=sh)

    def attn_in(self, x, residual, defer: bool = False):
        """``defer`` (no-grad decode, batch > 64): the qkv GEMM may return unreduced split-K
        partials (ops.SplitK) for the attention kernel to sum; ``x`` may itself be the previous
        layer's unreduced down projection (summed inside the norm)."""
        cfg = self.cfg
        if cfg.arch == "opt":
            h, residual = ops.layer_norm(x, self.ln1_w, self.ln1_b, cfg.norm_eps, residual)
        else:
            h, residual = ops.rms_norm(x, self.ln1_w, cfg.norm_eps, residual)
        lin = ops.linear_deferred if (defer and cfg.arch != "opt") else ops.linear
        qkv = lin(h, self.qkv_w, self._b("qkv_b"), lora=self._lg("qkv"), fp8=self._f8("qkv"))
        return qkv, residual

    def attn_in_rope(self, x, residual, rope):
        """Token-parallel forms (training / reference forwards, prefill): the qkv projection with the
        rotary embedding in its GEMM epilogue where that applies (``ops.linear_rope``; ``rope`` =
        (pos per row, cos, sin)). Returns (qkv, residual, rotated)."""
        cfg = self.cfg
        if rope is None or cfg.arch == "opt":
            qkv, residual = self.attn_in(x, residual)
            return qkv, residual, False
        h, residual = ops.rms_norm(x, self.ln1_w, cfg.norm_eps, residual)
        D = cfg.head_dim
        qkv, rotated = ops.linear_rope(h, self.qkv_w, self._b("qkv_b"), lora=self._lg("qkv"), fp8=self._f8("qkv"),
                                       rope=(rope[0], rope[1], rope[2], (cfg.num_heads + cfg.num_kv_heads) * D, D))
        return qkv, residual, rotated

    def mlp(self, a, residual, defer: bool = False):
        cfg = self.cfg
        defer = defer and cfg.arch != "opt"
        lin = ops.linear_deferred if defer else ops.linear
        a = lin(a, self.o_w, self._b("o_b"), lora=self._lg("o"), fp8=self._f8("o"))
        if cfg.arch == "opt":
            h, residual = ops.layer_norm(a, self.ln2_w, self.ln2_b, cfg.norm_eps, residual)
            f = ops.linear(h, self.fc1_w, self.fc1_b, act=cfg.hidden_act, lora=self._lg("fc1"), fp8=self._f8("fc1"))
            d = ops.linear(f, self.fc2_w, self.fc2_b, lora=self._lg("fc2"), fp8=self._f8("fc2"))
        else:
            h, residual = ops.rms_norm(a, self.ln2_w, cfg.norm_eps, residual)
            d = None
            if not (self.fp8_enabled and self.fp8_train):
                # training: one autograd node whose backward runs the SwiGLU backward inside the
                # down projection's dX GEMM (ops.swiglu_mlp; None when it does not apply)
                d = ops.swiglu_mlp(h, self.gate_up_w, self.down_w, self._lg("gate_up"), self._lg("down"))
            if d is None:
                # act="swiglu": one fused skinny GEMM in no-grad decode, GEMM + SwiGLU kernel otherwise
                f = ops.linear(h, self.gate_up_w, act="swiglu", lora=self._lg("gate_up"), fp8=self._f8("gate_up"))
                d = lin(f, self.down_w, lora=self._lg("down"), fp8=self._f8("down"))
        return d, residual


class CausalLM(nn.Module):
    def __init__(self, cfg: ModelConfig, device=None, dtype=torch.bfloat16, init: bool = True, seed: int = 0):
        super().__init__()
        assert cfg.is_decoder, cfg.arch
        self.cfg = cfg
        self.dtype = dtype
        kw = dict(device=device, dtype=dtype)
        self.embed = nn.Parameter(torch.empty(cfg.vocab_size, cfg.hidden_size, **kw))
        if cfg.arch == "opt":
            self.pos_embed = nn.Parameter(torch.empty(cfg.max_position + cfg.position_offset, cfg.hidden_size, **kw))
            self.norm_b = nn.Parameter(torch.zeros(cfg.hidden_size, **kw))
        self.norm_w = nn.Parameter(torch.ones(cfg.hidden_size, **kw))
        self.layers = nn.ModuleList([DecoderLayer(cfg, device, dtype) for _ in range(cfg.num_layers)])
        if not cfg.tie_embeddings:
            self.lm_head = nn.Parameter(torch.empty(cfg.vocab_size, cfg.hidden_size, **kw))
        self._rope = None
        self._head_shuf = None  # ShufCache of the LM head for decode at batch <= 16
        # decode steps run the fused 4-GEMM layer (norms folded into GEMMs, residual epilogues) up to
        # this batch: bf16 on the no-split tile-ordered GEMVs (M <= 16), then (17..64, serving) on
        # the 256-row wide kernel / 64-column LDS-DMA ring with the in-GEMM RMS norm — 3 % faster
        # decode steps than separate norm kernels (profiles/r6/decode_fused_max_ab.log); above it the
        # bf16 decode layer uses the token-parallel 256x128 split-K GEMMs with the split-K partials
        # summed inside the norm and attention-prologue kernels (``defer_splitk``). With fp8 weights
        # (config 5) the same up to batch 64: W8A16 tile-ordered GEMVs to 16 rows, then the fp8
        # LDS-DMA kernels with the same folded-norm / SwiGLU / residual epilogues
        self.fused_decode = True
        self.fused_decode_max_batch = 64
        self.fused_decode_max_batch_fp8 = 64
        # decode at batch > 64: leave split-K partials for the consumer kernels to sum
        self.defer_splitk = True
        # fp8 (e4m3fn) K/V cache for generators built on this model (config 5, ``model.fp8_kv``)
        self.kv_fp8 = False
        if init:
            self.reset_parameters(seed)

    # ------------------------------------------------------------------ init
    @torch.no_grad()
    def reset_parameters(self, seed: int = 0):
        """Random init (HF-style normal(0, initializer_range)); seeded -> identical on every DP rank."""
        g = torch.Generator(device="cpu").manual_seed(seed)
        std = self.cfg.initializer_range
        for name, p in self.named_parameters():
            if "lora" in name:
                continue
            if name.endswith("_w") and ("ln" in name or "norm" in name):
                p.fill_(1.0)
            elif name.endswith("_b") or name == "norm_b":
                p.zero_()
            else:
                _normal_(p, std, g)

    # ------------------------------------------------------------------ utils
    @property
    def head_weight(self):
        return self.embed if self.cfg.tie_embeddings else self.lm_head

    def rope(self, device):
        if self.cfg.arch == "opt":
            return None, None
        if self._rope is None or self._rope[0].device != torch.device(device):
            self._rope = ref.rope_tables(self.cfg.head_dim, self.cfg.max_position, self.cfg.rope_theta, device)
        return self._rope

    def positions(self, B, S, kv_start, device):
        ar = torch.arange(S, device=device)[None, :].expand(B, S)
        if kv_start is not None:
            ar = (ar - kv_start.long()[:, None]).clamp(min=0)
        return ar.reshape(-1).to(torch.int32)

    def embed_tokens(self, ids_flat, pos_flat):
        if self.cfg.arch == "opt":
            return ops.embedding(self.embed, ids_flat, self.pos_embed, pos_flat.long() + self.cfg.position_offset)
        return ops.embedding(self.embed, ids_flat)

    def final_norm(self, d, residual):
        cfg = self.cfg
        if cfg.arch == "opt":
            return ops.layer_norm(d, self.norm_w, self.norm_b, cfg.norm_eps, residual)[0]
        return ops.rms_norm(d, self.norm_w, cfg.norm_eps, residual)[0]

    def logits(self, hidden, out_f32: bool = False):
        if torch.is_grad_enabled() and hidden.requires_grad:
            return ops.linear(hidden, self.head_weight)
        hw = self.head_weight
        if ops.on_gpu(hidden) and shuffle_enabled(hidden.shape[0]) and hw.shape[0] % 16 == 0 and hw.is_contiguous():
            # decode at batch <= 16: the tile-ordered image of the LM head (split 8: 52 -> 48 us)
            if self._head_shuf is None:
                self._head_shuf = ops.ShufCache()
            return ops.native().gemm(hidden.contiguous(), self._head_shuf.get(hw), None, None, None, 0, out_f32,
                                     None, None, 0.0, True)
        return ops.gemm(hidden.contiguous(), hw, out_f32=out_f32)

    # ------------------------------------------------------------------ full forward
    def forward(self, input_ids: torch.Tensor, kv_start: Optional[torch.Tensor] = None,
                gradient_checkpointing: bool = False, packed_idx: Optional[torch.Tensor] = None,
                out_rows: Optional[torch.Tensor] = None) -> torch.Tensor:
        """input_ids [B, S] (left-padded; kv_start[b] = first real token) -> final hidden [B*S, H].

        ``packed_idx`` [N] (grid positions b*S + s of the tokens to compute, see ``packed_index``):
        varlen form — embeddings, norms and every projection GEMM run on the N real tokens only
        (attention scatters them into the [B, S] grid it tiles); returns [N, H] in that order.

        ``out_rows`` [R] (int64 rows of that [B*S] / [N] order): only these rows' hidden states are
        wanted (the scored positions). The last layer's K/V still cover every row, but its o_proj,
        MLP and the final norm run on the R rows only; returns [R, H]."""
        cfg = self.cfg
        B, S = input_ids.shape
        dev = input_ids.device
        pos = self.positions(B, S, kv_start, dev)
        cos, sin = self.rope(dev)
        ks = kv_start.to(torch.int32) if kv_start is not None else None
        packed_inv = None
        if packed_idx is not None:
            x = self.embed_tokens(input_ids.reshape(-1).index_select(0, packed_idx), pos.index_select(0, packed_idx))
            packed_inv = ops.packed_inverse(packed_idx, B * S)
        else:
            x = self.embed_tokens(input_ids.reshape(-1), pos)
        residual = None
        nl = len(self.layers)
        for li, layer in enumerate(self.layers):
            rows = out_rows if li == nl - 1 else None
            if gradient_checkpointing and torch.is_grad_enabled():
                x, residual = torch.utils.checkpoint.checkpoint(self._layer_fwd, layer, x, residual, pos, cos, sin,
                                                                B, S, ks, packed_idx, packed_inv, rows,
                                                                use_reentrant=False)
            else:
                x, residual = self._layer_fwd(layer, x, residual, pos, cos, sin, B, S, ks, packed_idx, packed_inv, rows)
        return self.final_norm(x, residual)

    def _layer_fwd(self, layer, x, residual, pos, cos, sin, B, S, ks, packed_idx=None, packed_inv=None,
                   out_rows=None):
        cfg = self.cfg
        rope = (pos, cos, sin) if cos is not None else None
        # the projection rotates its own rows: packed rows carry their own positions
        rows_pos = pos.index_select(0, packed_idx) if (packed_idx is not None and rope is not None) else pos
        qkv, residual, rotated = layer.attn_in_rope(x, residual, (rows_pos, cos, sin) if rope is not None else None)
        if packed_idx is not None:
            o = ops.flash_attention_packed(qkv, packed_idx, B, S, cfg.num_heads, cfg.num_kv_heads, cfg.head_dim, True,
                                           cfg.sliding_window, kv_start=ks, rope=rope, inv=packed_inv,
                                           rope_done=rotated)
        else:
            o = ops.flash_attention_qkv(qkv, B, S, cfg.num_heads, cfg.num_kv_heads, cfg.head_dim, True,
                                        cfg.sliding_window, kv_start=ks, rope=rope, rope_done=rotated)
        if out_rows is not None:
            # everything after attention is row-local: drop the rows nobody reads before o_proj
            inv = ops.packed_inverse(out_rows, o.shape[0])
            o = ops.gather_rows(o, out_rows, inv)
            residual = ops.gather_rows(residual, out_rows, inv)
        return layer.mlp(o, residual)

    # ------------------------------------------------------------------ generation
    @torch.no_grad()
    def prefill(self, input_ids, kv_start, cache, packed=None) -> torch.Tensor:
        """Prompt forward writing K/V into ``cache`` slots [0, S); returns final hidden at the last
        position of every row [B, H] (rows are left-padded so all end at S-1).

        ``packed`` = (idx [N] device grid positions, off host row offsets) from ``packed_index``:
        the projection GEMMs skip the left pads; each layer's qkv is scattered into the zeroed
        [B*S] grid for RoPE + cache append + attention, and the outputs gathered back."""
        cfg = self.cfg
        B, S = input_ids.shape
        dev = input_ids.device
        pos = self.positions(B, S, kv_start, dev)
        cos, sin = self.rope(dev)
        ks = kv_start.to(torch.int32)
        idx = packed[0] if packed is not None else None
        if idx is not None:
            x = self.embed_tokens(input_ids.reshape(-1).index_select(0, idx), pos.index_select(0, idx))
            inv = ops.packed_inverse(idx, B * S)
        else:
            x = self.embed_tokens(input_ids.reshape(-1), pos)
        residual = None
        rows_pos = pos.index_select(0, idx) if (idx is not None and cos is not None) else pos
        for li, layer in enumerate(self.layers):
            qkv, residual, rotated = layer.attn_in_rope(x, residual, (rows_pos, cos, sin) if cos is not None else None)
            if idx is not None:
                qkv = ops.scatter_rows(qkv, idx, inv, B * S)
            # rotated: q / k came out of the projection's epilogue already rotated (cache append only)
            rc, rs = (None, None) if rotated else (cos, sin)
            if getattr(cache, "fp8", False):
                # fp8 cache: rotate in place, then quantise the prompt K / V rows into it
                if not rotated:
                    ops.rope_qkv_(qkv, pos, cos, sin, cfg.num_heads, cfg.num_kv_heads, cfg.head_dim, S=S)
                k_sc, v_sc = cache.scales(li)
                ops.kv_store_fp8(qkv, cache.k[li], cache.v[li], k_sc, v_sc, B, S, cfg.num_heads)
            else:
                ops.rope_qkv_(qkv, pos, rc, rs, cfg.num_heads, cfg.num_kv_heads, cfg.head_dim, S=S,
                              k_cache=cache.k[li], v_cache=cache.v[li], slot_base=None)
            o = ops.flash_attention_qkv(qkv, B, S, cfg.num_heads, cfg.num_kv_heads, cfg.head_dim, True,
                                        cfg.sliding_window, kv_start=ks)
            if li == len(self.layers) - 1:
                # only the last position of every row is sampled from: the last layer's o_proj and
                # MLP run on B rows (its K/V above still covered the whole prompt)
                last = torch.arange(B, device=dev) * S + (S - 1)
                o = o.index_select(0, last)
                residual = residual.index_select(0, torch.from_numpy(packed[1][1:] - 1).to(dev)
                                                 if idx is not None else last)
            elif idx is not None:
                o = ops.gather_rows(o, idx, inv)
            x, residual = layer.mlp(o, residual)
        return self.final_norm(x, residual)

    @torch.no_grad()
    def decode(self, tokens, pos, slot, attn_len, kv_start, cache, workspace=None) -> torch.Tensor:
        """One step: tokens [B] at rotary position pos [B] written to cache slot ``slot`` [B];
        attention over ``attn_len`` [B] keys. Returns final hidden [B, H]."""
        cfg = self.cfg
        cos, sin = self.rope(tokens.device)
        x = self.embed_tokens(tokens, pos)
        fp8 = bool(self.layers) and self.layers[0].fp8_enabled
        max_b = self.fused_decode_max_batch_fp8 if fp8 else self.fused_decode_max_batch
        if (self.fused_decode and cfg.arch != "opt" and x.is_cuda and x.shape[0] <= max_b
                and not torch.is_grad_enabled()):
            h = x
            kv8 = getattr(cache, "fp8", False)
            for li, layer in enumerate(self.layers):
                def attend(qkv, li=li):
                    ks, vs = cache.scales(li) if kv8 else (None, None)
                    return ops.decode_step_attention(qkv, cache.k[li], cache.v[li], slot, attn_len, cfg.num_heads,
                                                     pos, cos, sin, kv_start, cfg.sliding_window,
                                                     workspace=workspace, k_scale=ks, v_scale=vs)
                h = layer.decode_fused(h, attend)
            y, _ = ops.rms_norm(h, self.norm_w, cfg.norm_eps)
            return y
        residual = None
        # batch > 64: split-K GEMM partials flow unreduced into the attention prologue and the norms
        defer = x.is_cuda and x.shape[0] > 64 and self.defer_splitk
        kv8 = getattr(cache, "fp8", False)
        for li, layer in enumerate(self.layers):
            qkv, residual = layer.attn_in(x, residual, defer)
            # one fused kernel: RoPE(q, k_new) + cache append + split-K attention + combine
            ks, vs = cache.scales(li) if kv8 else (None, None)
            o = ops.decode_step_attention(qkv, cache.k[li], cache.v[li], slot, attn_len, cfg.num_heads, pos, cos, sin,
                                          kv_start, cfg.sliding_window, workspace=workspace, k_scale=ks, v_scale=vs)
            x, residual = layer.mlp(o, residual, defer)
        return self.final_norm(x, residual)

    # ------------------------------------------------------------------ LoRA
    def add_lora(self, r: int = 16, alpha: float = 32.0, targets=None, dropout: float = 0.0, seed: int = 0):
        """Attach PEFT-style LoRA adapters (A kaiming-uniform, B zero) to the target projections."""
        from .lora import attach_lora

        return attach_lora(self, r, alpha, targets, dropout, seed)

    def lora_parameters(self) -> List[nn.Parameter]:
        out = []
        for layer in self.layers:
            out += list(layer.lora_params.values())
        return out

    def set_lora_enabled(self, on: bool):
        for layer in self.layers:
            layer.lora_enabled = on

    def set_lora_merged(self, on: bool):
        """Inference with merged adapter weights (W + s B A, kept in sync lazily after updates).
        Returns the previous setting."""
        prev = False
        for layer in self.layers:
            for g in layer.lora.values():
                prev = prev or g.use_merged
                g.use_merged = on
        return prev

    def refresh_decode_weights(self, batch: Optional[int] = None):
        """Eagerly refresh the images the fused decode layer's graph replays read (norm-folded /
        tile-ordered / fp8 weights). ``batch``: the decode batch about to run — above the fused
        layer's limit none of them is read, so batch-256 rollouts skip the refresh (a later
        small-batch generation refreshes them before its replays). Same-box A/B: within noise
        (profiles/r6/bench_decode_refresh_gating_ab.log)."""
        if batch is not None:
            fp8 = bool(self.layers) and self.layers[0].fp8_enabled
            if batch > (self.fused_decode_max_batch_fp8 if fp8 else self.fused_decode_max_batch):
                return
        if self.fused_decode:
            for layer in self.layers:
                layer.refresh_decode_weights()
        if self._head_shuf is not None:
            self._head_shuf.get(self.head_weight)

    def set_fp8(self, on: bool = True, train: Optional[bool] = None):
        """fp8 (e4m3fn) weights for no-grad forwards (prefill, decode, reference scoring):
        W8A8 MX-MFMA GEMMs for M > 64, W8A16 weight streaming for decode. ``train``: the frozen
        base product of LoRA training forwards runs W8A8 as well (the adapter term and every
        backward GEMM stay bf16); None keeps the current setting. Returns the previous ``on``."""
        prev = any(layer.fp8_enabled for layer in self.layers)
        for layer in self.layers:
            layer.fp8_enabled = on
            if train is not None:
                layer.fp8_train = bool(train) and on
        return prev

    def refresh_lora(self):
        """Rebuild every adapter's bf16 compute images after an optimizer step: one native launch
        for the whole model on the GPU (``ops.refresh_lora_batched``), per-group copies otherwise."""
        groups = [g for layer in self.layers for g in layer.lora.values()]
        if ops.refresh_lora_batched(groups, self.dtype):
            return
        for g in groups:
            g.refresh(dtype=self.dtype)

    def freeze_base(self):
        for n, p in self.named_parameters():
            if "lora" not in n:
                p.requires_grad_(False)


def packed_index(lo, hi, L: int, device):
    """Varlen packing of a [B, L] token grid: row b keeps its positions [lo[b], hi[b]) (host integer
    arrays). Returns (idx, off): ``idx`` [N] int64 on ``device`` = grid position b*L + s of every
    kept token in row-major order; ``off`` [B+1] host offsets of each row's first packed token."""
    lo = np.asarray(lo, dtype=np.int64).reshape(-1)
    hi = np.maximum(np.asarray(hi, dtype=np.int64).reshape(-1), lo)
    n = hi - lo
    off = np.zeros(len(n) + 1, dtype=np.int64)
    np.cumsum(n, out=off[1:])
    idx = np.repeat(np.arange(len(n), dtype=np.int64) * L - off[:-1] + lo, n) + np.arange(off[-1], dtype=np.int64)
    return torch.from_numpy(idx).to(device), off


def pack_enabled() -> bool:
    """Varlen packing of training / scoring / prefill forwards (RAGTL_PACK=0 turns it off)."""
    return os.environ.get("RAGTL_PACK", "1") != "0"


def shuffle_enabled(m: int) -> bool:
    """Decode GEMMs at batch ``m`` <= 16 stream tile-ordered weight images (ops.ShufCache; the
    split-K image launches run 5-20 % faster than row-major). RAGTL_DECODE_SHUF=0 turns it off."""
    return m <= 16 and os.environ.get("RAGTL_DECODE_SHUF", "1") != "0"


def _normal_(p: torch.Tensor, std: float, g: torch.Generator):
    # generate in chunks on CPU for reproducibility across devices, then copy
    flat = p.view(-1)
    n = flat.numel()
    chunk = 1 << 26
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        flat[s:e].copy_(torch.randn(e - s, generator=g) * std)


def fast_random_init_(model: nn.Module, seed: int = 0, std: float = 0.02):
    """Device-side random init for large models (bench/smoke): identical for every rank with the
    same seed. Norm weights 1, biases 0, LoRA untouched."""
    gen = None
    for name, p in model.named_parameters():
        if "lora" in name:
            continue
        with torch.no_grad():
            if name.endswith("_w") and ("ln" in name or "norm" in name):
                p.fill_(1.0)
            elif name.endswith("_b"):
                p.zero_()
            else:
                if gen is None or gen.device != p.device:
                    gen = torch.Generator(device=p.device).manual_seed(seed)
                p.normal_(0.0, std, generator=gen)
