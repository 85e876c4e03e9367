"""Sentence-transformer bi-encoders: BERT (all-MiniLM-L6-v2) and MPNet (all-mpnet-base-v2).

Post-LN transformer encoders with bidirectional, key-length-masked attention (MPNet adds a
bucketed relative-position bias, applied through a per-head LUT inside the flash kernel),
followed by masked mean pooling and L2 normalisation — the `SentenceTransformer.encode` path the
reference calls per string (reinforcement_learning_optimization_after_rag.py:55,66-67,75-76,102-103),
here batched into one forward.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from .. import ops
from .config import ModelConfig


def relative_position_bucket(rel: torch.Tensor, num_buckets: int = 32, max_distance: int = 128) -> torch.Tensor:
    """MPNet/T5 bidirectional bucket of relative position rel = key - query."""
    ret = torch.zeros_like(rel)
    n = -rel
    num_buckets //= 2
    ret = ret + (n < 0).long() * num_buckets
    n = n.abs()
    max_exact = num_buckets // 2
    is_small = n < max_exact
    val_large = max_exact + (torch.log(n.float().clamp(min=1) / max_exact) / math.log(max_distance / max_exact)
                             * (num_buckets - max_exact)).long()
    val_large = torch.minimum(val_large, torch.full_like(val_large, num_buckets - 1))
    return ret + torch.where(is_small, n, val_large)


class EncoderLayer(nn.Module):
    def __init__(self, cfg: ModelConfig, device=None, dtype=torch.bfloat16):
        super().__init__()
        H, F = cfg.hidden_size, cfg.intermediate_size
        kw = dict(device=device, dtype=dtype)
        self.qkv_w = nn.Parameter(torch.empty(3 * H, H, **kw))
        self.qkv_b = nn.Parameter(torch.zeros(3 * H, **kw))
        self.o_w = nn.Parameter(torch.empty(H, H, **kw))
        self.o_b = nn.Parameter(torch.zeros(H, **kw))
        self.ln1_w = nn.Parameter(torch.ones(H, **kw))
        self.ln1_b = nn.Parameter(torch.zeros(H, **kw))
        self.fc1_w = nn.Parameter(torch.empty(F, H, **kw))
        self.fc1_b = nn.Parameter(torch.zeros(F, **kw))
        self.fc2_w = nn.Parameter(torch.empty(H, F, **kw))
        self.fc2_b = nn.Parameter(torch.zeros(H, **kw))
        self.ln2_w = nn.Parameter(torch.ones(H, **kw))
        self.ln2_b = nn.Parameter(torch.zeros(H, **kw))


class SentenceEncoder(nn.Module):
    def __init__(self, cfg: ModelConfig, device=None, dtype=torch.bfloat16, init: bool = True, seed: int = 0):
        super().__init__()
        assert cfg.arch in ("bert", "mpnet")
        self.cfg = cfg
        self.dtype = dtype
        H = cfg.hidden_size
        kw = dict(device=device, dtype=dtype)
        self.word_embed = nn.Parameter(torch.empty(cfg.vocab_size, H, **kw))
        self.pos_embed = nn.Parameter(torch.empty(cfg.max_position, H, **kw))
        if cfg.type_vocab_size:
            self.type_embed = nn.Parameter(torch.empty(cfg.type_vocab_size, H, **kw))
        self.emb_ln_w = nn.Parameter(torch.ones(H, **kw))
        self.emb_ln_b = nn.Parameter(torch.zeros(H, **kw))
        self.layers = nn.ModuleList([EncoderLayer(cfg, device, dtype) for _ in range(cfg.num_layers)])
        if cfg.arch == "mpnet":
            self.rel_bias = nn.Parameter(torch.empty(cfg.relative_buckets, cfg.num_heads, **kw))
        self._lut = None
        if init:
            self.reset_parameters(seed)

    @torch.no_grad()
    def reset_parameters(self, seed: int = 0):
        g = torch.Generator(device="cpu").manual_seed(seed)
        for name, p in self.named_parameters():
            if name.endswith("_b"):
                p.zero_()
            elif "ln" in name and name.endswith("_w"):
                p.fill_(1.0)
            else:
                p.copy_((torch.randn(p.shape, generator=g) * self.cfg.initializer_range).to(p.dtype))

    def _bias_lut(self, L: int, device):
        """[heads, 2L-1] additive score bias in log2 units, indexed by (key - query) + L - 1."""
        if self.cfg.arch != "mpnet":
            return None, 0
        if self._lut is None or self._lut[1] < L or self._lut[0].device != torch.device(device):
            rel = torch.arange(-(L - 1), L, device=device)
            buckets = relative_position_bucket(rel, self.cfg.relative_buckets, self.cfg.relative_max_distance)
            lut = self.rel_bias.float()[buckets].t().contiguous() * (1.0 / math.log(2.0))
            self._lut = (lut, L)
        return self._lut

    def forward(self, input_ids: torch.Tensor, lengths: torch.Tensor) -> torch.Tensor:
        """input_ids [B, S] right-padded, lengths [B] -> token states [B*S, H]."""
        cfg = self.cfg
        B, S = input_ids.shape
        dev = input_ids.device
        H, nh, D = cfg.hidden_size, cfg.num_heads, cfg.head_dim
        ar = torch.arange(S, device=dev)[None, :].expand(B, S)
        valid = ar < lengths.to(dev).long()[:, None]
        if cfg.arch == "mpnet":
            pos = torch.where(valid, ar + cfg.pad_token_id + 1, torch.full_like(ar, cfg.pad_token_id))
        else:
            pos = ar
        x = ops.embedding(self.word_embed, input_ids.reshape(-1), self.pos_embed, pos.reshape(-1))
        if cfg.type_vocab_size:
            x = x + self.type_embed[0]
        x, _ = ops.layer_norm(x, self.emb_ln_w, self.emb_ln_b, cfg.norm_eps)
        lens32 = lengths.to(dev).to(torch.int32)
        lut, L = self._bias_lut(max(S, 1), dev)
        for layer in self.layers:
            qkv = ops.linear(x, layer.qkv_w, layer.qkv_b)
            q, k, v = qkv[:, :H], qkv[:, H:2 * H], qkv[:, 2 * H:]
            a = ops.attention(q, k, v, B, S, S, nh, nh, D, causal=False, kv_len=lens32, rel_bias_lut=lut, rb_L=L)
            a = ops.linear(a, layer.o_w, layer.o_b)
            x, _ = ops.layer_norm(a, layer.ln1_w, layer.ln1_b, cfg.norm_eps, residual=x)
            f = ops.linear(x, layer.fc1_w, layer.fc1_b, act=cfg.hidden_act)
            d = ops.linear(f, layer.fc2_w, layer.fc2_b)
            x, _ = ops.layer_norm(d, layer.ln2_w, layer.ln2_b, cfg.norm_eps, residual=x)
        return x

    @torch.no_grad()
    def encode_ids(self, input_ids: torch.Tensor, lengths: torch.Tensor, normalize: bool = True) -> torch.Tensor:
        B, S = input_ids.shape
        x = self.forward(input_ids, lengths)
        return ops.pool_normalize(x.view(B, S, -1), lengths.to(x.device), normalize)
