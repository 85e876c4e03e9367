"""Shared training pieces: sequence scoring (token log-probs / entropy / values in one forward),
masked reductions, LR schedules."""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import torch

from .. import ops
from ..models.decoder import pack_enabled, packed_index


def masked_mean(x: torch.Tensor, mask: torch.Tensor, dim=None) -> torch.Tensor:
    m = mask.to(x.dtype)
    if dim is None:
        return (x * m).sum() / m.sum().clamp(min=1.0)
    return (x * m).sum(dim) / m.sum(dim).clamp(min=1.0)


def masked_whiten(x: torch.Tensor, mask: torch.Tensor, shift_mean: bool = True, eps: float = 1e-8) -> torch.Tensor:
    mean = masked_mean(x, mask)
    var = masked_mean((x - mean) ** 2, mask)
    w = (x - mean) * torch.rsqrt(var + eps)
    if not shift_mean:
        w = w + mean
    return w * mask.to(x.dtype)


def response_mask(lengths: torch.Tensor, T: int) -> torch.Tensor:
    return torch.arange(T, device=lengths.device)[None, :] < lengths[:, None]


def score_sequences(model, prompt_ids: torch.Tensor, start: torch.Tensor, resp: torch.Tensor,
                    resp_len: torch.Tensor, inv_temp: float = 1.0, value_head=None,
                    gradient_checkpointing: bool = False, lengths=None):
    """See :func:`_score_sequences`. Runs under ``ops.batch_invariant()``: a row's log-probs /
    entropy / value are bitwise the same whatever rows share the forward (minibatch 32 or 128,
    padded or packed, grad or no grad) — the PPO ratio is exactly 1 at theta_old under
    ``old_logp="recompute"`` and the reference KL is exactly 0 at LoRA B = 0."""
    with ops.batch_invariant():
        return _score_sequences(model, prompt_ids, start, resp, resp_len, inv_temp, value_head,
                                gradient_checkpointing, lengths)


def _score_sequences(model, prompt_ids: torch.Tensor, start: torch.Tensor, resp: torch.Tensor,
                     resp_len: torch.Tensor, inv_temp: float = 1.0, value_head=None,
                     gradient_checkpointing: bool = False, lengths=None):
    """One forward over [prompt | response] -> per-response-token (logp, entropy, values).

    The hidden state at position S-1+t produces the distribution of response token t and is also
    the state whose value is V_t (the reference instead runs two forwards and scores a response
    against a different prompt).

    ``lengths`` = host (start, resp_len) integer arrays: varlen form. Row b needs only the inputs
    [start_b, S + resp_len_b - 1); when that drops >= 3 % of the [B, S+T] grid the forward runs
    packed (``CausalLM.forward(packed_idx=...)``: no GEMM / norm work on left or right pads), the
    lm_head / log-softmax / value head run on the sum(resp_len) scored rows only, and the outputs
    are scattered back to [B, T] (zeros at masked positions)."""
    B, S = prompt_ids.shape
    T = resp.shape[1]
    seq = torch.cat([prompt_ids, resp], 1)
    mask = response_mask(resp_len, T)
    grad = torch.is_grad_enabled()
    if lengths is not None and pack_enabled():
        st = np.asarray(lengths[0], dtype=np.int64).reshape(-1)
        rl = np.asarray(lengths[1], dtype=np.int64).reshape(-1)
        lo, hi = st, S + np.maximum(rl - 1, 0)
        n_tok = int(np.maximum(hi - lo, 0).sum())
        n_sc = int(rl.sum())
        if n_sc > 0 and n_tok < 0.97 * B * (S + T):
            dev = prompt_ids.device
            idx, off = packed_index(lo, hi, S + T, dev)
            b = np.repeat(np.arange(B, dtype=np.int64), rl)
            t = np.arange(n_sc, dtype=np.int64) - np.repeat(np.cumsum(rl) - rl, rl)
            sel = torch.from_numpy(off[:-1][b] + (S - 1 + t) - lo[b]).to(dev)
            dst = torch.from_numpy(b * T + t).to(dev)
            # hidden states of the scored rows only (the last layer's o_proj / MLP skip the rest)
            hs = model(seq, kv_start=start.to(torch.int32), gradient_checkpointing=gradient_checkpointing,
                       packed_idx=idx, out_rows=sel)
            tgt = resp.reshape(-1).index_select(0, dst)
            logits = ops.linear(hs, model.head_weight) if (grad and hs.requires_grad) else \
                ops.gemm(hs.contiguous(), model.head_weight)
            lp, ent = ops.token_logprobs(logits, tgt, inv_temp)
            logp = lp.new_zeros(B * T).index_copy(0, dst, lp).view(B, T)
            entf = ent.new_zeros(B * T).index_copy(0, dst, ent).view(B, T)
            values = None
            if value_head is not None:
                v = value_head(hs).reshape(-1)
                values = v.new_zeros(B * T).index_copy(0, dst, v).view(B, T)
            return logp, entf, values, mask
    rows = (torch.arange(B, device=seq.device)[:, None] * (S + T) +
            torch.arange(S - 1, S + T - 1, device=seq.device)[None, :]).reshape(-1)
    h = model(seq, kv_start=start.to(torch.int32), gradient_checkpointing=gradient_checkpointing, out_rows=rows)
    tgt = torch.where(mask, resp, torch.full_like(resp, -100)).reshape(-1)
    logits = ops.linear(h, model.head_weight) if (grad and h.requires_grad) else \
        ops.gemm(h.contiguous(), model.head_weight)
    logp, ent = ops.token_logprobs(logits, tgt, inv_temp)
    values = value_head(h).view(B, T) if value_head is not None else None
    return logp.view(B, T), ent.view(B, T), values, mask


def lr_at(step: int, base: float, schedule: str = "constant", warmup: int = 0, total: int = 0,
          min_ratio: float = 0.0) -> float:
    """constant / linear / cosine with linear warmup (the reference imports get_scheduler but never
    uses it, rl.py:11)."""
    if warmup and step < warmup:
        return base * (step + 1) / warmup
    if schedule == "constant" or total <= warmup:
        return base
    p = min(1.0, (step - warmup) / max(1, total - warmup))
    if schedule == "linear":
        return base * (min_ratio + (1 - min_ratio) * (1 - p))
    if schedule == "cosine":
        return base * (min_ratio + (1 - min_ratio) * 0.5 * (1 + math.cos(math.pi * p)))
    raise ValueError(schedule)
