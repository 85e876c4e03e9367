"""SwiGLU, embedding gather, token log-probs / entropy, sampler, retrieval and RL kernels."""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from . import reference as ref
from ._ext import native, on_gpu


# ------------------------------------------------------------------------------------ SwiGLU
class _SwiGLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu):
        gu = gu.contiguous()
        ctx.save_for_backward(gu)
        return native().swiglu_fwd(gu)

    @staticmethod
    def backward(ctx, dy):
        (gu,) = ctx.saved_tensors
        return native().swiglu_bwd(gu, dy.contiguous())


def _swiglu_grad(gu: torch.Tensor, dy: torch.Tensor) -> torch.Tensor:
    """d[gate | up] of silu(gate) * up given the [gate | up] pre-activation and dL/dy."""
    if on_gpu(gu):
        return native().swiglu_bwd(gu.contiguous(), dy.contiguous())
    with torch.enable_grad():
        p = gu.detach().float().requires_grad_(True)
        F2 = p.shape[-1]
        (g,) = torch.autograd.grad(F.silu(p[..., : F2 // 2]) * p[..., F2 // 2:], p, dy.float())
    return g.to(gu.dtype)


def swiglu(gu: torch.Tensor) -> torch.Tensor:
    """silu(gate) * up for gu = [gate | up] along the last dim."""
    if not on_gpu(gu):
        F2 = gu.shape[-1]
        return F.silu(gu[..., : F2 // 2]) * gu[..., F2 // 2:]
    if torch.is_grad_enabled() and gu.requires_grad:
        return _SwiGLUFn.apply(gu)
    return native().swiglu_fwd(gu.contiguous())


# --------------------------------------------------------------------------------- embedding
class _EmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, table, ids):
        ctx.save_for_backward(ids)
        ctx.shape = table.shape
        return native().embed(table, ids.contiguous(), None, None)

    @staticmethod
    def backward(ctx, g):
        """Table gradient without arrival-order atomics: the rows are sorted by id (stable) and each
        distinct id's rows summed in that fixed order (segment_mean kernel, sum mode), then added
        once per distinct id — bitwise reproducible (full fine-tuning trains the table)."""
        (ids,) = ctx.saved_tensors
        d = torch.zeros(ctx.shape, dtype=torch.float32, device=g.device)
        flat = ids.reshape(-1)
        g2 = g.reshape(-1, ctx.shape[1]).float().contiguous()
        order = torch.argsort(flat, stable=True)
        uniq, counts = torch.unique_consecutive(flat[order], return_counts=True)
        seg = torch.zeros(uniq.numel() + 1, dtype=torch.int32, device=g.device)
        seg[1:] = counts.cumsum(0)
        sums = torch.empty(uniq.numel(), ctx.shape[1], dtype=torch.float32, device=g.device)
        native().segment_mean(g2, order, seg, 2, sums)
        d.index_add_(0, uniq, sums)  # distinct rows: one add per element
        return d.to(g.dtype), None


def embedding(table: torch.Tensor, ids: torch.Tensor, pos_table=None, pos_ids=None) -> torch.Tensor:
    if not on_gpu(table):
        out = F.embedding(ids, table)
        if pos_table is not None:
            out = out + F.embedding(pos_ids, pos_table)
        return out
    if torch.is_grad_enabled() and table.requires_grad:
        out = _EmbedFn.apply(table, ids.long())
        if pos_table is not None:
            out = out + _EmbedFn.apply(pos_table, pos_ids.long()) if pos_table.requires_grad else \
                out + native().embed(pos_table, pos_ids.long().contiguous(), None, None)
        return out
    return native().embed(table, ids.long().contiguous(), pos_table,
                          pos_ids.long().contiguous() if pos_ids is not None else None)


# --------------------------------------------------------------------------- token log-probs
class _LogProbFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, targets, inv_temp):
        logp, ent, lse, ex = native().logprob_fwd(logits, targets, inv_temp, True)
        ctx.save_for_backward(logits, targets if targets is not None else torch.empty(0, dtype=torch.long), lse, ex)
        ctx.inv_temp = inv_temp
        ctx.has_t = targets is not None
        return logp, ent

    @staticmethod
    def backward(ctx, g_lp, g_ent):
        logits, targets, lse, ex = ctx.saved_tensors
        gl = g_lp.float().contiguous() if g_lp is not None else None
        ge = g_ent.float().contiguous() if g_ent is not None else None
        d = native().logprob_bwd(logits, targets if ctx.has_t else None, ctx.inv_temp, lse, ex, gl, ge)
        return d.to(logits.dtype), None, None


def token_logprobs(logits: torch.Tensor, targets, inv_temp: float = 1.0):
    """Per-row (log p(target), entropy) of softmax(logits * inv_temp); logits [T, V]."""
    if not on_gpu(logits):
        lp, ent, _, _ = ref.logprob(logits, targets, inv_temp)
        return lp, ent
    if logits.stride(-1) != 1:
        logits = logits.contiguous()
    V = logits.shape[-1]
    if V % 8 or logits.stride(0) % 8:
        # the kernel streams 16-B row vectors: pad the vocabulary up to a multiple of 8 columns with a
        # large negative logit (probability exactly 0 and p * x = 0 in the entropy; finite even after
        # the temperature scaling, unlike finfo.min)
        Vp = (V + 7) // 8 * 8
        pad = torch.full((logits.shape[0], Vp - V), -1e30, dtype=logits.dtype, device=logits.device)
        logits = torch.cat([logits, pad], 1)
    if torch.is_grad_enabled() and logits.requires_grad:
        return _LogProbFn.apply(logits, targets, inv_temp)
    lp, ent, _, _ = native().logprob_fwd(logits, targets, inv_temp, True)
    return lp, ent


# --------------------------------------------------------------------------------- sampler
def sample(logits, inv_temp=1.0, top_k=0, top_p=1.0, greedy=False, seed=0, offset=None, active=None,
           out_tok=None, out_logp=None, generator=None):
    """Draw one token per row; returns (tokens int64 [B], logp of drawn token [B])."""
    B = logits.shape[0]
    if not on_gpu(logits):
        tok, lp = ref.sample(logits, inv_temp, top_k, top_p, greedy, generator)
        if out_tok is not None:
            out_tok.copy_(tok)
            tok = out_tok
        if out_logp is not None:
            out_logp.copy_(lp)
            lp = out_logp
        return tok, lp
    if out_tok is None:
        out_tok = torch.empty(B, dtype=torch.long, device=logits.device)
    if out_logp is None:
        out_logp = torch.empty(B, dtype=torch.float32, device=logits.device)
    native().sample(logits, inv_temp, top_k, top_p, greedy, seed, offset, active, out_tok, out_logp)
    return out_tok, out_logp


# ------------------------------------------------------------------------------- retrieval
def pool_normalize(x: torch.Tensor, lengths=None, normalize: bool = True) -> torch.Tensor:
    """Masked mean over tokens + L2 normalisation: [B, S, H] -> [B, H] fp32."""
    if on_gpu(x):
        return native().pool_norm(x.contiguous(), lengths.int() if lengths is not None else None, normalize)
    return ref.pool_norm(x, lengths, normalize)


def topk(scores: torch.Tensor, k: int, idmap=None):
    """Row-wise top-k (descending) of fp32 scores [nq, N] -> (values, ids)."""
    if on_gpu(scores) and k <= 512:
        return native().topk(scores.float().contiguous(), k, idmap)
    return ref.topk(scores, k, idmap)


def ivf_scan(q, probes, lstart, lsize, vecs, ids, maxlen, sqnorm=None, l2: bool = False):
    """IVF list scan (GPU): scores of every vector of each probed list -> (cand [nq, nprobe*maxlen],
    ids); inner product, or the negated squared L2 distance."""
    return native().ivf_scan(q.contiguous(), probes.int().contiguous(), lstart, lsize, vecs, ids, sqnorm, l2, maxlen)


def segment_mean(x, order, seg, normalize: bool, out):
    """out[c] = mean(x[order[seg[c]:seg[c+1]]]) (L2-normalised if asked); empty segments untouched."""
    if on_gpu(x):
        return native().segment_mean(x.float().contiguous(), order.long().contiguous(), seg.int().contiguous(),
                                     int(bool(normalize)), out)
    return ref.segment_mean(x, order, seg, normalize, out)


# ---------------------------------------------------------------------------------------- RL
class _PPOLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, lp, vals, ent, old, adv, ret, mask, vold, eps, c_v, c_e, vclip, ref_lp, kl_coef):
        f = lambda t: t.detach().float().contiguous()  # noqa: E731
        stats, dlp, dv, dent = native().ppo_loss(f(lp), f(old), f(adv), f(vals), f(ret),
                                                 f(vold) if vold is not None else None, f(ent), f(mask),
                                                 eps, c_v, c_e, vclip if vclip else 0.0,
                                                 f(ref_lp) if ref_lp is not None else None, kl_coef)
        ctx.save_for_backward(dlp, dv, dent)
        ctx.mark_non_differentiable(stats)
        return stats[0], stats

    @staticmethod
    def backward(ctx, g, _gstats):
        dlp, dv, dent = ctx.saved_tensors
        return dlp * g, dv * g, dent * g, None, None, None, None, None, None, None, None, None, None, None


def ppo_loss(lp, vals, ent, old, adv, ret, mask, eps: float, c_v: float, c_e: float, vclip=None, vold=None,
             ref_lp=None, kl_coef: float = 0.0):
    """Token-level clipped PPO objective: ``(loss, stats)`` with stats = [loss,
    policy_loss, value_loss, entropy, approx_kl, clipfrac, kl_ref_k3, kl_ref_k1, n_tokens]; one
    fused HIP kernel computes the loss and its gradient (w.r.t. lp, vals, ent) together on the GPU.
    ``ref_lp`` (frozen-reference log-probs of the same tokens): adds ``kl_coef * mean(k3)`` with
    k3 = exp(ref - lp) - (ref - lp) - 1, the reference-KL penalty on the update forward's own
    (training-numerics) log-probs (PPOConfig.kl_in_loss)."""
    if on_gpu(lp):
        return _PPOLossFn.apply(lp, vals, ent, old, adv, ret, mask.float(), vold, float(eps), float(c_v),
                                float(c_e), float(vclip) if vclip else 0.0, ref_lp, float(kl_coef))
    return ref.ppo_loss(lp, old, adv, vals, ret, ent, mask.float(), eps, c_v, c_e, vclip, vold, ref_lp, kl_coef)


class _RowDotFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, w, b):
        ctx.save_for_backward(h, w)
        return native().rowdot(h, w, b)

    @staticmethod
    def backward(ctx, g):
        h, w = ctx.saved_tensors
        g = g.float()
        dh = (g[:, None] * w[None, :]).to(h.dtype) if ctx.needs_input_grad[0] else None
        dw = (g[:, None] * h.float()).sum(0) if ctx.needs_input_grad[1] else None
        db = g.sum().reshape(1) if ctx.needs_input_grad[2] else None
        return dh, dw, db


def row_dot(h: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Per-row h . w (+ b) in fp32 (the scalar value head): on the GPU one wave per row in a fixed
    order (``rowdot_kernel``), so a row's value is bitwise independent of the other rows in the
    launch; h [T, H] bf16, w [H] fp32. CPU: the fp32 expression."""
    if on_gpu(h) and h.dtype == torch.bfloat16 and h.shape[-1] % 8 == 0:
        h2 = h.reshape(-1, h.shape[-1])
        if h2.stride(-1) != 1 or h2.stride(0) % 8 or h2.data_ptr() % 16:
            h2 = h2.contiguous()
        y = _RowDotFn.apply(h2, w.contiguous(), b)
        return y.reshape(h.shape[:-1])
    y = (h.float() * w).sum(-1)
    return y + b if b is not None else y


def ppo_advantages(old_logp, ref_logp, values, scores, resp_len, kl_coef: float, gamma: float, lam: float,
                   whiten: bool = True, eps: float = 1e-8):
    """Token rewards (-kl_coef (old - ref) per token + the score at the last response token), GAE
    over the old values and masked advantage whitening in one launch on GPU.
    -> (advantages, returns, token rewards, per-sequence KL sum)."""
    f = lambda t: t.float().contiguous()  # noqa: E731
    if on_gpu(old_logp):
        return native().ppo_advantages(f(old_logp), f(ref_logp), f(values), f(scores), resp_len.int().contiguous(),
                                       kl_coef, gamma, lam, whiten, eps)
    return ref.ppo_advantages(f(old_logp), f(ref_logp), f(values), f(scores), resp_len, kl_coef, gamma, lam, whiten,
                              eps)


def gae(rewards, values, mask, gamma: float, lam: float):
    if on_gpu(rewards):
        return native().gae(rewards.float().contiguous(), values.float().contiguous(), mask.float().contiguous(),
                            gamma, lam)
    return ref.gae(rewards.float(), values.float(), mask.float(), gamma, lam)
