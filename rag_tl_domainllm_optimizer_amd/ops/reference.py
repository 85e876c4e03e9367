"""Eager PyTorch implementations of every native op.

These are (a) the execution path for CPU tensors (the CPU plumbing config, unit tests without a
GPU) and (b) the fp32 numerics oracles the HIP kernels are tested against. They mirror the exact
contract of the corresponding kernel in ``csrc/kernels`` (layouts, masks, rounding points).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

ACT_NONE, ACT_RELU, ACT_GELU, ACT_GELU_TANH, ACT_SILU = 0, 1, 2, 3, 4


def apply_act(y: torch.Tensor, act: int) -> torch.Tensor:
    if act == ACT_RELU:
        return F.relu(y)
    if act == ACT_GELU:
        return F.gelu(y)
    if act == ACT_GELU_TANH:
        return F.gelu(y, approximate="tanh")
    if act == ACT_SILU:
        return F.silu(y)
    return y


def gemm(a, w, u=None, ub=None, bias=None, act=ACT_NONE, out_f32=False):
    y = a.float() @ w.float().t()
    if u is not None:
        y = y + u.float() @ ub.float().t()
    if bias is not None:
        y = y + bias.float()
    y = apply_act(y, act)
    return y if out_f32 else y.to(a.dtype)


def norm(x, w, b=None, eps=1e-6, residual=None, layernorm=False):
    """Returns (y, h, rstd, mean): h = x + residual (rounded to x.dtype), y = norm(h)*w (+b)."""
    h = x
    if residual is not None:
        h = (x.float() + residual.float()).to(x.dtype)
    hf = h.float()
    if layernorm:
        mean = hf.mean(-1)
        var = (hf - mean[..., None]).pow(2).mean(-1)
        rstd = torch.rsqrt(var + eps)
        y = (hf - mean[..., None]) * rstd[..., None] * w.float()
        if b is not None:
            y = y + b.float()
    else:
        mean = None
        rstd = torch.rsqrt(hf.pow(2).mean(-1) + eps)
        y = hf * rstd[..., None] * w.float()
    return y.to(x.dtype), (h if residual is not None else None), rstd.reshape(-1), (
        mean.reshape(-1) if mean is not None else None)


def rope_tables(D: int, max_pos: int, theta: float = 10000.0, device=None):
    inv = 1.0 / (theta ** (torch.arange(0, D, 2, dtype=torch.float64) / D))
    t = torch.arange(max_pos, dtype=torch.float64)
    fr = torch.outer(t, inv)
    return fr.cos().float().to(device), fr.sin().float().to(device)


def rope_qkv(qkv, pos, cos, sin, Hq, Hkv, D, sign=1.0, rope_q=True):
    """Returns a rotated copy of the fused qkv rows ([T, >= (Hq+2Hkv)*D])."""
    out = qkv.clone()
    T = qkv.shape[0]
    half = D // 2
    c = cos[pos.long()].float()  # [T, D/2]
    s = sin[pos.long()].float() * sign
    heads = list(range(Hq if rope_q else 0)) + list(range(Hq, Hq + Hkv))
    for h in heads:
        x = qkv[:, h * D:(h + 1) * D].float()
        x1, x2 = x[:, :half], x[:, half:]
        y = torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)
        out[:, h * D:(h + 1) * D] = y.to(qkv.dtype)
    return out


def swiglu(gu):
    F2 = gu.shape[-1]
    g, u = gu[..., : F2 // 2].float(), gu[..., F2 // 2:].float()
    return (F.silu(g) * u).to(gu.dtype)


def swiglu_bwd(gu, dy):
    F2 = gu.shape[-1]
    g, u = gu[..., : F2 // 2].float(), gu[..., F2 // 2:].float()
    d = dy.float()
    sg = torch.sigmoid(g)
    du = d * g * sg
    dg = d * u * sg * (1 + g * (1 - sg))
    return torch.cat([dg, du], -1).to(gu.dtype)


def attention(q, k, v, B, Sq, Sk, Hq, Hkv, D, causal=True, window=0, scale=None, kv_start=None, kv_len=None,
              rel_bias=None, rb_L=0):
    """Token-major attention: q [B*Sq, >=Hq*D], k/v [B*Sk, >=Hkv*D] -> (o [B*Sq, Hq*D], lse [B,Hq,Sq])."""
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    qh = q[:, : Hq * D].float().reshape(B, Sq, Hq, D).transpose(1, 2)
    kh = k[:, : Hkv * D].float().reshape(B, Sk, Hkv, D).transpose(1, 2)
    vh = v[:, : Hkv * D].float().reshape(B, Sk, Hkv, D).transpose(1, 2)
    rep = Hq // Hkv
    kh = kh.repeat_interleave(rep, dim=1)
    vh = vh.repeat_interleave(rep, dim=1)
    s = torch.einsum("bhqd,bhkd->bhqk", qh, kh) * scale
    qi = torch.arange(Sq, device=q.device)[:, None]
    ki = torch.arange(Sk, device=q.device)[None, :]
    mask = torch.ones(B, 1, Sq, Sk, dtype=torch.bool, device=q.device)
    if causal:
        mask &= (ki <= qi)[None, None]
    if window and window > 0:
        mask &= ((qi - ki) < window)[None, None]
    if kv_start is not None:
        mask &= (ki[None] >= kv_start.long().view(B, 1, 1))[:, None]
    if kv_len is not None:
        mask &= (ki[None] < kv_len.long().view(B, 1, 1))[:, None]
    if rel_bias is not None:
        idx = (ki - qi) + rb_L - 1  # [Sq, Sk]
        s = s + rel_bias[:, idx].float()[None] / math.log2(math.e)
    s = s.masked_fill(~mask, float("-inf"))
    lse = torch.logsumexp(s, dim=-1)
    p = torch.exp(s - lse[..., None])
    p = torch.nan_to_num(p, nan=0.0)
    o = torch.einsum("bhqk,bhkd->bhqd", p, vh)
    lse = torch.where(torch.isfinite(lse), lse, torch.full_like(lse, float("inf")))
    return o.transpose(1, 2).reshape(B * Sq, Hq * D).to(q.dtype), lse


def decode_attention(q, kc, vc, kv_len, Hq, kv_start=None, window=0, scale=None):
    """q [B, >=Hq*D]; caches [B, Hkv, Smax, D]; returns o [B, Hq*D]."""
    B, Hkv, Smax, D = kc.shape
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    rep = Hq // Hkv
    qh = q[:, : Hq * D].float().reshape(B, Hq, D)
    kh = kc.float().repeat_interleave(rep, dim=1)
    vh = vc.float().repeat_interleave(rep, dim=1)
    s = torch.einsum("bhd,bhkd->bhk", qh, kh) * scale
    ki = torch.arange(Smax, device=q.device)[None, :]
    lo = torch.zeros(B, dtype=torch.long, device=q.device) if kv_start is None else kv_start.long()
    if window and window > 0:
        lo = torch.maximum(lo, kv_len.long() - window)
    mask = (ki >= lo[:, None]) & (ki < kv_len.long()[:, None])
    s = s.masked_fill(~mask[:, None, :], float("-inf"))
    vh = vh.masked_fill(~mask[:, None, :, None], 0.0)  # never touch unwritten cache slots
    p = torch.softmax(s, -1)
    p = torch.nan_to_num(p, nan=0.0)
    return torch.einsum("bhk,bhkd->bhd", p, vh).reshape(B, Hq * D).to(q.dtype)


def logprob(logits, targets=None, inv_temp=1.0):
    """Returns (logp [T], entropy [T], lse [T], E[x'] [T]) of the tempered distribution."""
    x = logits.float() * inv_temp
    lse = torch.logsumexp(x, -1)
    p = torch.exp(x - lse[:, None])
    ex = (p * x).sum(-1)
    ent = lse - ex
    if targets is not None:
        t = targets.long()
        valid = t >= 0
        lp = x.gather(1, t.clamp(min=0)[:, None])[:, 0] - lse
        lp = torch.where(valid, lp, torch.zeros_like(lp))
    else:
        lp = torch.zeros_like(lse)
    return lp, ent, lse, ex


def filter_logits(logits, inv_temp=1.0, top_k=0, top_p=1.0):
    """Boolean keep-mask matching the sampler's top-k / top-p thresholds (ties kept)."""
    x = logits.float()
    keep = torch.ones_like(x, dtype=torch.bool)
    V = x.shape[-1]
    if 0 < top_k < V:
        kth = torch.topk(x, top_k, dim=-1).values[:, -1:]
        keep &= x >= kth
    if top_p < 1.0:
        xs = x * inv_temp
        m = xs.max(-1, keepdim=True).values
        w = torch.exp(xs - m) * keep
        sk = w.sum(-1, keepdim=True)
        order = torch.argsort(x, dim=-1, descending=True)
        ws = w.gather(-1, order)
        cum_before = torch.cumsum(ws, -1) - ws
        thr_pos = (cum_before < top_p * sk).sum(-1, keepdim=True) - 1  # last index needed
        thr_val = x.gather(-1, order).gather(-1, thr_pos.clamp(min=0))
        keep &= x >= thr_val
    return keep


def sample(logits, inv_temp=1.0, top_k=0, top_p=1.0, greedy=False, generator=None):
    x = logits.float() * inv_temp
    lse = torch.logsumexp(x, -1)
    if greedy:
        tok = x.argmax(-1)
    else:
        keep = filter_logits(logits, inv_temp, top_k, top_p)
        xm = x.masked_fill(~keep, float("-inf"))
        probs = torch.softmax(xm, -1)
        tok = torch.multinomial(probs, 1, generator=generator)[:, 0]
    return tok, x.gather(1, tok[:, None])[:, 0] - lse


def pool_norm(x, lengths=None, normalize=True):
    B, S, H = x.shape
    xf = x.float()
    if lengths is None:
        m = xf.mean(1)
    else:
        mask = (torch.arange(S, device=x.device)[None, :] < lengths.long()[:, None]).float()
        m = (xf * mask[..., None]).sum(1) / mask.sum(1).clamp(min=1)[:, None]
    return F.normalize(m, dim=-1, eps=1e-12) if normalize else m


def topk(scores, k, idmap=None):
    v, i = torch.topk(scores.float(), k, dim=-1)
    if idmap is not None:
        i = idmap.gather(1, i)
    return v, i


def gae(rewards, values, mask, gamma, lam):
    B, T = rewards.shape
    adv = torch.zeros_like(rewards)
    ret = torch.zeros_like(rewards)
    nextv = torch.zeros(B, device=rewards.device)
    last = torch.zeros(B, device=rewards.device)
    for t in range(T - 1, -1, -1):
        m = mask[:, t] > 0
        delta = rewards[:, t] + gamma * nextv - values[:, t]
        new_last = delta + gamma * lam * last
        adv[:, t] = torch.where(m, new_last, torch.zeros_like(new_last))
        ret[:, t] = torch.where(m, new_last + values[:, t], torch.zeros_like(new_last))
        last = torch.where(m, new_last, last)
        nextv = torch.where(m, values[:, t], nextv)
    return adv, ret


def ppo_loss(lp, old, adv, vals, ret, ent, mask, eps, c_v, c_e, vclip=None, vold=None, ref_lp=None, kl_coef=0.0):
    """Token-level PPO objective (eager oracle of the fused kernel): returns (loss, stats[9]) with
    stats = loss, policy_loss, value_loss, entropy, approx_kl, clipfrac, kl_ref_k3, kl_ref_k1,
    n_tokens; ``ref_lp``: + kl_coef * mean(exp(ref - lp) - (ref - lp) - 1)."""
    m = mask.to(lp.dtype)
    n = m.sum().clamp(min=1.0)
    ratio = torch.exp(lp - old)
    pg = (-torch.min(ratio * adv, torch.clamp(ratio, 1 - eps, 1 + eps) * adv) * m).sum() / n
    if vclip is not None and vclip > 0:
        vc = vold + torch.clamp(vals - vold, -vclip, vclip)
        vl = 0.5 * (torch.max((vals - ret) ** 2, (vc - ret) ** 2) * m).sum() / n
    else:
        vl = 0.5 * (((vals - ret) ** 2) * m).sum() / n
    em = (ent * m).sum() / n
    loss = pg + c_v * vl - c_e * em
    zero = lp.new_zeros(())
    k3 = k1 = zero
    if ref_lp is not None:
        d = ref_lp - lp
        k3 = ((torch.exp(d) - d - 1) * m).sum() / n
        k1 = (-d * m).sum() / n
        if kl_coef:
            loss = loss + kl_coef * k3
    with torch.no_grad():
        kl = ((old - lp) * m).sum() / n
        cf = ((((ratio - 1).abs() > eps).to(lp.dtype)) * m).sum() / n
        stats = torch.stack([loss.detach(), pg.detach(), vl.detach(), em.detach(), kl, cf, k3.detach(), k1.detach(),
                             m.sum()])
    return loss, stats


def adamw_(p, g, m, v, lr, b1, b2, eps, wd, step, max_norm=0.0):
    """In-place torch.optim.AdamW semantics with global-norm clipping; returns (norm, skipped)."""
    norm = g.float().norm()
    if not torch.isfinite(norm):
        return norm, True
    clip = min(1.0, max_norm / (float(norm) + 1e-6)) if max_norm > 0 else 1.0
    gr = g * clip
    m.mul_(b1).add_(gr, alpha=1 - b1)
    v.mul_(b2).addcmul_(gr, gr, value=1 - b2)
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    p.mul_(1 - lr * wd)
    denom = (v / bc2).sqrt().add_(eps)
    p.addcdiv_(m, denom, value=-lr / bc1)
    return norm, False


def segment_mean(x, order, seg, normalize: bool, out):
    """fp32 oracle of the segment_mean kernel: out[c] = mean(x[order[seg[c]:seg[c+1]]]) (+ L2 norm);
    rows of empty segments are left as they are."""
    k = seg.numel() - 1
    cnt = (seg[1:] - seg[:-1]).long()
    lab = torch.repeat_interleave(torch.arange(k, device=x.device), cnt)
    sums = torch.zeros(k, x.shape[1], device=x.device).index_add_(0, lab, x[order.long()].float())
    m = sums / cnt.clamp(min=1)[:, None]
    if normalize:
        m = torch.nn.functional.normalize(m, dim=-1)
    nz = cnt > 0
    out[nz] = m[nz].to(out.dtype)
    return out


def ppo_advantages(old_logp, ref_logp, values, scores, resp_len, kl_coef, gamma, lam, whiten=True, eps=1e-8):
    """fp32 oracle of the ppo_advantages kernel (the eager token-reward + GAE + whitening path)."""
    B, T = old_logp.shape
    mask = torch.arange(T, device=old_logp.device)[None, :] < resp_len.long()[:, None]
    kl = (old_logp - ref_logp) * mask
    rewards = -kl_coef * kl
    last = (resp_len.long() - 1).clamp(min=0)
    rewards[torch.arange(B, device=old_logp.device), last] += scores
    rewards = rewards * mask
    adv, ret = gae(rewards, values * mask, mask.float(), gamma, lam)
    if whiten:
        m = mask.float()
        n = m.sum().clamp(min=1)
        mean = (adv * m).sum() / n
        var = (((adv - mean) ** 2) * m).sum() / n
        adv = (adv - mean) * torch.rsqrt(var + eps) * m
    return adv, ret, rewards, kl.sum(-1)
