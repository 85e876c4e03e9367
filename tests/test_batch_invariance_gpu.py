"""Batch-invariant PPO scoring on the MI355X kernels: a rollout's per-token
log-probs, entropies and values come out bitwise the same whatever rows share the scoring forward
(minibatch 32 / 128 subsets, padded or packed, grad or no grad), so

* ``old_logp="recompute"`` gives a PPO ratio of exactly 1 on the first minibatch (gap 0, clip 0);
* the in-loss reference KL is exactly 0 at LoRA B = 0 (policy == reference);

and the value head / fused loss pieces this relies on match their fp32 oracles."""
import numpy as np
import pytest
import torch

from rag_tl_domainllm_optimizer_amd import models, ops
from rag_tl_domainllm_optimizer_amd.models import ValueHead
from rag_tl_domainllm_optimizer_amd.models.config import PRESETS
from rag_tl_domainllm_optimizer_amd.train.common import score_sequences

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def test_row_dot_value_head():
    """ops.row_dot == the fp32 row dot; a row's value is bitwise independent of the launch's rows."""
    torch.manual_seed(0)
    for T, H in ((1, 4096), (37, 4096), (1000, 256), (5, 264)):
        h = torch.randn(T, H, device=DEV).to(torch.bfloat16)
        w = torch.randn(H, device=DEV)
        b = torch.randn(1, device=DEV)
        y = ops.row_dot(h, w, b)
        torch.testing.assert_close(y, (h.float() * w).sum(-1) + b, rtol=1e-5, atol=1e-4)
        if T > 3:
            assert torch.equal(ops.row_dot(h[1:3], w, b), y[1:3])
    # autograd: dh, dw, db == the eager expression's
    h = torch.randn(64, 256, device=DEV).to(torch.bfloat16).requires_grad_(True)
    w = torch.randn(256, device=DEV, requires_grad=True)
    b = torch.zeros(1, device=DEV, requires_grad=True)
    g = torch.randn(64, device=DEV)
    (ops.row_dot(h, w, b) * g).sum().backward()
    grads = [t.grad.clone() for t in (h, w, b)]
    for t in (h, w, b):
        t.grad = None
    (((h.float() * w).sum(-1) + b) * g).sum().backward()
    torch.testing.assert_close(grads[0].float(), h.grad.float(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(grads[1], w.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(grads[2], b.grad, rtol=1e-5, atol=1e-4)


def _model(seed=11, lora_std=0.02):
    cfg = PRESETS["tiny-mistral"]
    m = models.CausalLM(cfg, device=DEV, dtype=torch.bfloat16, seed=seed)
    m.add_lora(8, 16.0, None, seed=2)
    if lora_std:
        with torch.no_grad():
            for p in m.lora_parameters():
                p.normal_(0, lora_std)
    m.refresh_lora()
    return m, ValueHead(cfg.hidden_size, device=DEV, seed=3)


def _batch(B, S, T, V, seed=0):
    g = np.random.default_rng(seed)
    st = g.integers(0, S - 4, B)
    rl = g.integers(1, T + 1, B)
    pid = torch.from_numpy(g.integers(5, V, (B, S)))
    resp = torch.from_numpy(g.integers(5, V, (B, T)))
    for b in range(B):
        pid[b, :st[b]] = 0
        resp[b, rl[b]:] = 0
    return pid.to(DEV), torch.tensor(st, dtype=torch.int32, device=DEV), resp.to(DEV), \
        torch.tensor(rl, device=DEV), st, rl


def _score(m, vh, pid, start, resp, rlen, lengths, grad=False):
    with torch.set_grad_enabled(grad):
        lp, ent, val, mask = score_sequences(m, pid, start, resp, rlen, 1 / 0.7, vh, lengths=lengths)
    return lp.detach(), ent.detach(), val.detach(), mask


@pytest.mark.parametrize("B,S,T", [(8, 96, 32), (24, 64, 40)])
def test_score_sequences_bitwise_across_batches(B, S, T):
    """Per-row outputs of the scoring forward are bitwise equal for: the whole batch vs row subsets
    of different sizes (minibatch 32 vs 128 in the bench), padded vs packed, grad vs no grad."""
    m, vh = _model()
    pid, start, resp, rlen, st, rl = _batch(B, S, T, m.cfg.vocab_size)
    full = _score(m, vh, pid, start, resp, rlen, (st, rl))
    mask = full[3]
    variants = {"padded": _score(m, vh, pid, start, resp, rlen, None),
                "grad": _score(m, vh, pid, start, resp, rlen, (st, rl), grad=True)}
    for name, out in variants.items():
        for a, b in zip(full[:3], out[:3]):
            assert torch.equal(a * mask, b * mask), name
    perm = torch.randperm(B, generator=torch.Generator().manual_seed(1)).tolist()
    for size in (1, 3, B // 2):
        for lo in range(0, B, size):
            rows = perm[lo:lo + size]
            idx = torch.tensor(rows, device=DEV)
            sub = _score(m, vh, pid[idx], start[idx], resp[idx], rlen[idx], (st[rows], rl[rows]), grad=size == 3)
            for a, b in zip(full[:3], sub[:3]):
                assert torch.equal(a[idx] * mask[idx], b * mask[idx]), (size, rows)


def _ppo_trainer(old_logp, kl_in_loss=True, lora_std=0.0, full=False):
    from rag_tl_domainllm_optimizer_amd.data import RecordLoader, SyntheticCorpus
    from rag_tl_domainllm_optimizer_amd.retrieval import Encoder
    from rag_tl_domainllm_optimizer_amd.rewards import RewardModel
    from rag_tl_domainllm_optimizer_amd.tokenizer import Tokenizer
    from rag_tl_domainllm_optimizer_amd.train.ppo import PPOConfig, PPOTrainer

    cfg = PRESETS["tiny-mistral"]
    tok = Tokenizer.synthetic(cfg.vocab_size, "mistral")
    policy = models.CausalLM(cfg, device=DEV, dtype=torch.bfloat16, seed=5)
    ecfg = PRESETS["tiny-bert"]
    enc = Encoder(models.SentenceEncoder(ecfg, device=DEV, dtype=torch.bfloat16, seed=2).eval(),
                  Tokenizer.synthetic(ecfg.vocab_size, "bert"), max_length=64)
    corpus = SyntheticCorpus(tok.words(), n_docs=40, doc_words=20, seed=3)
    recs = [{"query": it.query, "retrieved_docs": [corpus.docs[it.gold_doc]], "ground_truth": it.ground_truth}
            for it in corpus.sample_queries(16)]
    tr = PPOTrainer(policy, tok, RewardModel(enc),
                    PPOConfig(max_new_tokens=12, max_prompt_tokens=64, minibatch_size=4, ref_minibatch_size=16,
                              lr=1e-3, old_logp=old_logp, kl_in_loss=kl_in_loss, lora_r=8, full_finetune=full),
                    max_batch=16)
    if lora_std:
        with torch.no_grad():
            for p in policy.lora_parameters():
                p.normal_(0, lora_std)
        policy.refresh_lora()
    return tr, next(iter(RecordLoader(recs, batch_size=16, seed=0)))


def _ppo(old_logp, kl_in_loss=True, lora_std=0.0, trainer=False, full=False):
    tr, batch = _ppo_trainer(old_logp, kl_in_loss, lora_std, full)
    ms = [tr.step(batch) for _ in range(2)]
    return (ms, tr) if trainer else ms


def _trainable(tr, full):
    ps = [p for p in tr.policy.parameters() if p.requires_grad] if full else list(tr.policy.lora_parameters())
    return [p.detach().clone() for p in ps] + [p.detach().clone() for p in tr.value_head.parameters()]


def test_ppo_recompute_ratio_exactly_one():
    """old_logp="recompute" scores theta_old in the update forward's exact numerics (16-row no-grad
    chunks vs 4-row grad minibatches): the first minibatch's |logp - old_logp| is 0 and nothing clips,
    at every step (adapters away from zero after the first update)."""
    for m in _ppo("recompute", lora_std=0.02):
        assert m["behaviour_logp_gap"] == 0.0, m["behaviour_logp_gap"]
        assert m["clipfrac_first_mb"] == 0.0
        assert m["rollout_engine_logp_gap"] < 0.05


def test_ppo_kl_in_loss_zero_at_init():
    """LoRA B = 0 at the first step: policy == reference in training numerics, so the in-loss KL at
    theta_old is exactly 0 (the sampler-based sum_t (old - ref) is not, and is reported apart); after
    updates the KL is positive."""
    ms = _ppo("rollout", kl_in_loss=True)
    assert ms[0]["kl_ref_theta_old"] == 0.0
    assert ms[0]["kl_ref_k3"] >= 0.0
    assert ms[1]["kl_ref_theta_old"] != 0.0


@pytest.mark.parametrize("full", [False, True])
def test_ppo_steps_bitwise_reproducible(full):
    """Two PPO steps (rollout, reference / reward, GAE, minibatch updates with AdamW) from the same
    seeds end in bitwise-identical trainable weights, value head and metrics: every reduction on the
    path is fixed-order — split-K slabs instead of fp32 atomics in the LoRA forward / backward
    products (the arrival order of atomic partials changed the gradient bits run to run); under
    full fine-tuning also the RMSNorm weight and embedding-table gradients."""
    runs = []
    for _ in range(2):
        torch.manual_seed(0)
        ms, tr = _ppo("rollout", lora_std=0.0 if full else 0.02, trainer=True, full=full)
        runs.append((ms, _trainable(tr, full)))
    (m0, p0), (m1, p1) = runs
    for a, b in zip(p0, p1):
        assert torch.equal(a, b)
    for s0, s1 in zip(m0, m1):
        for k, v in s0.items():
            if "time" in k or "per_s" in k or k.endswith("_s") or not isinstance(v, (int, float)):
                continue
            assert v == s1[k] or (v != v and s1[k] != s1[k]), (k, v, s1[k])


@pytest.mark.parametrize("full", [False, True])
def test_ppo_resume_bitwise(tmp_path, full):
    """Checkpoint after one PPO step, resume in a fresh trainer, take the next step: the weights,
    value head, optimizer-driven update and metrics are bitwise those of the uninterrupted run (the
    checkpoint carries everything the step depends on: adapters / weights, AdamW state, step
    counter, sampler RNG position)."""
    prefix = str(tmp_path / "ck" / "s1")
    torch.manual_seed(0)
    tr, batch = _ppo_trainer("rollout", lora_std=0.0 if full else 0.02, full=full)
    tr.step(batch)
    tr.save_checkpoint(prefix, full_policy=full)
    m_a = tr.step(batch)
    p_a = _trainable(tr, full)
    torch.manual_seed(0)
    tr2, batch2 = _ppo_trainer("rollout", lora_std=0.0 if full else 0.02, full=full)
    tr2.load_checkpoint(prefix)
    m_b = tr2.step(batch2)
    p_b = _trainable(tr2, full)
    assert len(p_a) == len(p_b)
    for a, b in zip(p_a, p_b):
        assert torch.equal(a, b)
    for k, v in m_a.items():
        if "time" in k or "per_s" in k or k.endswith("_s") or not isinstance(v, (int, float)):
            continue
        assert v == m_b[k] or (v != v and m_b[k] != m_b[k]), (k, v, m_b[k])
