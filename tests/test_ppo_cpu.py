"""End-to-end PPO step on CPU with tiny random-init models (config-4 plumbing)."""
import math
import os

import torch

from rag_tl_domainllm_optimizer_amd import models
from rag_tl_domainllm_optimizer_amd.data import RecordLoader, SyntheticCorpus
from rag_tl_domainllm_optimizer_amd.models.config import PRESETS
from rag_tl_domainllm_optimizer_amd.retrieval import Encoder
from rag_tl_domainllm_optimizer_amd.rewards import RewardModel
from rag_tl_domainllm_optimizer_amd.tokenizer import Tokenizer
from rag_tl_domainllm_optimizer_amd.train.ppo import PPOConfig, PPOTrainer

REF_KEYS = ["reward_mean", "reward_std", "factual_accuracy", "relevance", "conciseness", "policy_loss",
            "value_loss", "entropy_loss", "total_loss", "approx_kl"]


def _setup(tmp_path=None, seed=0):
    torch.manual_seed(seed)
    cfg = PRESETS["tiny-llama"]
    tok = Tokenizer.synthetic(cfg.vocab_size, "llama")
    policy = models.CausalLM(cfg, dtype=torch.float32, seed=1)
    enc_cfg = PRESETS["tiny-bert"]
    enc = Encoder(models.SentenceEncoder(enc_cfg, dtype=torch.float32, seed=2).eval(),
                  Tokenizer.synthetic(enc_cfg.vocab_size, "bert"), max_length=64)
    corpus = SyntheticCorpus(tok.words(), n_docs=40, doc_words=20, seed=3)
    items = corpus.sample_queries(16)
    recs = [{"query": it.query, "retrieved_docs": [corpus.docs[it.gold_doc]], "ground_truth": it.ground_truth}
            for it in items]
    pc = PPOConfig(max_new_tokens=8, max_prompt_tokens=64, minibatch_size=4, lora_r=4, lora_alpha=8.0, lr=1e-3,
                   rollout_chunks=2)
    tr = PPOTrainer(policy, tok, RewardModel(enc), pc, max_batch=8)
    return tr, recs


def test_ppo_step_runs_and_updates(tmp_path):
    tr, recs = _setup()
    before = [p.detach().clone() for p in tr.policy.lora_parameters()]
    loader = RecordLoader(recs, batch_size=8, seed=0)
    m = tr.step(next(iter(loader)))
    for k in REF_KEYS + ["kl_ref", "rollout_tokens_per_s", "grad_norm"]:
        assert k in m and math.isfinite(m[k]), k
    after = list(tr.policy.lora_parameters())
    assert any(not torch.equal(a, b) for a, b in zip(before, after)), "LoRA parameters did not move"
    # behaviour policy == policy before the first minibatch; later minibatches drift only slightly
    assert abs(m["approx_kl"]) < 0.05
    tr.save_checkpoint(str(tmp_path / "ck" / "best_model"))
    for suf in ("_policy", "_tokenizer", "_adapter", "_trainer_state"):
        assert os.path.isdir(str(tmp_path / "ck" / "best_model") + suf), suf
    vh = torch.load(str(tmp_path / "ck" / "best_model") + "_value_head.pt", weights_only=True)
    assert vh["weight"].shape == (1, tr.policy.cfg.hidden_size) and vh["bias"].shape == (1,)


def test_ppo_resume_reproduces_next_step(tmp_path):
    tr, recs = _setup(seed=0)
    loader = RecordLoader(recs, batch_size=8, seed=0)
    batches = list(loader)
    tr.step(batches[0])
    tr.save_checkpoint(str(tmp_path / "r" / "s1"), full_policy=False)
    m_a = tr.step(batches[1])
    params_a = [p.detach().clone() for p in tr.policy.lora_parameters()]
    tr2, _ = _setup(seed=0)
    tr2.load_checkpoint(str(tmp_path / "r" / "s1"))
    m_b = tr2.step(batches[1])
    params_b = list(tr2.policy.lora_parameters())
    for a, b in zip(params_a, params_b):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    assert abs(m_a["total_loss"] - m_b["total_loss"]) < 1e-5


def test_ppo_deterministic_across_runs():
    """Same seeds -> identical rollouts, rewards and losses in two independent runs."""
    outs = []
    for _ in range(2):
        tr, recs = _setup(seed=0)
        loader = RecordLoader(recs, batch_size=8, seed=0)
        b = next(iter(loader))
        m = tr.step(b)
        outs.append((m, [p.detach().clone() for p in tr.policy.lora_parameters()]))
    (m1, p1), (m2, p2) = outs
    for k in REF_KEYS + ["kl_ref"]:
        assert m1[k] == m2[k], (k, m1[k], m2[k])
    assert all(torch.equal(a, b) for a, b in zip(p1, p2))


def test_fault_injection_then_resume_matches(tmp_path, monkeypatch):
    """RAGTL_FAULT_AT_STEP raises mid-run; resuming from the last checkpoint reproduces the
    uninterrupted run's next step."""
    import pytest

    tr, recs = _setup(seed=0)
    batches = list(RecordLoader(recs, batch_size=8, seed=0))
    tr.step(batches[0])
    ck = str(tmp_path / "f" / "s1")
    tr.save_checkpoint(ck, full_policy=False)
    ref = tr.step(batches[1])
    tr2, _ = _setup(seed=0)
    tr2.load_checkpoint(ck)
    monkeypatch.setenv("RAGTL_FAULT_AT_STEP", str(tr2.global_step))
    with pytest.raises(RuntimeError):
        tr2.step(batches[1])
    monkeypatch.delenv("RAGTL_FAULT_AT_STEP")
    tr3, _ = _setup(seed=0)
    tr3.load_checkpoint(ck)
    got = tr3.step(batches[1])
    for k in ("reward_mean", "total_loss", "policy_loss", "kl_ref"):
        assert abs(got[k] - ref[k]) < 1e-6, (k, got[k], ref[k])


def test_ppo_advantages_oracle_matches_eager_path():
    """ops.ppo_advantages (CPU oracle) == the eager token-reward + GAE + whitening composition."""
    import torch

    from rag_tl_domainllm_optimizer_amd import ops
    from rag_tl_domainllm_optimizer_amd.train.common import masked_whiten, response_mask

    g = torch.Generator().manual_seed(0)
    B, T = 6, 9
    old, refl, vals = (torch.randn(B, T, generator=g) for _ in range(3))
    scores = torch.randn(B, generator=g)
    lens = torch.tensor([9, 1, 0, 5, 8, 3])
    mask = response_mask(lens, T)
    kl = (old - refl) * mask
    rew = -0.1 * kl
    last = (lens - 1).clamp(min=0)
    rew[torch.arange(B), last] += scores
    rew = rew * mask
    adv, ret = ops.gae(rew, vals * mask, mask.float(), 0.99, 0.95)
    adv = masked_whiten(adv, mask)
    a2, r2, w2, k2 = ops.ppo_advantages(old, refl, vals, scores, lens, 0.1, 0.99, 0.95, True)
    torch.testing.assert_close(a2, adv, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(r2, ret)
    torch.testing.assert_close(w2, rew)
    torch.testing.assert_close(k2, kl.sum(-1))


def test_ppo_old_logp_recompute_ratio_is_one_at_theta_old():
    """old_logp = "recompute": the ratio's theta_old log-probs come from a training-numerics forward
    (LoRA on, unmerged), so the first minibatch scores exactly theta_old: no gap, nothing clipped.
    The rollout engine's own deviation is still reported (rollout_engine_logp_gap)."""
    import dataclasses

    tr, recs = _setup()
    tr.cfg = dataclasses.replace(tr.cfg, old_logp="recompute")
    loader = RecordLoader(recs, batch_size=8, seed=0)
    for _ in range(2):  # the second step runs with trained (non-zero) adapters
        m = tr.step(next(iter(loader)))
        assert m["behaviour_logp_gap"] < 1e-5, m["behaviour_logp_gap"]
        assert m["clipfrac_first_mb"] == 0.0
        assert math.isfinite(m["rollout_engine_logp_gap"]) and m["rollout_engine_logp_gap"] >= 0.0


def test_kl_in_loss_exact_zero_at_init_and_oracle():
    """The reference KL in the loss (PPOConfig.kl_in_loss): at LoRA B = 0 the policy IS the reference,
    so the first minibatch's KL at theta_old is 0 (up to the CPU GEMMs' batch-size-dependent
    blocking; exactly 0 on the GPU, tests/test_batch_invariance_gpu.py; the sampler-based sum
    (old - ref) is reported apart); the loss oracle adds kl_coef * mean(exp(d) - d - 1), d = ref - lp, whose
    gradient is kl_coef * (1 - exp(d)) / n per masked token."""
    from rag_tl_domainllm_optimizer_amd.ops import reference as ref

    tr, recs = _setup(seed=4)
    assert tr.cfg.kl_in_loss
    m = tr.step(next(iter(RecordLoader(recs, batch_size=8, seed=1))))
    assert abs(m["kl_ref_theta_old"]) < 1e-5
    assert m["kl_ref_k3"] >= 0.0 and math.isfinite(m["kl_old_ref"])
    torch.manual_seed(0)
    B, T, beta = 3, 7, 0.05
    lp = (torch.randn(B, T) * 0.3 - 2).requires_grad_(True)
    refl = lp.detach() + torch.randn(B, T) * 0.2
    z = torch.zeros(B, T)
    mask = torch.ones(B, T)
    mask[0, 5:] = 0
    loss0, st0 = ref.ppo_loss(lp, lp.detach(), z, z, z, z, mask, 0.2, 0.5, 0.0)
    loss1, st1 = ref.ppo_loss(lp, lp.detach(), z, z, z, z, mask, 0.2, 0.5, 0.0, None, None, refl, beta)
    d = refl - lp.detach()
    n = mask.sum()
    k3 = ((torch.exp(d) - d - 1) * mask).sum() / n
    torch.testing.assert_close(loss1 - loss0, beta * k3)
    torch.testing.assert_close(st1[6], k3)
    torch.testing.assert_close(st1[7], ((-d) * mask).sum() / n)
    (g,) = torch.autograd.grad(loss1 - loss0, lp)
    torch.testing.assert_close(g, beta * (1 - torch.exp(d)) * mask / n)
