"""Full-parameter fine-tuning — the reference's mode (AdamW over every policy weight and the value
head, reinforcement_learning_optimization_after_rag.py:153-156,228-232) — on CPU tensors:
MixedFlatParams + FusedAdamW == torch.optim.AdamW + clip_grad_norm_ on fp32 masters, the bf16
compute copies follow the masters, and a full-FT PPO step trains every weight against a frozen
reference copy."""
import math

import torch

from rag_tl_domainllm_optimizer_amd import ops


def _mixed_params():
    g = torch.Generator().manual_seed(0)
    w16 = [torch.nn.Parameter(torch.randn(37, 8, generator=g).to(torch.bfloat16)),
           torch.nn.Parameter(torch.randn(5, generator=g).to(torch.bfloat16))]
    w32 = [torch.nn.Parameter(torch.randn(3, 4, generator=g))]
    return w16, w32


def test_mixed_flat_layout_and_slices():
    w16, w32 = _mixed_params()
    flat = ops.flat_params(w32 + w16)
    assert isinstance(flat, ops.MixedFlatParams)
    # bf16 members first (one contiguous bf16 segment), fp32 members after it
    assert all(p is q for p, q in zip(flat.params, w16 + w32))
    assert flat.n16 % 16 == 0 and flat.numel == flat.n16 + flat.grad32.numel()
    for p, o in zip(flat.params, flat.offsets):
        n = p.numel()
        buf = flat.data16 if p.dtype == torch.bfloat16 else flat.data
        assert p.data_ptr() == buf[o:o + n].data_ptr()
        torch.testing.assert_close(flat.data[o:o + n].view(p.shape), p.detach().float())
    sl = flat.grad_slices(0, flat.numel)
    assert [t.dtype for t in sl] == [torch.bfloat16, torch.float32]
    assert sum(t.numel() for t in sl) == flat.numel
    assert len(flat.grad_slices(0, flat.n16)) == 1 and len(flat.grad_slices(flat.n16, flat.numel)) == 1
    assert isinstance(ops.flat_params(w32), ops.FlatParams)


def test_mixed_adamw_matches_torch_on_masters():
    w16, w32 = _mixed_params()
    members = w16 + w32
    masters = [p.detach().float().clone().requires_grad_(True) for p in members]
    flat = ops.MixedFlatParams(members)
    opt = ops.FusedAdamW(flat, lr=1e-2, weight_decay=0.01, max_grad_norm=0.5)
    topt = torch.optim.AdamW(masters, lr=1e-2, weight_decay=0.01)
    g = torch.Generator().manual_seed(1)
    for _ in range(3):
        grads = [torch.randn(p.shape, generator=g) for p in members]
        opt.zero_grad()
        for p, gr in zip(members, grads):
            p.grad.copy_(gr)
        opt.step()
        for m, p, gr in zip(masters, members, grads):
            m.grad = gr.to(p.dtype).float()  # the optimizer sees the bf16-rounded gradient
        torch.nn.utils.clip_grad_norm_(masters, 0.5)
        topt.step()
    for m, p, o in zip(masters, flat.params, flat.offsets):
        master = flat.data[o:o + p.numel()].view(p.shape)
        torch.testing.assert_close(master, m.detach(), rtol=1e-5, atol=1e-6)
        assert torch.equal(p.detach(), master.to(p.dtype))
    # a non-finite gradient skips the step
    before = flat.data.clone()
    opt.zero_grad()
    w16[0].grad[0, 0] = float("nan")
    opt.step()
    assert torch.equal(before, flat.data) and int(opt.skipped) == 1


def test_ppo_full_finetune_cpu():
    from rag_tl_domainllm_optimizer_amd import models
    from rag_tl_domainllm_optimizer_amd.data import RecordLoader, SyntheticCorpus
    from rag_tl_domainllm_optimizer_amd.models.config import PRESETS
    from rag_tl_domainllm_optimizer_amd.retrieval import Encoder
    from rag_tl_domainllm_optimizer_amd.rewards import RewardModel
    from rag_tl_domainllm_optimizer_amd.tokenizer import Tokenizer
    from rag_tl_domainllm_optimizer_amd.train.ppo import PPOConfig, PPOTrainer

    torch.manual_seed(0)
    cfg = PRESETS["tiny-llama"]
    tok = Tokenizer.synthetic(cfg.vocab_size, "llama")
    policy = models.CausalLM(cfg, dtype=torch.float32, seed=1)
    ecfg = PRESETS["tiny-bert"]
    enc = Encoder(models.SentenceEncoder(ecfg, dtype=torch.float32, seed=2).eval(),
                  Tokenizer.synthetic(ecfg.vocab_size, "bert"), max_length=64)
    corpus = SyntheticCorpus(tok.words(), n_docs=40, doc_words=20, seed=3)
    recs = [{"query": it.query, "retrieved_docs": [corpus.docs[it.gold_doc]], "ground_truth": it.ground_truth}
            for it in corpus.sample_queries(8)]
    before = {n: p.detach().clone() for n, p in policy.named_parameters()}
    tr = PPOTrainer(policy, tok, RewardModel(enc), PPOConfig(full_finetune=True, max_new_tokens=8,
                                                             max_prompt_tokens=64, minibatch_size=4, lr=1e-3),
                    max_batch=8)
    assert getattr(policy, "lora_config", None) is None and tr.ref_policy is not policy
    batch = next(iter(RecordLoader(recs, batch_size=8, seed=0)))
    m1 = tr.step(batch)
    m2 = tr.step(batch)
    for m in (m1, m2):
        for k in ("reward_mean", "total_loss", "policy_loss", "value_loss", "kl_ref", "grad_norm"):
            assert math.isfinite(m[k]), k
    for n, p in policy.named_parameters():
        assert not torch.equal(p.detach(), before[n]), f"{n} did not train"
    for n, p in tr.ref_policy.named_parameters():
        assert torch.equal(p, before[n]) and not p.requires_grad, n
    assert m2["kl_ref"] != 0.0


def _fullft_kl(lr, steps=2):
    from rag_tl_domainllm_optimizer_amd import models
    from rag_tl_domainllm_optimizer_amd.data import RecordLoader, SyntheticCorpus
    from rag_tl_domainllm_optimizer_amd.models.config import PRESETS
    from rag_tl_domainllm_optimizer_amd.retrieval import Encoder
    from rag_tl_domainllm_optimizer_amd.rewards import RewardModel
    from rag_tl_domainllm_optimizer_amd.tokenizer import Tokenizer
    from rag_tl_domainllm_optimizer_amd.train.ppo import PPOConfig, PPOTrainer

    torch.manual_seed(0)
    cfg = PRESETS["tiny-llama"]
    tok = Tokenizer.synthetic(cfg.vocab_size, "llama")
    policy = models.CausalLM(cfg, dtype=torch.float32, seed=1)
    ecfg = PRESETS["tiny-bert"]
    enc = Encoder(models.SentenceEncoder(ecfg, dtype=torch.float32, seed=2).eval(),
                  Tokenizer.synthetic(ecfg.vocab_size, "bert"), max_length=64)
    corpus = SyntheticCorpus(tok.words(), n_docs=40, doc_words=20, seed=3)
    recs = [{"query": it.query, "retrieved_docs": [corpus.docs[it.gold_doc]], "ground_truth": it.ground_truth}
            for it in corpus.sample_queries(8)]
    tr = PPOTrainer(policy, tok, RewardModel(enc), PPOConfig(full_finetune=True, max_new_tokens=8,
                                                             max_prompt_tokens=64, minibatch_size=4, lr=lr),
                    max_batch=8)
    batch = next(iter(RecordLoader(recs, batch_size=8, seed=0)))
    return [tr.step(batch) for _ in range(steps)]


def test_full_finetune_kl_and_ratio_at_theta_old():
    """Full-parameter PPO (the reference's mode): (1) the first minibatch scores the rollouts at
    theta = theta_old, so |logp - old_logp| is numerics only and nothing clips; (2) the frozen-
    reference KL after one update grows with the learning rate (0.035 -> 0.37 nats per 8-token
    sequence for lr 5e-6 -> 5e-5 on this tiny model) — AdamW's first steps
    move EVERY weight by ~lr whatever its gradient's size, so on a random-init model at the
    reference's lr 5e-5 the per-sequence KL is large (docs/DESIGN.md 'Round 5': the bench's
    full-FT kl_ref of ~500 nats / 128-token sequence is this effect, not a bug in MixedFlatParams)."""
    lo = _fullft_kl(5e-6)
    hi = _fullft_kl(5e-5)
    for ms in (lo, hi):
        for m in ms:
            assert m["behaviour_logp_gap"] < 1e-4, m["behaviour_logp_gap"]
            assert m["clipfrac_first_mb"] == 0.0
        assert abs(ms[0]["kl_ref_theta_old"]) < 1e-4  # no update yet: policy == reference
    assert hi[1]["kl_ref"] > 5 * lo[1]["kl_ref"] > 0
