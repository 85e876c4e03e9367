"""Full-parameter training on the MI355X (the reference's mode, rl.py:153-156,228-232): the
mixed-precision fused AdamW kernel (bf16 gradients and compute copy, fp32 master and moments)
against torch.optim.AdamW on fp32 masters; full-FT PPO and SFT steps of a bf16 policy."""
import math

import pytest
import torch

from rag_tl_domainllm_optimizer_amd import models, ops
from rag_tl_domainllm_optimizer_amd.models.config import PRESETS

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_adamw_mixed_kernel_matches_torch():
    torch.manual_seed(0)
    w16 = [torch.nn.Parameter(torch.randn(1000, 24, device=DEV).to(torch.bfloat16)),
           torch.nn.Parameter(torch.randn(333, device=DEV).to(torch.bfloat16))]
    w32 = [torch.nn.Parameter(torch.randn(17, device=DEV))]
    members = w16 + w32
    masters = [p.detach().float().clone().requires_grad_(True) for p in members]
    flat = ops.MixedFlatParams(members)
    opt = ops.FusedAdamW(flat, lr=1e-2, weight_decay=0.01, max_grad_norm=0.5)
    topt = torch.optim.AdamW(masters, lr=1e-2, weight_decay=0.01)
    for _ in range(3):
        grads = [torch.randn(p.shape, device=DEV) for p in members]
        opt.zero_grad()
        for p, g in zip(members, grads):
            p.grad.copy_(g)
        opt.step()
        for m, p, g in zip(masters, members, grads):
            m.grad = g.to(p.dtype).float()
        torch.nn.utils.clip_grad_norm_(masters, 0.5)
        topt.step()
    torch.cuda.synchronize()
    for m, p, o in zip(masters, flat.params, flat.offsets):
        master = flat.data[o:o + p.numel()].view(p.shape)
        torch.testing.assert_close(master, m.detach(), rtol=1e-4, atol=1e-5)
        assert torch.equal(p.detach(), master.to(p.dtype))
    # a non-finite bf16 gradient skips the whole step (master, moments and compute copy unchanged)
    before, before16 = flat.data.clone(), flat.data16.clone()
    opt.zero_grad()
    w16[1].grad[3] = float("inf")
    opt.step()
    torch.cuda.synchronize()
    assert torch.equal(before, flat.data) and torch.equal(before16, flat.data16) and int(opt.skipped) == 1


def _stack(seed):
    from rag_tl_domainllm_optimizer_amd.data import SyntheticCorpus
    from rag_tl_domainllm_optimizer_amd.retrieval import Encoder
    from rag_tl_domainllm_optimizer_amd.tokenizer import Tokenizer

    cfg = PRESETS["tiny-mistral"]
    tok = Tokenizer.synthetic(cfg.vocab_size, "mistral")
    pol = models.CausalLM(cfg, device=DEV, dtype=torch.bfloat16, seed=seed)
    ecfg = PRESETS["tiny-bert"]
    enc = Encoder(models.SentenceEncoder(ecfg, device=DEV, dtype=torch.bfloat16, seed=seed + 1).eval(),
                  Tokenizer.synthetic(ecfg.vocab_size, "bert"), max_length=64)
    corpus = SyntheticCorpus(tok.words(), n_docs=32, doc_words=16, seed=seed + 2)
    return pol, tok, enc, corpus


def test_ppo_full_finetune_gpu():
    from rag_tl_domainllm_optimizer_amd.generation import Generator, SamplingParams
    from rag_tl_domainllm_optimizer_amd.rewards import RewardModel
    from rag_tl_domainllm_optimizer_amd.train.common import score_sequences
    from rag_tl_domainllm_optimizer_amd.train.ppo import PPOConfig, PPOTrainer

    pol, tok, enc, corpus = _stack(3)
    items = corpus.sample_queries(8, seed=6)
    batch = {"query": [i.query for i in items], "retrieved_docs": [[corpus.docs[i.gold_doc]] for i in items],
             "ground_truth": [i.ground_truth for i in items]}
    names = {id(p): n for n, p in pol.named_parameters()}
    before = {n: p.detach().clone() for n, p in pol.named_parameters()}
    tr = PPOTrainer(pol, tok, RewardModel(enc), PPOConfig(full_finetune=True, max_new_tokens=6, max_prompt_tokens=96,
                                                          minibatch_size=4, lr=1e-3), max_batch=8)
    assert isinstance(tr.flat, ops.MixedFlatParams) and tr.ref_policy is not None
    m1 = tr.step(batch)
    m2 = tr.step(batch)
    for m in (m1, m2):
        for k in ("reward_mean", "total_loss", "kl_ref", "grad_norm"):
            assert math.isfinite(m[k]), k
    for p, o in zip(tr.flat.params, tr.flat.offsets):
        if id(p) in names:  # every fp32 master moved
            n = names[id(p)]
            assert not torch.equal(tr.flat.data[o:o + p.numel()].view(p.shape), before[n].float()), n
    assert not torch.equal(pol.layers[0].qkv_w.detach(), before["layers.0.qkv_w"])
    for n, p in tr.ref_policy.named_parameters():
        assert torch.equal(p, before[n]), n
    assert m2["kl_ref"] != 0.0
    # decoding after the updates reads the updated weights (graph replay + norm-folded batch-<=16
    # decode images rebuilt from the bumped version counters)
    prompts = [[5, 9, 33, 41, 7, 8, 9, 10], [12, 300, 4]]
    out = Generator(pol, 2, 64, DEV).generate(prompts, SamplingParams(max_new_tokens=8, temperature=0.7, top_k=0,
                                                                      seed=5), pad_id=0, eos_ids=[-1])
    with torch.no_grad():
        lp, _, _, _ = score_sequences(pol, out.prompt_ids, out.prompt_start, out.tokens, out.lengths, 1 / 0.7)
    torch.testing.assert_close(lp, out.logprobs, rtol=0.0, atol=0.08)


def test_sft_full_finetune_gpu():
    from rag_tl_domainllm_optimizer_amd.train import SFTConfig, SFTTrainer, build_raft_examples

    pol, tok, _, corpus = _stack(7)
    ex = build_raft_examples([{"query": i.query, "ground_truth": i.ground_truth, "gold_doc": i.gold_doc}
                              for i in corpus.sample_queries(8, seed=9)], corpus.docs)
    tr = SFTTrainer(pol, tok, SFTConfig(full_finetune=True, batch_size=8, lr=1e-3, warmup_steps=0,
                                        lr_schedule="constant", max_seq=160))
    assert isinstance(tr.flat, ops.MixedFlatParams) and pol.embed.dtype == torch.bfloat16
    losses = [tr.step(ex)["loss"] for _ in range(6)]
    assert all(math.isfinite(x) for x in losses) and losses[-1] < losses[0], losses
