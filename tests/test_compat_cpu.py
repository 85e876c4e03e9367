"""Reference-API façade and behavioural spec (Appendix A) on CPU."""
import math
import os

import pytest
import torch

from rag_tl_domainllm_optimizer_amd import compat
from rag_tl_domainllm_optimizer_amd.metrics import bleu, rouge_scores
from rag_tl_domainllm_optimizer_amd.rag.prompt import INSTRUCTION, build_prompt, extract_answer
from rag_tl_domainllm_optimizer_amd.rewards import RewardConfig, conciseness


def test_prompt_template_byte_exact():
    p = build_prompt("What is X?", ["doc one", "doc two"])
    assert p == ("Query: What is X?\n\nContext:\n- doc one\n- doc two\n\n"
                 "Based on the above information, please answer the query concisely and accurately.")
    assert extract_answer(p + " The answer.") == "The answer."
    assert extract_answer("no instruction here") == "no instruction here"


@pytest.mark.parametrize("wc,expected", [(0, 0.5), (19, max(0.5, 19 / 20)), (20, 1.0), (150, 1.0),
                                         (151, 1 - 1 / 150), (300, 0.0), (301, 0.0), (5, 0.5)])
def test_conciseness_breakpoints(wc, expected):
    assert conciseness(wc) == pytest.approx(expected)


def test_gae_reference_formula():
    t = compat.PPOTrainer.__new__(compat.PPOTrainer)
    t.gamma = 0.99
    # dones True -> A = r - V
    assert t.compute_advantages([1.0, 0.5], [0.3, 0.1], [True, True]) == pytest.approx([0.7, 0.4])
    # dones False (SURVEY 4.2 probed values)
    adv = t.compute_advantages([1.0, 0.5, 0.2], [0.3, 0.1, 0.4], [False, False, False])
    assert adv == pytest.approx([1.37073, 0.6079, -0.2], abs=1e-4)


class _FakeEncoder:
    """Deterministic hash -> unit vector encoder (no model): isolates the reward formula."""

    def __init__(self, dim=16):
        self.dim = dim

    def encode(self, texts):
        out = []
        for t in texts:
            g = torch.Generator().manual_seed(abs(hash(t)) % (2 ** 31))
            v = torch.randn(self.dim, generator=g)
            out.append(v / v.norm())
        return torch.stack(out)


def test_reward_formula_matches_reference():
    from rag_tl_domainllm_optimizer_amd.rewards import RewardModel

    rm = RewardModel(_FakeEncoder())
    enc = rm.encoder
    resp, q, docs, gt = "a b c", "query", ["d1", "d2"], "truth"
    r, c = rm.calculate_reward(resp, q, docs, gt)
    e = enc.encode([resp, q, docs[0], docs[1], gt])
    F = max(float(e[0] @ e[2]), float(e[0] @ e[3]))
    Rel = float(e[0] @ e[1])
    C = conciseness(3)
    G = float(e[0] @ e[4])
    expect = 0.7 * (0.5 * F + 0.3 * Rel + 0.2 * C) + 0.3 * G
    assert r == pytest.approx(expect, abs=1e-5)
    assert set(c) == {"factual_accuracy", "relevance", "conciseness", "ground_truth_similarity", "total_reward"}
    r2, c2 = rm.calculate_reward(resp, q, docs, None)
    assert c2["ground_truth_similarity"] is None
    assert r2 == pytest.approx(0.5 * F + 0.3 * Rel + 0.2 * C, abs=1e-5)
    assert rm.calculate_factual_accuracy(resp, []) == 0.0


def test_rouge_bleu():
    r = rouge_scores("the cat sat on the mat", "the cat sat on a mat")
    assert 0 < r["rouge1"] < 1 and r["rougeL"] >= r["rouge2"]
    assert rouge_scores("a b c", "a b c")["rouge1"] == pytest.approx(1.0)
    b = bleu(["the cat sat on the mat today"], [["the cat sat on the mat today"]])
    assert b["bleu"] == pytest.approx(1.0)
    assert bleu(["completely different"], [["the cat sat on the mat"]])["bleu"] == 0.0


def test_compat_classes_end_to_end(tmp_path):
    env = compat.RAGEnvironment("tiny-llama:random", "tiny-llama:random")
    out = env.generate_response("what is it", ["doc a", "doc b"], max_length=96)
    assert isinstance(out, str)
    ppo = compat.PPOTrainer("tiny-llama:random", "tiny-llama:random", lora_r=4)
    qs = ["what is x", "who is y"]
    rs = ["x is a thing", "y"]
    with torch.no_grad():
        old, _, vals = ppo.sequence_logprobs(qs, rs)
    m = ppo.ppo_update(qs, rs, old, torch.tensor([1.0, 0.2]), vals, torch.tensor([0.5, -0.5]))
    assert set(m) == {"policy_loss", "value_loss", "entropy_loss", "total_loss", "approx_kl"}
    assert all(math.isfinite(v) for v in m.values())
    assert abs(m["approx_kl"]) < 1e-4  # same policy before the step


def test_compat_main(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    report = compat.main(checkpoint_dir=str(tmp_path / "ck"), epochs=1)
    assert list(report.columns) == ["Base Model", "RAG Model", "RL-finetuned Model"]
    assert {"relevance", "factual_accuracy", "overall_score"} <= set(report.index)
    assert os.path.exists(tmp_path / "model_comparison_results.csv")
    for suf in ("_policy", "_tokenizer", "_value_head.pt", "_adapter", "_trainer_state"):
        assert os.path.exists(str(tmp_path / "ck" / "best_model") + suf)
        assert os.path.exists(str(tmp_path / "ck" / "epoch_1") + suf)


def test_reference_loop_body_verbatim(tmp_path):
    """One iteration of the reference's RL loop body (rl.py:286-351) and its checkpoint calls
    (rl.py:365-379) run UNCHANGED against compat.RLTrainer: ``env.generate_response``,
    ``ppo_trainer.{tokenizer, policy, value_head, device, compute_advantages, ppo_update}`` and the
    HF calling convention of the policy (labels / output_hidden_states)."""
    import numpy as np

    trainer = compat.RLTrainer("tiny-llama:random", "tiny-llama:random", "tiny-bert:random", batch_size=2, epochs=1,
                               checkpoint_dir=str(tmp_path / "ck"), max_new_tokens=8, max_prompt_tokens=96,
                               minibatch_size=2)
    self = trainer
    assert isinstance(self.env, compat.RAGEnvironment) and isinstance(self.ppo_trainer, compat.PPOTrainer)
    assert self.env.model is self.ppo_trainer.policy.model  # one shared policy
    for attr in ("tokenizer", "policy", "value_head", "device", "optimizer", "ref_model"):
        assert hasattr(self.ppo_trainer, attr), attr
    batch = {"query": ["what is alpha", "who made the beta thing"],
             "retrieved_docs": [["alpha is a letter", "greek letters"], ["beta was made by someone"]],
             "ground_truth": ["a letter", "someone"]}
    logged = {}

    # ---- verbatim from rl.py:286-351 (wandb.log -> dict) ----
    queries = batch['query']
    retrieved_docs_batch = batch['retrieved_docs']
    ground_truths = batch.get('ground_truth', [None] * len(queries))

    # Generate responses with current policy
    responses = []
    for query, docs in zip(queries, retrieved_docs_batch):
        response = self.env.generate_response(query, docs, max_length=160)
        responses.append(response)

    # Calculate rewards
    rewards = []
    reward_components = []
    for response, query, docs, gt in zip(responses, queries, retrieved_docs_batch, ground_truths):
        reward, components = self.reward_model.calculate_reward(response, query, docs, gt)
        rewards.append(reward)
        reward_components.append(components)

    # Collect old log probabilities for PPO
    old_log_probs = []
    values = []
    with torch.no_grad():
        for query, response in zip(queries, responses):
            inputs = self.ppo_trainer.tokenizer(query, return_tensors="pt").to(self.ppo_trainer.device)
            response_ids = self.ppo_trainer.tokenizer(response, return_tensors="pt").to(self.ppo_trainer.device)

            # Get log probabilities
            outputs = self.ppo_trainer.policy(**inputs, labels=response_ids.input_ids)
            old_log_prob = -outputs.loss
            old_log_probs.append(old_log_prob.item())

            # Get value predictions
            value_outputs = self.ppo_trainer.policy(**inputs, output_hidden_states=True)
            hidden_states = value_outputs.hidden_states[-1][:, -1, :]
            value = self.ppo_trainer.value_head(hidden_states).squeeze(-1)
            values.append(value.item())

    # Compute advantages
    dones = [True] * len(rewards)  # All episodes end after one step in this setup
    advantages = self.ppo_trainer.compute_advantages(rewards, values, dones)

    # Update policy with PPO
    metrics = self.ppo_trainer.ppo_update(
        queries, responses,
        torch.tensor(old_log_probs).to(self.ppo_trainer.device),
        torch.tensor(rewards).to(self.ppo_trainer.device),
        torch.tensor(values).to(self.ppo_trainer.device),
        torch.tensor(advantages).to(self.ppo_trainer.device)
    )
    logged.update({
        "reward_mean": np.mean(rewards),
        "reward_std": np.std(rewards),
        "factual_accuracy": np.mean([comp["factual_accuracy"] for comp in reward_components]),
        "relevance": np.mean([comp["relevance"] for comp in reward_components]),
        "conciseness": np.mean([comp["conciseness"] for comp in reward_components]),
        "policy_loss": metrics["policy_loss"],
        "value_loss": metrics["value_loss"],
        "entropy_loss": metrics["entropy_loss"],
        "total_loss": metrics["total_loss"],
        "approx_kl": metrics["approx_kl"]
    })
    # ---- end verbatim ----
    assert all(math.isfinite(float(v)) for v in logged.values())
    # the old log-probs gathered the reference's way are the quantity ppo_update uses: before the
    # step the ratio is 1 (approx_kl ~ 0 up to batch-vs-single padding numerics)
    assert abs(metrics["approx_kl"]) < 1e-3
    assert advantages == pytest.approx([r - v for r, v in zip(rewards, values)])

    # rl.py:365-379 through the façade: save, perturb, load restores
    ck = str(tmp_path / "ck" / "it")
    self.save_checkpoint(ck)
    for suf in ("_policy", "_tokenizer", "_value_head.pt"):
        assert os.path.exists(ck + suf)
    w0 = self.ppo_trainer.value_head.linear.weight.detach().clone()
    lora0 = [p.detach().clone() for p in self.ppo_trainer.policy.lora_parameters()]
    with torch.no_grad():
        self.ppo_trainer.value_head.linear.weight.add_(1.0)
        for p in self.ppo_trainer.policy.lora_parameters():
            p.add_(0.5)
    self.load_checkpoint(ck)
    assert torch.equal(self.ppo_trainer.value_head.linear.weight, w0)
    for a, b in zip(self.ppo_trainer.policy.lora_parameters(), lora0):
        assert torch.equal(a, b)


def test_hf_policy_standard_labels_and_padding():
    """HF-style policy: labels == input_ids -> the shifted causal-LM loss; right padding gives the
    same last-token hidden state as the unpadded row."""
    ppo = compat.PPOTrainer("tiny-llama:random", "tiny-llama:random", lora_r=4)
    tok, pol = ppo.tokenizer, ppo.policy
    enc = tok("alpha beta gamma delta", return_tensors="pt")
    with torch.no_grad():
        out = pol(**enc, labels=enc.input_ids)
        lg = out.logits[0, :-1].float()
        ce = torch.nn.functional.cross_entropy(lg, enc.input_ids[0, 1:])
        assert float(out.loss) == pytest.approx(float(ce), rel=1e-4, abs=1e-4)
        h1 = pol(**enc, output_hidden_states=True).hidden_states[-1][0, -1]
        encr = tok(["alpha beta gamma delta", "x"], side="right")
        hr = pol(**encr, output_hidden_states=True).hidden_states[-1]
        n = int(encr.attention_mask[0].sum())
        torch.testing.assert_close(hr[0, n - 1], h1, rtol=1e-4, atol=1e-4)


def test_prompt_budget_drops_docs_not_query():
    """Evaluator / rollouts / RAG answers: an over-long prompt loses its lowest-ranked documents
    first; the "Query: ..." head and the instruction survive (the evaluator used to cut the head)."""
    from rag_tl_domainllm_optimizer_amd.rag.prompt import encode_prompt
    from rag_tl_domainllm_optimizer_amd.tokenizer import Tokenizer

    tok = Tokenizer.synthetic(512, "llama")
    w = tok.words()
    docs = [" ".join(w[i * 40:(i + 1) * 40]) for i in range(3)]
    q = " ".join(w[200:205])
    full = tok.encode(build_prompt(q, docs))
    one = tok.encode(build_prompt(q, docs[:1]))
    ids = encode_prompt(tok, q, docs, len(one) + 2)
    assert ids == one
    # same head (query) and same tail (instruction) as the full prompt
    assert ids[:8] == full[:8] and ids[-8:] == full[-8:] and len(full) > len(ids)
