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
