"""Embedding-similarity reward (reference ``RewardModel``, reinforcement_learning_optimization_after_rag.py:53-123),
batched: every distinct response / query / document / ground-truth string of a rollout batch is
encoded exactly once in one encoder pass (on its own HIP stream when overlapped with rollout), and
all cosines are dot products of the normalised embeddings on device.

Formula (reference defaults, named fields):
  F   = max_i cos(resp, doc_i)           (0 if no docs)           rl.py:63-71
  Rel = cos(resp, query)                                          rl.py:73-79
  C   = wc<20: max(0.5, wc/20); wc<=150: 1; else max(0, 1-(wc-150)/150)   rl.py:81-91
  R   = 0.5 F + 0.3 Rel + 0.2 C ; with ground truth: R = 0.7 R + 0.3 cos(resp, gt)   rl.py:93-115
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch


@dataclass
class RewardConfig:
    weights: Dict[str, float] = field(default_factory=lambda: {"factual_accuracy": 0.5, "relevance": 0.3,
                                                               "conciseness": 0.2})
    gt_mix: Tuple[float, float] = (0.7, 0.3)
    short_words: int = 20      # rl.py:86
    long_words: int = 150      # rl.py:88 (the comment says 200; the code uses 150 — SURVEY B18)
    min_short_score: float = 0.5


def conciseness(word_count: int, cfg: RewardConfig = RewardConfig()) -> float:
    if word_count < cfg.short_words:
        return max(cfg.min_short_score, word_count / cfg.short_words)
    if word_count <= cfg.long_words:
        return 1.0
    return max(0.0, 1.0 - (word_count - cfg.long_words) / cfg.long_words)


class RewardModel:
    def __init__(self, encoder, cfg: Optional[RewardConfig] = None):
        self.encoder = encoder
        self.cfg = cfg or RewardConfig()

    @property
    def weights(self):
        return self.cfg.weights

    @torch.no_grad()
    def score(self, responses: Sequence[str], queries: Sequence[str], docs: Sequence[Sequence[str]],
              ground_truths: Optional[Sequence[Optional[str]]] = None):
        """-> (rewards fp32 [B], components dict of [B] tensors / lists)."""
        B = len(responses)
        gts = list(ground_truths) if ground_truths is not None else [None] * B
        texts: List[str] = []
        slot = {}

        def idx(t):
            if t not in slot:
                slot[t] = len(texts)
                texts.append(t)
            return slot[t]

        r_i = [idx(r) for r in responses]
        q_i = [idx(q) for q in queries]
        d_i = [[idx(d) for d in ds] for ds in docs]
        g_i = [idx(g) if g else -1 for g in gts]
        emb = self.encoder.encode(texts)  # [U, d] unit vectors, one pass
        dev = emb.device
        R = emb[torch.tensor(r_i, device=dev)]
        Q = emb[torch.tensor(q_i, device=dev)]
        rel = (R * Q).sum(-1)
        fact = torch.zeros(B, device=dev)
        maxd = max((len(x) for x in d_i), default=0)
        if maxd:
            pad = torch.tensor([x + [-1] * (maxd - len(x)) for x in d_i], device=dev)
            Dm = emb[pad.clamp(min=0)]                      # [B, maxd, d]
            sims = (R[:, None, :] * Dm).sum(-1).masked_fill(pad < 0, float("-inf"))
            fact = torch.where(pad.ge(0).any(-1), sims.max(-1).values, torch.zeros_like(rel))
        wc = [len(r.split()) for r in responses]
        conc = torch.tensor([conciseness(w, self.cfg) for w in wc], device=dev)
        w = self.cfg.weights
        reward = w["factual_accuracy"] * fact + w["relevance"] * rel + w["conciseness"] * conc
        has_gt = torch.tensor([g >= 0 for g in g_i], device=dev)
        gsim = torch.zeros(B, device=dev)
        if has_gt.any():
            G = emb[torch.tensor([max(g, 0) for g in g_i], device=dev)]
            gsim = torch.where(has_gt, (R * G).sum(-1), torch.zeros_like(rel))
            a, b = self.cfg.gt_mix
            reward = torch.where(has_gt, a * reward + b * gsim, reward)
        gl = gsim.tolist()  # one device->host copy, not one per row
        comps = {"factual_accuracy": fact, "relevance": rel, "conciseness": conc,
                 "ground_truth_similarity": [gl[i] if g_i[i] >= 0 else None for i in range(B)],
                 "total_reward": reward}
        return reward, comps

    # ----------------------------------------------------- reference per-sample API (rl.py:63-123)
    def calculate_factual_accuracy(self, response: str, retrieved_docs: Sequence[str]) -> float:
        if not retrieved_docs:
            return 0.0
        _, c = self.score([response], [""], [list(retrieved_docs)])
        return float(c["factual_accuracy"][0])

    def calculate_relevance(self, response: str, query: str) -> float:
        _, c = self.score([response], [query], [[]])
        return float(c["relevance"][0])

    def calculate_conciseness(self, response: str) -> float:
        return conciseness(len(response.split()), self.cfg)

    def calculate_reward(self, response: str, query: str, retrieved_docs: Sequence[str], ground_truth=None):
        r, c = self.score([response], [query], [list(retrieved_docs)], [ground_truth])
        comps = {"factual_accuracy": float(c["factual_accuracy"][0]), "relevance": float(c["relevance"][0]),
                 "conciseness": float(c["conciseness"][0]),
                 "ground_truth_similarity": c["ground_truth_similarity"][0] if ground_truth else None,
                 "total_reward": float(r[0])}
        return float(r[0]), comps
