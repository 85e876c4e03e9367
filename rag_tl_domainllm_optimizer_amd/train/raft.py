"""RAFT-style training data (README "RAFT-Inspired Training: distractor document handling",
README.md:2; declared, not implemented, in the reference).

For each question: with probability ``p_oracle`` the context holds the oracle (gold) document plus
``num_distractors`` distractors, otherwise distractors only (forcing the model to also rely on what
it has learned); documents are shuffled; the target is the ground-truth answer. The prompt is the
reference RAG template (rl.py:33-34), so SFT trains exactly the distribution PPO later rolls out.
"""
from __future__ import annotations

import random
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

from ..rag.prompt import build_prompt


@dataclass
class RaftConfig:
    num_distractors: int = 3
    p_oracle: float = 0.8
    seed: int = 0


def build_raft_examples(items, docs: Sequence[str], cfg: Optional[RaftConfig] = None) -> List[Dict[str, str]]:
    """items: objects/dicts with query, ground_truth, gold_doc (index into docs)."""
    cfg = cfg or RaftConfig()
    rng = random.Random(cfg.seed)
    out = []
    n = len(docs)
    for it in items:
        q = it["query"] if isinstance(it, dict) else it.query
        gt = it["ground_truth"] if isinstance(it, dict) else it.ground_truth
        gold = it["gold_doc"] if isinstance(it, dict) else it.gold_doc
        k = min(cfg.num_distractors, n - 1)
        dis = set()
        while len(dis) < k:
            j = rng.randrange(n)
            if j != gold:
                dis.add(j)
        ctx = list(dis)
        oracle = rng.random() < cfg.p_oracle
        if oracle:
            ctx.append(gold)
        rng.shuffle(ctx)
        out.append({"prompt": build_prompt(q, [docs[i] for i in ctx]), "answer": gt, "oracle": oracle,
                    "doc_ids": ctx})
    return out
