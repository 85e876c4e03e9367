"""Synthetic RAG corpora (no network on the GPU boxes: SURVEY N11).

A corpus is a set of "fact documents" about pseudo-word entities; each query asks for one
attribute of one entity and has a ground-truth answer sentence and a gold document, so retrieval
recall, RAFT training and PPO rewards all have something checkable to work with. The vocabulary is
the tokenizer's own word list, so every generated string tokenises without <unk>.
"""
from __future__ import annotations

import json
import random
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence


@dataclass
class QAItem:
    query: str
    ground_truth: str
    gold_doc: int
    entity: str
    relation: str
    value: str

    def to_row(self, docs: Sequence[str], retrieved: Optional[List[int]] = None) -> Dict[str, str]:
        ids = retrieved if retrieved is not None else [self.gold_doc]
        return {"query": self.query, "retrieved_docs": json.dumps([docs[i] for i in ids]),
                "ground_truth": self.ground_truth}


class SyntheticCorpus:
    def __init__(self, words: Sequence[str], n_docs: int = 1000, facts_per_doc: int = 6, doc_words: int = 60,
                 n_relations: int = 64, seed: int = 0):
        rng = random.Random(seed)
        words = list(words)
        if len(words) < 200:
            raise ValueError("need at least 200 vocabulary words for a synthetic corpus")
        rng.shuffle(words)
        n_rel = min(n_relations, len(words) // 10)
        self.relations = words[:n_rel]
        pool = words[n_rel:]
        self.entities = [pool[i % len(pool)] + ("" if i < len(pool) else "") for i in range(n_docs)]
        if n_docs > len(pool):  # compound entity names when the vocab is small
            self.entities = [f"{pool[i % len(pool)]} {pool[(i * 7 + 3) % len(pool)]}" for i in range(n_docs)]
        self.values_pool = pool
        self.filler = pool
        self.docs: List[str] = []
        self.facts: List[List[tuple]] = []
        for i, e in enumerate(self.entities):
            rels = rng.sample(self.relations, min(facts_per_doc, len(self.relations)))
            fs = [(e, r, rng.choice(self.values_pool)) for r in rels]
            sent = [f"{a} {r} {v} ." for a, r, v in fs]
            text = " ".join(sent)
            n_fill = max(0, doc_words - len(text.split()))
            if n_fill:
                text += " " + " ".join(rng.choice(self.filler) for _ in range(n_fill)) + " ."
            self.docs.append(text)
            self.facts.append(fs)
        self._rng = rng

    def __len__(self):
        return len(self.docs)

    def sample_queries(self, n: int, seed: int = 1) -> List[QAItem]:
        rng = random.Random(seed)
        out = []
        for _ in range(n):
            d = rng.randrange(len(self.docs))
            e, r, v = rng.choice(self.facts[d])
            out.append(QAItem(query=f"what {r} {e} ?", ground_truth=f"{e} {r} {v} .", gold_doc=d, entity=e,
                              relation=r, value=v))
        return out

    def distractors(self, gold: int, k: int, rng: random.Random) -> List[int]:
        out = set()
        while len(out) < min(k, len(self.docs) - 1):
            j = rng.randrange(len(self.docs))
            if j != gold:
                out.add(j)
        return list(out)

    def to_csv(self, path: str, n: int, k_docs: int = 3, seed: int = 2):
        """Reference training-CSV schema: query, retrieved_docs (JSON list), ground_truth (rl.py:270-288)."""
        import csv

        rng = random.Random(seed)
        items = self.sample_queries(n, seed)
        with open(path, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=["query", "retrieved_docs", "ground_truth"])
            w.writeheader()
            for it in items:
                ids = [it.gold_doc] + self.distractors(it.gold_doc, k_docs - 1, rng)
                rng.shuffle(ids)
                w.writerow(it.to_row(self.docs, ids))
        return path
