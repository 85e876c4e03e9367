"""Datasets: reference-schema CSV loading, collation, rank sharding, synthetic corpora."""
from __future__ import annotations

import ast
import csv
import json
import random
from typing import Dict, Iterator, List, Optional, Sequence

from .synthetic import QAItem, SyntheticCorpus  # noqa: F401


def parse_docs(value) -> List[str]:
    """``retrieved_docs`` cell -> list of strings. Accepts JSON / Python list literals or a plain
    string (one document). Fixes the reference's character-iteration of CSV strings."""
    if isinstance(value, (list, tuple)):
        return [str(v) for v in value]
    if value is None:
        return []
    s = str(value).strip()
    if s.startswith("["):
        for parser in (json.loads, ast.literal_eval):
            try:
                v = parser(s)
                if isinstance(v, (list, tuple)):
                    return [str(x) for x in v]
            except Exception:
                pass
    return [s] if s else []


def load_records(path: str) -> List[Dict]:
    """CSV / JSONL / JSON with columns query, retrieved_docs, optional ground_truth (rl.py:270-288)."""
    if path.endswith(".jsonl"):
        with open(path) as f:
            rows = [json.loads(l) for l in f if l.strip()]
    elif path.endswith(".json"):
        with open(path) as f:
            rows = json.load(f)
    else:
        with open(path, newline="") as f:
            rows = list(csv.DictReader(f))
    out = []
    for r in rows:
        gt = r.get("ground_truth")
        out.append({"query": r["query"], "retrieved_docs": parse_docs(r.get("retrieved_docs")),
                    "ground_truth": gt if gt not in ("", None) else None})
    return out


class RecordLoader:
    """Shuffled mini-batches of records (lists kept per sample, not collated), sharded by rank so
    every data-parallel rank sees a disjoint slice of each epoch."""

    def __init__(self, records: Sequence[Dict], batch_size: int, shuffle: bool = True, seed: int = 0,
                 rank: int = 0, world: int = 1, drop_last: bool = False):
        self.records = list(records)
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.seed = seed
        self.rank, self.world = rank, world
        self.drop_last = drop_last
        self.epoch = 0
        self.start_batch = 0  # mid-epoch resume: batches of the current epoch already consumed

    def set_epoch(self, e: int, start_batch: int = 0):
        self.epoch = e
        self.start_batch = start_batch

    def state_dict(self) -> dict:
        return {"epoch": self.epoch, "start_batch": self.start_batch, "seed": self.seed}

    def _indices(self) -> List[int]:
        idx = list(range(len(self.records)))
        if self.shuffle:
            random.Random(self.seed + self.epoch).shuffle(idx)
        n = len(idx) // self.world * self.world if self.drop_last else len(idx)
        if not self.drop_last and len(idx) % self.world:
            idx += idx[: self.world - len(idx) % self.world]
            n = len(idx)
        return idx[self.rank:n:self.world]

    def __iter__(self) -> Iterator[Dict[str, list]]:
        idx = self._indices()
        skip, self.start_batch = self.start_batch, 0  # the resume offset applies to one epoch
        for s in range(skip * self.batch_size, len(idx), self.batch_size):
            chunk = idx[s:s + self.batch_size]
            if self.drop_last and len(chunk) < self.batch_size:
                break
            recs = [self.records[i] for i in chunk]
            yield {"query": [r["query"] for r in recs], "retrieved_docs": [r["retrieved_docs"] for r in recs],
                   "ground_truth": [r.get("ground_truth") for r in recs]}

    def __len__(self):
        n = len(self._indices())
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size
