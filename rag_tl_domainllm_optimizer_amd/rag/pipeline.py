"""End-to-end RAG answering: embed query -> index top-k -> reference prompt template -> generate.

The minimum end-to-end slice of SURVEY §7.3 and config 2 ("Mistral-7B bf16 RAG answer on 1 MI355X,
100k-doc IVF index in HBM"). Per-stage wall-clock latency is reported for every answer; this is
the "p50 RAG answer latency" half of the headline metric (README.md:38 publishes 2.4 s / 3.1 s).
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np
import torch

from ..generation import Generator, SamplingParams
from .prompt import build_prompt, extract_answer, encode_prompt


@dataclass
class RagAnswer:
    query: str
    answer: str
    doc_ids: List[int]
    docs: List[str]
    scores: List[float]
    timings: dict = field(default_factory=dict)


class RagPipeline:
    def __init__(self, encoder, index, docs: Sequence[str], model, tokenizer, top_k: int = 3,
                 sampling: Optional[SamplingParams] = None, max_prompt_tokens: int = 1024, max_batch: int = 1,
                 use_graph: bool = True):
        self.encoder, self.index, self.docs = encoder, index, list(docs)
        self.model, self.tok = model, tokenizer
        self.top_k = top_k
        self.sampling = sampling or SamplingParams(max_new_tokens=128)
        self.max_prompt_tokens = max_prompt_tokens
        self.gen = Generator(model, max_batch, max_prompt_tokens + self.sampling.max_new_tokens + 8,
                             use_graph=use_graph)
        self.max_batch = max_batch

    @property
    def device(self):
        return self.model.embed.device

    def _sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize()

    def retrieve(self, queries: Sequence[str], k: Optional[int] = None):
        q = self.encoder.encode(list(queries))
        return self.index.search(q, k or self.top_k)

    def _prompt_ids(self, query: str, docs: List[str]) -> List[int]:
        return encode_prompt(self.tok, query, docs, self.max_prompt_tokens)

    @torch.no_grad()
    def answer(self, queries: Sequence[str], top_ks: Optional[Sequence[Optional[int]]] = None) -> List[RagAnswer]:
        """Answers in batches of ``max_batch`` (one retrieval, one prefill, one graph-replayed
        decode per batch). ``top_ks``: per-query document counts (None = the pipeline's top_k):
        the batch retrieves the largest and each row keeps its own prefix."""
        out: List[RagAnswer] = []
        for s in range(0, len(queries), self.max_batch):
            qs = list(queries[s:s + self.max_batch])
            ks = [(k or self.top_k) for k in (top_ks[s:s + self.max_batch] if top_ks else [None] * len(qs))]
            t0 = time.perf_counter()
            scores, ids = self.retrieve(qs, max(ks))
            ids_l = [row[:k] for row, k in zip(ids.tolist(), ks)]
            scores = [row[:k] for row, k in zip(scores.tolist(), ks)]
            self._sync()
            t1 = time.perf_counter()
            docs = [[self.docs[i] for i in row if i >= 0] for row in ids_l]
            prompts = [self._prompt_ids(q, d) for q, d in zip(qs, docs)]
            t2 = time.perf_counter()
            g = self.gen.generate(prompts, self.sampling, pad_id=self.tok.pad_token_id,
                                  eos_ids=[self.tok.eos_token_id])
            t3 = time.perf_counter()
            for b, q in enumerate(qs):
                n = int(g.lengths[b])
                text = extract_answer(self.tok.decode(g.tokens[b, :n].tolist()))
                t4 = time.perf_counter()
                out.append(RagAnswer(q, text, ids_l[b], docs[b], scores[b],
                                     {"retrieve_s": t1 - t0, "prompt_s": t2 - t1, "generate_s": t3 - t2,
                                      "prefill_s": g.timings.get("prefill_s", 0.0),
                                      "decode_s": g.timings.get("decode_s", 0.0),
                                      "new_tokens": n, "prompt_tokens": len(prompts[b]), "total_s": t4 - t0}))
        return out

    def latency_stats(self, queries: Sequence[str], warmup: int = 2) -> dict:
        """p50 / p90 of single-query answers over ``queries[warmup:]``; the first ``warmup`` queries
        only warm up (graph capture, workspaces) and are not measured."""
        for q in queries[:warmup]:
            self.answer([q])
        measured = queries[warmup:] if len(queries) > warmup else queries
        lat, toks, ptoks, stages = [], [], [], {}
        for q in measured:
            a = self.answer([q])[0]
            lat.append(a.timings["total_s"])
            toks.append(a.timings["new_tokens"])
            ptoks.append(a.timings["prompt_tokens"])
            for k in ("retrieve_s", "prompt_s", "prefill_s", "decode_s"):
                stages.setdefault(k, []).append(a.timings[k])
        lat = np.array(lat)
        return {"p50_s": float(np.percentile(lat, 50)), "p90_s": float(np.percentile(lat, 90)),
                "mean_s": float(lat.mean()), "n": len(lat), "mean_new_tokens": float(np.mean(toks)),
                "mean_prompt_tokens": float(np.mean(ptoks)),
                "stage_mean_s": {k: float(np.mean(v)) for k, v in stages.items()}}
