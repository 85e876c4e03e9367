"""Evaluation (reference ``ModelEvaluator``, reinforcement_learning_optimization_after_rag.py:381-463).

Per test item: generate an answer (batched, on device), then ROUGE-1/2/L + BLEU-4 against the
ground truth when present, and the reward components (relevance, factual accuracy, overall score);
metrics are means over the items that produced them. ``compare_models`` returns a DataFrame with
metrics as rows and model names as columns, as the reference does.
Fixed vs the reference: the RAG prompt includes the retrieved documents by default
(``include_docs=True``) and the prompt echo is not scored.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..generation import Generator, SamplingParams
from ..metrics import bleu, rouge_scores
from ..rag.prompt import encode_prompt, extract_answer

METRIC_KEYS = ["rouge1", "rouge2", "rougeL", "bleu", "relevance", "factual_accuracy", "overall_score"]


@dataclass
class EvalConfig:
    max_length: int = 512          # rl.py:413 (prompt + answer)
    max_new_tokens: int = 128
    temperature: float = 0.7       # rl.py:414
    do_sample: bool = True         # rl.py:415
    top_k: int = 50
    include_docs: bool = True
    batch_size: int = 16
    seed: int = 0
    # ``cli pipeline`` ends with the reference's model comparison (rl.py:444-463, 491-525) over this
    # many held-out queries (0 disables it)
    compare_items: int = 32


class Evaluator:
    def __init__(self, reward_model, cfg: Optional[EvalConfig] = None):
        self.reward_model = reward_model
        self.cfg = cfg or EvalConfig()

    @torch.no_grad()
    def generate(self, model, tokenizer, items: Sequence[dict], include_docs: Optional[bool] = None) -> List[str]:
        c = self.cfg
        if include_docs is not None and include_docs != c.include_docs:
            c = dataclasses.replace(c, include_docs=include_docs)
        prompts = []
        # the prompt keeps room for the answer: documents are dropped lowest-ranked first (as in
        # the rollouts) instead of cutting "Query: ..." off the front
        budget = max(1, c.max_length - c.max_new_tokens)
        for it in items:
            if c.include_docs:
                prompts.append(encode_prompt(tokenizer, it["query"], it.get("retrieved_docs") or [], budget))
            else:
                ids = tokenizer.encode(it["query"])
                prompts.append(ids[-(c.max_length - 1):])
        S = max(len(p) for p in prompts)
        T = max(1, min(c.max_new_tokens, c.max_length - S))
        gen = Generator(model, min(c.batch_size, len(prompts)), S + T + 1)
        params = SamplingParams(max_new_tokens=T, temperature=c.temperature, top_k=c.top_k, do_sample=c.do_sample,
                                seed=c.seed)
        out_txt = []
        for s in range(0, len(prompts), gen.max_batch):
            o = gen.generate(prompts[s:s + gen.max_batch], params, pad_id=tokenizer.pad_token_id,
                             eos_ids=[tokenizer.eos_token_id])
            for b in range(o.tokens.shape[0]):
                n = int(o.lengths[b])
                out_txt.append(extract_answer(tokenizer.decode(o.tokens[b, :n].tolist())))
        return out_txt

    def evaluate_model(self, model, tokenizer, test_data: Sequence[dict],
                       include_docs: Optional[bool] = None) -> Dict[str, float]:
        """Under data parallelism each rank scores its shard (items rank::world); the per-item
        scores are all-gathered (object all-gather) so every rank returns the same
        means over the whole test set."""
        from ..parallel import all_gather_object, info

        di = info()
        full = list(test_data)
        test_data = full[di.rank::di.world] if di.world > 1 else full
        responses = self.generate(model, tokenizer, test_data, include_docs) if test_data else []
        res = {k: [] for k in METRIC_KEYS}
        for it, resp in zip(test_data, responses):
            gt = it.get("ground_truth")
            if gt:
                r = rouge_scores(resp, gt)
                res["rouge1"].append(r["rouge1"])
                res["rouge2"].append(r["rouge2"])
                res["rougeL"].append(r["rougeL"])
                res["bleu"].append(bleu([resp], [[gt]])["bleu"])
        if test_data:
            rewards, comps = self.reward_model.score(responses, [it["query"] for it in test_data],
                                                     [it.get("retrieved_docs") or [] for it in test_data],
                                                     [it.get("ground_truth") for it in test_data])
            res["relevance"] = comps["relevance"].tolist()
            res["factual_accuracy"] = comps["factual_accuracy"].tolist()
            res["overall_score"] = rewards.tolist()
        self.last_responses = responses
        if di.world > 1:
            parts = all_gather_object(res)
            res = {k: sum((p[k] for p in parts), []) for k in res}
        return {k: float(np.mean(v)) for k, v in res.items() if v}

    def compare_models(self, models: Dict[str, tuple], test_data: Sequence[dict]):
        """``models``: name -> (model, tokenizer) or (model, tokenizer, opts) with opts
        ``include_docs`` (per-model prompt mode: the reference's "Base Model" answers the bare
        query, the "RAG Model" sees the retrieved documents) and ``prepare`` (a callable run right
        before that model is evaluated, e.g. loading an adapter into a shared base)."""
        import pandas as pd

        comparison = {}
        for name, spec in models.items():
            model, tok = spec[0], spec[1]
            opts = spec[2] if len(spec) > 2 else {}
            if opts.get("prepare") is not None:
                opts["prepare"]()
            print(f"Evaluating {name}...")
            comparison[name] = self.evaluate_model(model, tok, test_data, opts.get("include_docs"))
        return pd.DataFrame(comparison)
