"""In-repo ROUGE-1/2/L and BLEU-4 (the reference loads them via `evaluate`, rl.py:28-29,386-387,
which is not installed here). Semantics follow the public packages:

* ROUGE (rouge_score defaults used by `evaluate`): lowercase, non-alphanumerics -> spaces,
  whitespace split, no stemming; F-measure of n-gram overlap / LCS.
* BLEU (`evaluate`'s bleu = nmt corpus BLEU): 13a tokenisation, max_order 4, no smoothing,
  brevity penalty exp(1 - r/c) when c < r.

The reference passes pre-split token lists to BLEU (rl.py:430); here strings are
tokenised by 13a like the package does.
"""
from __future__ import annotations

import math
import re
from collections import Counter
from typing import Dict, List, Sequence


def _rouge_tokens(s: str) -> List[str]:
    return re.sub(r"[^a-z0-9]+", " ", s.lower()).split()


def _ngrams(toks, n):
    return Counter(tuple(toks[i:i + n]) for i in range(len(toks) - n + 1))


def _f1(overlap, pred_n, ref_n):
    if pred_n == 0 or ref_n == 0 or overlap == 0:
        return 0.0
    p, r = overlap / pred_n, overlap / ref_n
    return 2 * p * r / (p + r)


def _lcs(a, b):
    if not a or not b:
        return 0
    prev = [0] * (len(b) + 1)
    for x in a:
        cur = [0]
        for j, y in enumerate(b):
            cur.append(prev[j] + 1 if x == y else max(prev[j + 1], cur[j]))
        prev = cur
    return prev[-1]


def rouge_scores(prediction: str, reference: str) -> Dict[str, float]:
    p, r = _rouge_tokens(prediction), _rouge_tokens(reference)
    out = {}
    for n in (1, 2):
        pn, rn = _ngrams(p, n), _ngrams(r, n)
        out[f"rouge{n}"] = _f1(sum((pn & rn).values()), max(len(p) - n + 1, 0), max(len(r) - n + 1, 0))
    out["rougeL"] = _f1(_lcs(p, r), len(p), len(r))
    return out


def rouge(predictions: Sequence[str], references: Sequence[str]) -> Dict[str, float]:
    """Mean F-measures over pairs (what `evaluate.load('rouge').compute` reports, aggregated)."""
    acc = {"rouge1": 0.0, "rouge2": 0.0, "rougeL": 0.0}
    for p, r in zip(predictions, references):
        for k, v in rouge_scores(p, r).items():
            acc[k] += v
    n = max(len(predictions), 1)
    return {k: v / n for k, v in acc.items()}


def tokenize_13a(line: str) -> List[str]:
    line = line.replace("<skipped>", "").replace("-\n", "").replace("\n", " ")
    if "&" in line:
        line = line.replace("&quot;", '"').replace("&amp;", "&").replace("&lt;", "<").replace("&gt;", ">")
    line = f" {line} "
    line = re.sub(r"([\{-\~\[-\` -\&\(-\+\:-\@\/])", r" \1 ", line)
    line = re.sub(r"([^0-9])([\.,])", r"\1 \2 ", line)
    line = re.sub(r"([\.,])([^0-9])", r" \1 \2", line)
    line = re.sub(r"([0-9])(-)", r"\1 \2 ", line)
    return line.split()


def bleu(predictions: Sequence[str], references: Sequence[Sequence[str]], max_order: int = 4,
         smooth: bool = False) -> Dict[str, float]:
    matches = [0] * max_order
    possible = [0] * max_order
    ref_len = trans_len = 0
    for pred, refs in zip(predictions, references):
        if isinstance(refs, str):
            refs = [refs]
        pt = tokenize_13a(pred)
        rts = [tokenize_13a(r) for r in refs]
        ref_len += min(len(r) for r in rts)
        trans_len += len(pt)
        merged = Counter()
        for rt in rts:
            for n in range(1, max_order + 1):
                merged |= _ngrams(rt, n)
        for n in range(1, max_order + 1):
            pn = _ngrams(pt, n)
            ov = pn & merged
            matches[n - 1] += sum(ov.values())
            possible[n - 1] += max(len(pt) - n + 1, 0)
    precisions = []
    for i in range(max_order):
        if smooth:
            precisions.append((matches[i] + 1.0) / (possible[i] + 1.0))
        else:
            precisions.append(matches[i] / possible[i] if possible[i] > 0 else 0.0)
    geo = math.exp(sum(math.log(p) for p in precisions) / max_order) if min(precisions) > 0 else 0.0
    ratio = trans_len / ref_len if ref_len else 0.0
    bp = 1.0 if ratio > 1.0 else (math.exp(1 - 1.0 / ratio) if ratio > 0 else 0.0)
    return {"bleu": geo * bp, "precisions": precisions, "brevity_penalty": bp, "length_ratio": ratio,
            "translation_length": trans_len, "reference_length": ref_len}
