"""RAG prompt template and answer extraction — byte-exact with the reference
(reinforcement_learning_optimization_after_rag.py:33-34 and :46-48)."""
from __future__ import annotations

from typing import List, Sequence

INSTRUCTION = "Based on the above information, please answer the query concisely and accurately."


def build_prompt(query: str, docs: Sequence[str]) -> str:
    if isinstance(docs, str):
        docs = [docs]
    context = f"Query: {query}\n\nContext:\n" + "\n".join([f"- {doc}" for doc in docs])
    return f"{context}\n\n{INSTRUCTION}"


def extract_answer(decoded: str) -> str:
    """Text after the instruction sentence (full text when the sentence is not reproduced)."""
    return decoded.split(INSTRUCTION)[-1].strip()


def fit_docs(query: str, docs: List[str], count_tokens, max_prompt_tokens: int) -> List[str]:
    """Drop the lowest-ranked documents until the prompt fits the token budget (SURVEY §5.7 d)."""
    docs = list(docs)
    while docs and count_tokens(build_prompt(query, docs)) > max_prompt_tokens:
        docs.pop()
    return docs


def encode_prompt(tokenizer, query: str, docs: Sequence[str], budget: int) -> List[int]:
    """Token ids of the RAG prompt within ``budget`` tokens: the lowest-ranked documents are
    dropped first, so the query and the instruction always survive; only a prompt that is still
    too long with no documents left is cut, from the left. Shared by rollouts, RAG answers and the
    evaluator."""
    if isinstance(docs, str):
        docs = [docs]
    docs = list(docs)
    ids = tokenizer.encode(build_prompt(query, docs))
    if len(ids) <= budget or not docs:
        return ids[-budget:] if len(ids) > budget else ids
    # the prompt length grows with the number of kept documents: binary search for the most that
    # fit (a long-context prompt of dozens of retrieved documents costs log2(n) encodes, not n)
    lo, hi, best = 0, len(docs) - 1, None
    while lo <= hi:
        mid = (lo + hi) // 2
        cand = tokenizer.encode(build_prompt(query, docs[:mid]))
        if len(cand) <= budget:
            best, lo = cand, mid + 1
        else:
            hi = mid - 1
    if best is None:  # even the query alone is too long: cut from the left
        ids = tokenizer.encode(build_prompt(query, []))
        return ids[-budget:]
    return best
