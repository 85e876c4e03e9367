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
