"""Document ingestion: word-window chunking with overlap (plain text; PDF text is extracted upstream)."""
from __future__ import annotations

from typing import Iterable, List, Tuple


def chunk_text(text: str, chunk_words: int = 120, overlap: int = 20) -> List[str]:
    words = text.split()
    if not words:
        return []
    if len(words) <= chunk_words:
        return [" ".join(words)]
    step = max(1, chunk_words - overlap)
    out = []
    for s in range(0, len(words), step):
        out.append(" ".join(words[s:s + chunk_words]))
        if s + chunk_words >= len(words):
            break
    return out


def chunk_documents(docs: Iterable[str], chunk_words: int = 120, overlap: int = 20) -> Tuple[List[str], List[int]]:
    """-> (chunks, source doc index per chunk)."""
    chunks, src = [], []
    for i, d in enumerate(docs):
        for c in chunk_text(d, chunk_words, overlap):
            chunks.append(c)
            src.append(i)
    return chunks, src


def read_text_file(path: str) -> str:
    with open(path, "r", encoding="utf-8", errors="replace") as f:
        return f.read()
