"""Dense retrieval: bi-encoder embedding, chunking, and flat / IVF vector indexes resident in HBM.

This is the README's declared "RAG Core" (Sentence Transformers + ChromaDB/FAISS, README.md:12,26-28)
that the reference never implements (its RAG environment receives pre-retrieved documents,
reinforcement_learning_optimization_after_rag.py:287).
"""
from .encoder import Encoder  # noqa: F401
from .index import FlatIndex, IVFIndex, load_index  # noqa: F401
from .chunking import chunk_text, chunk_documents  # noqa: F401
