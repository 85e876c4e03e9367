"""Batched sentence encoder (mean pooling + L2 normalisation), one forward for many strings.

Replaces the reference's per-string ``SentenceTransformer.encode`` calls (1 + k + 2 (+2) separate
forwards per reward, reinforcement_learning_optimization_after_rag.py:66-67,75-76,102-103): texts
are tokenised natively in parallel, sorted by length into padded batches, encoded on the GPU.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch

from ..models import build_model
from ..models.encoder import SentenceEncoder
from ..tokenizer import Tokenizer, load_tokenizer


class Encoder:
    def __init__(self, model: SentenceEncoder, tokenizer: Tokenizer, max_length: int = 256, batch_size: int = 256):
        self.model = model
        self.tokenizer = tokenizer
        self.max_length = min(max_length, model.cfg.max_position - model.cfg.position_offset)
        self.batch_size = batch_size

    @classmethod
    def from_name(cls, name_or_path: str = "all-MiniLM-L6-v2:random", device="cpu", max_length: int = 256,
                  batch_size: int = 256, seed: int = 0) -> "Encoder":
        model = build_model(name_or_path, device=device, seed=seed)
        tok = load_tokenizer(name_or_path, model.cfg.vocab_size, model.cfg.arch)
        return cls(model.eval(), tok, max_length, batch_size)

    @property
    def device(self):
        return self.model.word_embed.device

    @property
    def dim(self) -> int:
        return self.model.cfg.hidden_size

    @torch.no_grad()
    def encode(self, texts: Sequence[str], normalize: bool = True) -> torch.Tensor:
        """-> fp32 [N, dim] on the model's device (unit vectors when normalize)."""
        texts = list(texts)
        N = len(texts)
        out = torch.empty(N, self.dim, dtype=torch.float32, device=self.device)
        if N == 0:
            return out
        enc = self.tokenizer.encode_batch(texts, True, self.max_length)
        order = sorted(range(N), key=lambda i: len(enc[i]))
        for s in range(0, N, self.batch_size):
            idx = order[s:s + self.batch_size]
            batch = self.tokenizer.pad([enc[i] for i in idx], side="right", device=self.device)
            emb = self.model.encode_ids(batch["input_ids"], batch["lengths"], normalize)
            out[torch.tensor(idx, device=self.device)] = emb.float()
        return out

    def encode_unique(self, texts: Sequence[str], normalize: bool = True):
        """Encode each distinct string once; returns (embeddings [U, d], index map list -> row)."""
        uniq, where = {}, []
        for t in texts:
            if t not in uniq:
                uniq[t] = len(uniq)
            where.append(uniq[t])
        emb = self.encode(list(uniq.keys()), normalize)
        return emb, torch.tensor(where, dtype=torch.long, device=emb.device)
