"""Tokenizers: HF ``tokenizer.json``-compatible WordLevel / WordPiece / byte-level BPE /
SentencePiece-BPE, executed by the native C++ runtime (``_C.NativeTokenizer``).

Random-init presets come with a deterministic synthetic word-level vocabulary of exactly the
model's vocab size (special ids placed where the model family expects them), so generated ids
always decode to words; real checkpoints bring their own ``tokenizer.json``.
"""
from __future__ import annotations

import json
import os
import random
from typing import Dict, List, Optional, Sequence

import torch

FAMILY_SPECIALS = {
    # family: (unk, bos, eos, pad) as (token, id); pad None -> eos (reference pad fix, rl.py:143-146)
    "llama": {"unk": ("<unk>", 0), "bos": ("<s>", 1), "eos": ("</s>", 2), "pad": None},
    "opt": {"pad": ("<pad>", 1), "bos": ("</s>", 2), "eos": ("</s>", 2), "unk": ("<unk>", 3)},
    "bert": {"pad": ("[PAD]", 0), "unk": ("[UNK]", 100), "bos": ("[CLS]", 101), "eos": ("[SEP]", 102),
             "mask": ("[MASK]", 103)},
    "mpnet": {"bos": ("<s>", 0), "pad": ("<pad>", 1), "eos": ("</s>", 2), "unk": ("<unk>", 3)},
}
_TEMPLATE = {"llama": "bos", "mistral": "bos", "opt": "bos", "bert": "cls_sep", "mpnet": "cls_sep"}
PUNCT = list(".,;:?!'\"()-")


def family_of(arch: str) -> str:
    return {"mistral": "llama", "llama": "llama"}.get(arch, arch)


def synthetic_words(n: int, seed: int = 1234) -> List[str]:
    """n distinct pronounceable lowercase pseudo-words, deterministic."""
    rng = random.Random(seed)
    cons = "bcdfghjklmnprstvwz"
    vow = "aeiou"
    words, seen = [], set()
    length = 2
    while len(words) < n:
        for _ in range(n * 4):
            w = "".join(rng.choice(cons) + rng.choice(vow) for _ in range(length))
            if rng.random() < 0.3:
                w += rng.choice(cons)
            if w not in seen:
                seen.add(w)
                words.append(w)
                if len(words) >= n:
                    break
        length += 1
    return words


class BatchEncoding(dict):
    """dict of tensors with attribute access and ``.to(device)`` (the shape of HF's BatchEncoding
    that reference-style code unpacks into a model call: ``model(**enc)``)."""

    def __getattr__(self, name):
        try:
            return self[name]
        except KeyError as e:
            raise AttributeError(name) from e

    def to(self, device):
        return BatchEncoding({k: (v.to(device) if isinstance(v, torch.Tensor) else v) for k, v in self.items()})


class Tokenizer:
    def __init__(self, kind: str, vocab: Dict[str, int], merges=None, specials: Optional[dict] = None,
                 lowercase: bool = False, continuing_prefix: str = "##", add_prefix_space: bool = False,
                 byte_fallback: bool = False, template: str = "bos", padding_side: str = "left",
                 extra_special: Sequence[str] = ()):
        from ..ops._ext import native

        self.kind = kind
        self.vocab = dict(vocab)
        self.merges = [tuple(m) for m in (merges or [])]
        self.specials = dict(specials or {})
        self.lowercase = lowercase
        self.continuing_prefix = continuing_prefix
        self.add_prefix_space = add_prefix_space
        self.byte_fallback = byte_fallback
        self.template = template
        self.padding_side = padding_side
        special_tokens = sorted({v[0] for v in self.specials.values() if v} | set(extra_special))
        self.special_tokens = special_tokens
        unk = self.specials.get("unk")
        self._impl = native().NativeTokenizer(kind, self.vocab, self.merges, unk[0] if unk else "", lowercase,
                                              continuing_prefix, add_prefix_space, byte_fallback, special_tokens)

    # --------------------------------------------------------------- special ids
    def _sid(self, name):
        v = self.specials.get(name)
        return v[1] if v else None

    @property
    def bos_token_id(self):
        return self._sid("bos")

    @property
    def eos_token_id(self):
        return self._sid("eos")

    @property
    def unk_token_id(self):
        return self._sid("unk")

    @property
    def pad_token_id(self):
        p = self._sid("pad")
        return p if p is not None else self.eos_token_id

    @property
    def pad_token(self):
        p = self.specials.get("pad") or self.specials.get("eos")
        return p[0] if p else None

    @pad_token.setter
    def pad_token(self, tok: str):
        """``tokenizer.pad_token = tokenizer.eos_token`` (the reference's pad fix, rl.py:143-146)."""
        self.specials["pad"] = (tok, self.token_to_id(tok))

    @property
    def eos_token(self):
        e = self.specials.get("eos")
        return e[0] if e else None

    @property
    def vocab_size(self) -> int:
        return int(self._impl.vocab_size())

    def __len__(self):
        return self.vocab_size

    # --------------------------------------------------------------- encode/decode
    def _wrap(self, ids: List[int], add_special: bool) -> List[int]:
        if not add_special:
            return ids
        if self.template == "cls_sep":
            return [self.bos_token_id] + ids + [self.eos_token_id]
        if self.bos_token_id is not None:
            return [self.bos_token_id] + ids
        return ids

    def encode(self, text: str, add_special_tokens: bool = True, max_length: Optional[int] = None) -> List[int]:
        ids = self._wrap(list(self._impl.encode(text)), add_special_tokens)
        if max_length is not None and len(ids) > max_length:
            ids = ids[:max_length - 1] + [ids[-1]] if self.template == "cls_sep" else ids[:max_length]
        return ids

    def encode_batch(self, texts: Sequence[str], add_special_tokens: bool = True,
                     max_length: Optional[int] = None, nthreads: int = 8) -> List[List[int]]:
        raw = self._impl.encode_batch(list(texts), nthreads)
        out = []
        for ids in raw:
            ids = self._wrap(list(ids), add_special_tokens)
            if max_length is not None and len(ids) > max_length:
                ids = ids[:max_length - 1] + [ids[-1]] if self.template == "cls_sep" else ids[:max_length]
            out.append(ids)
        return out

    def decode(self, ids, skip_special_tokens: bool = True) -> str:
        if isinstance(ids, torch.Tensor):
            ids = ids.tolist()
        return self._impl.decode([int(i) for i in ids], skip_special_tokens)

    def batch_decode(self, seqs, skip_special_tokens: bool = True) -> List[str]:
        return [self.decode(s, skip_special_tokens) for s in seqs]

    def token_to_id(self, t: str) -> int:
        return int(self._impl.token_to_id(t))

    def id_to_token(self, i: int) -> str:
        return self._impl.id_to_token(int(i))

    def pad(self, seqs: List[List[int]], side: Optional[str] = None, max_length: Optional[int] = None,
            device=None):
        """-> dict(input_ids [B, S], attention_mask [B, S], lengths [B], start [B])."""
        side = side or self.padding_side
        S = max_length or max((len(s) for s in seqs), default=1)
        S = max(S, 1)
        B = len(seqs)
        ids = torch.full((B, S), self.pad_token_id, dtype=torch.long)
        mask = torch.zeros((B, S), dtype=torch.long)
        lens = torch.tensor([min(len(s), S) for s in seqs], dtype=torch.long)
        for b, s in enumerate(seqs):
            s = s[-S:] if side == "left" else s[:S]
            n = len(s)
            if side == "left":
                ids[b, S - n:] = torch.tensor(s, dtype=torch.long)
                mask[b, S - n:] = 1
            else:
                ids[b, :n] = torch.tensor(s, dtype=torch.long)
                mask[b, :n] = 1
        start = (S - lens) if side == "left" else torch.zeros_like(lens)
        out = {"input_ids": ids, "attention_mask": mask, "lengths": lens, "start": start}
        if device is not None:
            out = {k: v.to(device) for k, v in out.items()}
        return out

    def __call__(self, texts, padding: bool = True, max_length: Optional[int] = None, add_special_tokens=True,
                 side: Optional[str] = None, device=None, return_tensors: Optional[str] = "pt",
                 truncation: bool = False):
        """HF-style call (``tokenizer(text, return_tensors="pt").to(device)``, rl.py:36,196,309):
        a :class:`BatchEncoding` of torch tensors (``input_ids``, ``attention_mask``, plus
        ``lengths`` / ``start``). ``return_tensors`` other than "pt" is not supported."""
        if return_tensors not in (None, "pt"):
            raise ValueError(f"return_tensors={return_tensors!r}: only torch tensors are supported")
        single = isinstance(texts, str)
        seqs = self.encode_batch([texts] if single else list(texts), add_special_tokens,
                                 max_length if (truncation or max_length) else None)
        return BatchEncoding(self.pad(seqs, side=side, device=device))

    # --------------------------------------------------------------- persistence
    def to_hf_json(self) -> dict:
        added = []
        for name, v in self.specials.items():
            if v:
                added.append({"id": v[1], "content": v[0], "single_word": False, "lstrip": False, "rstrip": False,
                              "normalized": False, "special": True})
        uniq = {a["id"]: a for a in added}
        model = {"type": {"wordlevel": "WordLevel", "wordpiece": "WordPiece", "bpe": "BPE", "sp_bpe": "BPE"}[self.kind],
                 "vocab": self.vocab}
        unk = self.specials.get("unk")
        if self.kind == "wordlevel":
            model["unk_token"] = unk[0] if unk else "<unk>"
        elif self.kind == "wordpiece":
            model.update({"unk_token": unk[0] if unk else "[UNK]", "continuing_subword_prefix": self.continuing_prefix,
                          "max_input_chars_per_word": 100})
        else:
            model.update({"merges": [list(m) for m in self.merges], "dropout": None,
                          "unk_token": unk[0] if (unk and self.kind == "sp_bpe") else None,
                          "byte_fallback": self.byte_fallback, "fuse_unk": self.kind == "sp_bpe",
                          "continuing_subword_prefix": None, "end_of_word_suffix": None, "ignore_merges": False})
        if self.kind in ("wordlevel", "wordpiece"):
            pre = {"type": "BertPreTokenizer"}
            norm = {"type": "Lowercase"} if self.lowercase else None
            dec = {"type": "WordPiece", "prefix": self.continuing_prefix, "cleanup": True} \
                if self.kind == "wordpiece" else None
        elif self.kind == "bpe":
            pre = {"type": "ByteLevel", "add_prefix_space": self.add_prefix_space, "trim_offsets": True,
                   "use_regex": True}
            norm = None
            dec = {"type": "ByteLevel", "add_prefix_space": True, "trim_offsets": True, "use_regex": True}
        else:
            pre = None
            norm = {"type": "Sequence", "normalizers": (
                [{"type": "Prepend", "prepend": "▁"}] if self.add_prefix_space else []) +
                [{"type": "Replace", "pattern": {"String": " "}, "content": "▁"}]}
            dec = {"type": "Sequence", "decoders": [
                {"type": "Replace", "pattern": {"String": "▁"}, "content": " "}, {"type": "ByteFallback"},
                {"type": "Fuse"}, {"type": "Strip", "content": " ", "start": 1, "stop": 0}]}
        return {"version": "1.0", "truncation": None, "padding": None, "added_tokens": sorted(uniq.values(),
                key=lambda a: a["id"]), "normalizer": norm, "pre_tokenizer": pre, "post_processor": None,
                "decoder": dec, "model": model}

    def save_pretrained(self, path: str):
        os.makedirs(path, exist_ok=True)
        with open(os.path.join(path, "tokenizer.json"), "w") as f:
            json.dump(self.to_hf_json(), f, ensure_ascii=False)
        cfg = {"tokenizer_class": "PreTrainedTokenizerFast", "padding_side": self.padding_side,
               "model_max_length": 1000000, "clean_up_tokenization_spaces": False,
               "ragtl_template": self.template, "ragtl_kind": self.kind}
        stm = {}
        for name in ("bos", "eos", "unk", "pad"):
            v = self.specials.get(name)
            if v:
                cfg[f"{name}_token"] = v[0]
                stm[f"{name}_token"] = v[0]
        with open(os.path.join(path, "tokenizer_config.json"), "w") as f:
            json.dump(cfg, f, indent=2)
        with open(os.path.join(path, "special_tokens_map.json"), "w") as f:
            json.dump(stm, f, indent=2)

    @classmethod
    def from_pretrained(cls, path: str, arch: Optional[str] = None) -> "Tokenizer":
        with open(os.path.join(path, "tokenizer.json")) as f:
            tj = json.load(f)
        cfg = {}
        if os.path.exists(os.path.join(path, "tokenizer_config.json")):
            with open(os.path.join(path, "tokenizer_config.json")) as f:
                cfg = json.load(f)
        return cls.from_hf_json(tj, cfg, arch)

    @classmethod
    def from_hf_json(cls, tj: dict, tcfg: Optional[dict] = None, arch: Optional[str] = None) -> "Tokenizer":
        tcfg = tcfg or {}
        model = tj["model"]
        mtype = model["type"]
        vocab = model["vocab"]
        added = {a["content"]: a["id"] for a in tj.get("added_tokens", [])}
        vocab = dict(vocab)
        vocab.update(added)
        norm = json.dumps(tj.get("normalizer") or {})
        pre = json.dumps(tj.get("pre_tokenizer") or {})
        lowercase = "Lowercase" in norm or '"lowercase": true' in norm
        if mtype == "WordPiece":
            kind = "wordpiece"
        elif mtype == "WordLevel":
            kind = "wordlevel"
        elif mtype == "BPE":
            kind = "bpe" if "ByteLevel" in pre or "ByteLevel" in json.dumps(tj.get("decoder") or {}) else "sp_bpe"
        else:
            raise ValueError(f"unsupported tokenizer model {mtype}")
        merges = []
        for m in model.get("merges", []) or []:
            merges.append(tuple(m.split(" ", 1)) if isinstance(m, str) else tuple(m))
        add_prefix = ('"add_prefix_space": true' in pre) if kind == "bpe" else ("Prepend" in norm or
                                                                                 '"prepend_scheme": "always"' in pre)
        specials = {}
        for name in ("bos", "eos", "unk", "pad"):
            tok = tcfg.get(f"{name}_token")
            if isinstance(tok, dict):
                tok = tok.get("content")
            if tok and tok in vocab:
                specials[name] = (tok, vocab[tok])
        if "unk" not in specials and model.get("unk_token") in vocab:
            specials["unk"] = (model["unk_token"], vocab[model["unk_token"]])
        if not specials.get("bos") or not specials.get("eos"):
            for cand in (("<s>", "</s>"), ("[CLS]", "[SEP]")):
                if cand[0] in vocab and "bos" not in specials:
                    specials["bos"] = (cand[0], vocab[cand[0]])
                if cand[1] in vocab and "eos" not in specials:
                    specials["eos"] = (cand[1], vocab[cand[1]])
        template = tcfg.get("ragtl_template") or ("cls_sep" if kind == "wordpiece" or (arch in ("bert", "mpnet"))
                                                   else "bos")
        side = tcfg.get("padding_side", "right" if template == "cls_sep" else "left")
        return cls(kind, vocab, merges, specials, lowercase, model.get("continuing_subword_prefix") or "##",
                   add_prefix, bool(model.get("byte_fallback", False)), template, side,
                   extra_special=[a["content"] for a in tj.get("added_tokens", []) if a.get("special")])

    # --------------------------------------------------------------- synthetic
    @classmethod
    def synthetic(cls, vocab_size: int, arch: str = "llama", seed: int = 1234) -> "Tokenizer":
        fam = family_of(arch)
        sp = {k: v for k, v in FAMILY_SPECIALS[fam].items() if v}
        vocab: Dict[str, int] = {}
        used = set()
        for tok, i in sp.values():
            vocab[tok] = i
            used.add(i)
        free = [i for i in range(vocab_size) if i not in used]
        fill = PUNCT + [str(d) for d in range(10)]
        words = synthetic_words(len(free) - len(fill), seed)
        for i, w in zip(free, fill + words):
            vocab[w] = i
        template = _TEMPLATE.get(arch, "bos")
        specials = dict(FAMILY_SPECIALS[fam])
        return cls("wordlevel", vocab, [], specials, False, "##", False, False, template,
                   "right" if template == "cls_sep" else "left")

    def words(self) -> List[str]:
        """Ordinary (non-special, alphabetic) vocabulary entries — the synthetic corpus alphabet."""
        sp = set(self.special_tokens)
        return [w for w, _ in sorted(self.vocab.items(), key=lambda kv: kv[1]) if w not in sp and w.isalpha()]


def load_tokenizer(name_or_path: str, vocab_size: Optional[int] = None, arch: str = "llama") -> Tokenizer:
    """tokenizer.json directory, or a synthetic vocab for random-init presets."""
    if os.path.isdir(name_or_path) and os.path.exists(os.path.join(name_or_path, "tokenizer.json")):
        return Tokenizer.from_pretrained(name_or_path, arch)
    from ..models.config import resolve_preset

    cfg = resolve_preset(name_or_path)
    if cfg is None and vocab_size is None:
        raise ValueError(f"cannot build a tokenizer for {name_or_path!r}")
    return Tokenizer.synthetic(vocab_size or cfg.vocab_size, cfg.arch if cfg else arch)
