"""Native C++ tokenizer parity against the HF `tokenizers` library (installed) on synthetic data."""
import json

import pytest

from rag_tl_domainllm_optimizer_amd.tokenizer import Tokenizer, synthetic_words

tk = pytest.importorskip("tokenizers")

CORPUS = [
    "The quick brown fox jumps over the lazy dog.",
    "Retrieval augmented generation grounds answers in documents, doesn't it?",
    "PPO optimises a clipped surrogate objective; GAE estimates advantages (lambda=0.95).",
    "MI355X has 256 compute units and 288 GB of HBM3E memory!",
    "  leading spaces and   multiple   gaps  ",
    "numbers 12345 and mixed CASE Words.",
] * 20


def test_synthetic_roundtrip_and_hf_load(tmp_path):
    t = Tokenizer.synthetic(5000, "llama")
    assert t.vocab_size == 5000 and t.bos_token_id == 1 and t.eos_token_id == 2
    words = t.words()[:50]
    text = " ".join(words[:20]) + " . " + " ".join(words[20:30]) + " ?"
    ids = t.encode(text, add_special_tokens=False)
    assert t.decode(ids) == text
    t.save_pretrained(str(tmp_path))
    hf = tk.Tokenizer.from_file(str(tmp_path / "tokenizer.json"))
    assert hf.encode(text, add_special_tokens=False).ids == ids
    t2 = Tokenizer.from_pretrained(str(tmp_path))
    assert t2.encode(text) == t.encode(text)


def test_wordpiece_matches_hf():
    words = sorted({w.lower().strip(".,;!?()'=") for s in CORPUS for w in s.split()} - {""})
    vocab = {"[PAD]": 0, "[UNK]": 1, "[CLS]": 2, "[SEP]": 3}
    for w in words:
        vocab.setdefault(w[:3], len(vocab))
        if len(w) > 3:
            vocab.setdefault("##" + w[3:], len(vocab))
    for p in ".,;!?()'=":
        vocab.setdefault(p, len(vocab))
    hf = tk.Tokenizer(tk.models.WordPiece(vocab, unk_token="[UNK]"))
    hf.normalizer = tk.normalizers.Lowercase()
    hf.pre_tokenizer = tk.pre_tokenizers.BertPreTokenizer()
    ours = Tokenizer.from_hf_json(json.loads(hf.to_str()), {"unk_token": "[UNK]", "bos_token": "[CLS]",
                                                            "eos_token": "[SEP]", "pad_token": "[PAD]"})
    for s in CORPUS[:6]:
        assert ours.encode(s, add_special_tokens=False) == hf.encode(s, add_special_tokens=False).ids, s


def test_byte_level_bpe_matches_hf():
    bpe = tk.ByteLevelBPETokenizer()
    bpe.train_from_iterator(CORPUS, vocab_size=400, min_frequency=1, show_progress=False)
    tj = json.loads(bpe._tokenizer.to_str())
    ours = Tokenizer.from_hf_json(tj, {})
    for s in CORPUS[:6] + ["unseen wordz xyz"]:
        exp = bpe.encode(s).ids
        assert ours.encode(s, add_special_tokens=False) == exp, s
        assert ours.decode(exp) == bpe.decode(exp)


def test_sentencepiece_bpe_byte_fallback_matches_hf():
    vocab_bytes = [f"<0x{i:02X}>" for i in range(256)]
    model = tk.models.BPE(unk_token="<unk>", byte_fallback=True, fuse_unk=True)
    hf = tk.Tokenizer(model)
    hf.normalizer = tk.normalizers.Sequence([tk.normalizers.Prepend("▁"), tk.normalizers.Replace(" ", "▁")])
    hf.decoder = tk.decoders.Sequence([tk.decoders.Replace("▁", " "), tk.decoders.ByteFallback(), tk.decoders.Fuse(),
                                       tk.decoders.Strip(" ", 1, 0)])
    trainer = tk.trainers.BpeTrainer(vocab_size=500, special_tokens=["<unk>", "<s>", "</s>"] + vocab_bytes,
                                     show_progress=False)
    hf.train_from_iterator(CORPUS, trainer)
    ours = Tokenizer.from_hf_json(json.loads(hf.to_str()), {"bos_token": "<s>", "eos_token": "</s>",
                                                            "unk_token": "<unk>"})
    for s in CORPUS[:6] + ["unicode é ü 😀 fallback"]:
        exp = hf.encode(s, add_special_tokens=False).ids
        got = ours.encode(s, add_special_tokens=False)
        assert got == exp, (s, got[:20], exp[:20])
        assert ours.decode(exp) == hf.decode(exp)


def test_synthetic_words_deterministic():
    assert synthetic_words(100) == synthetic_words(100)
    assert len(set(synthetic_words(3000))) == 3000


def test_padding_left_right():
    t = Tokenizer.synthetic(1000, "llama")
    out = t([" ".join(t.words()[:3]), t.words()[5]])
    assert out["input_ids"].shape == (2, 4)
    assert out["start"].tolist() == [0, 2]
    e = Tokenizer.synthetic(1000, "bert")
    out = e([" ".join(e.words()[:3]), e.words()[5]])
    assert out["input_ids"][1].tolist()[:3] == [101, e.token_to_id(e.words()[5]), 102]
    assert out["lengths"].tolist() == [5, 3]
