"""Varlen (packed) forwards on CPU: the packed scoring / SFT / prefill paths equal the padded ones
(values and LoRA gradients), so the GEMMs can skip left and right pads."""
import numpy as np
import pytest
import torch

from rag_tl_domainllm_optimizer_amd import models
from rag_tl_domainllm_optimizer_amd.generation import Generator, SamplingParams
from rag_tl_domainllm_optimizer_amd.models import ValueHead, packed_index
from rag_tl_domainllm_optimizer_amd.models.config import PRESETS
from rag_tl_domainllm_optimizer_amd.train.common import score_sequences


def test_packed_index_layout():
    idx, off = packed_index([0, 3, 5], [4, 5, 5], 6, "cpu")
    assert idx.tolist() == [0, 1, 2, 3, 9, 10]  # row 0: 0..3, row 1: 3..4, row 2: empty
    assert off.tolist() == [0, 4, 6, 6]


def _batch(cfg, seed=0):
    g = torch.Generator().manual_seed(seed)
    B, S, T = 4, 12, 6
    st = np.array([0, 3, 7, 5])
    rl = np.array([6, 2, 1, 4])
    pid = torch.randint(5, cfg.vocab_size, (B, S), generator=g)
    resp = torch.randint(5, cfg.vocab_size, (B, T), generator=g)
    for b in range(B):
        pid[b, :st[b]] = 0
        resp[b, rl[b]:] = 0
    return pid, torch.tensor(st, dtype=torch.int32), resp, torch.tensor(rl), st, rl


@pytest.mark.parametrize("preset", ["tiny-mistral", "tiny-opt"])
def test_score_sequences_packed_matches_padded(preset):
    cfg = PRESETS[preset]
    m = models.CausalLM(cfg, dtype=torch.float32, seed=1)
    m.add_lora(4, 8.0, None, seed=2)
    with torch.no_grad():
        for p in m.lora_parameters():
            p.normal_(0, 0.05)
    m.refresh_lora()
    vh = ValueHead(cfg.hidden_size, seed=3)
    pid, start, resp, rlen, st, rl = _batch(cfg)
    outs, grads = [], []
    for lengths in (None, (st, rl)):
        for p in m.lora_parameters():
            p.grad = None
        lp, ent, val, mask = score_sequences(m, pid, start, resp, rlen, 1.3, vh, lengths=lengths)
        loss = ((lp + 0.1 * ent + 0.5 * val) * mask).sum()
        loss.backward()
        outs.append((lp.detach(), ent.detach(), val.detach(), mask))
        grads.append([p.grad.clone() for p in m.lora_parameters()])
    (a_lp, a_ent, a_val, mask), (b_lp, b_ent, b_val, _) = outs
    for x, y in ((a_lp, b_lp), (a_ent, b_ent), (a_val, b_val)):
        torch.testing.assert_close(x * mask, y * mask, rtol=1e-5, atol=1e-5)
    assert float((b_lp * ~mask).abs().max()) == 0.0  # masked positions are zero in the packed form
    for ga, gb in zip(*grads):
        torch.testing.assert_close(ga, gb, rtol=1e-4, atol=1e-5)  # fp32 summation order


def test_score_sequences_no_padding_stays_unpacked(monkeypatch):
    """Full-length rows drop only the last token (< 3 % of the grid): the padded path runs."""
    cfg = PRESETS["tiny-llama"]
    m = models.CausalLM(cfg, dtype=torch.float32, seed=1)
    calls = []
    orig = m.forward

    def spy(*a, **k):
        calls.append(k.get("packed_idx") is not None)
        return orig(*a, **k)

    monkeypatch.setattr(m, "forward", spy)
    B, S, T = 2, 40, 10
    pid = torch.randint(5, 200, (B, S))
    resp = torch.randint(5, 200, (B, T))
    with torch.no_grad():
        score_sequences(m, pid, torch.zeros(B, dtype=torch.int32), resp, torch.full((B,), T), 1.0,
                        lengths=(np.zeros(B, np.int64), np.full(B, T)))
        score_sequences(m, pid, torch.tensor([20, 0], dtype=torch.int32), resp, torch.full((B,), T), 1.0,
                        lengths=(np.array([20, 0]), np.full(B, T)))
    assert calls == [False, True]


def test_sft_loss_packed_matches_padded(monkeypatch):
    from rag_tl_domainllm_optimizer_amd.tokenizer import Tokenizer
    from rag_tl_domainllm_optimizer_amd.train import SFTConfig, SFTTrainer

    cfg = PRESETS["tiny-mistral"]
    tok = Tokenizer.synthetic(cfg.vocab_size, "mistral")
    m = models.CausalLM(cfg, dtype=torch.float32, seed=4)
    tr = SFTTrainer(m, tok, SFTConfig(batch_size=3, lora_r=4, max_seq=64))
    words = tok.words()
    prompts = [" ".join(words[i:i + n]) for i, n in ((0, 20), (30, 5), (50, 11))]
    answers = [" ".join(words[i:i + n]) for i, n in ((90, 3), (95, 7), (99, 2))]
    ids, start, tgt = tr.encode(prompts, answers)
    res = []
    for flag in ("0", "1"):
        monkeypatch.setenv("RAGTL_PACK", flag)
        for p in m.lora_parameters():
            p.grad = None
        loss, n = tr.loss(ids, start, tgt)
        loss.backward()
        res.append((float(loss.detach()), n, [p.grad.clone() for p in m.lora_parameters()]))
    assert res[0][1] == res[1][1]
    assert abs(res[0][0] - res[1][0]) < 1e-5
    for ga, gb in zip(res[0][2], res[1][2]):
        torch.testing.assert_close(ga, gb, rtol=1e-4, atol=1e-5)  # fp32 summation order


@pytest.mark.parametrize("preset", ["tiny-llama", "tiny-opt"])
def test_prefill_packed_matches_padded(preset, monkeypatch):
    cfg = PRESETS[preset]
    m = models.CausalLM(cfg, dtype=torch.float32, seed=5)
    prompts = [[5, 9, 33, 41, 7, 8, 9, 10, 11, 12], [12, 300, 4], [77, 78]]
    res = []
    for flag in ("0", "1"):
        monkeypatch.setenv("RAGTL_PACK", flag)
        gen = Generator(m, max_batch=4, max_seq=32, device="cpu")
        out = gen.generate(prompts, SamplingParams(max_new_tokens=5, do_sample=False), pad_id=0, eos_ids=[-5])
        res.append((out.tokens.clone(), out.logprobs.clone()))
    assert torch.equal(res[0][0], res[1][0])
    torch.testing.assert_close(res[0][1], res[1][1], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("preset", ["tiny-mistral", "tiny-opt"])
@pytest.mark.parametrize("packed", [False, True])
def test_forward_out_rows_matches_full(preset, packed):
    """``out_rows``: the last layer's o_proj / MLP / final norm on the selected rows only gives the
    same hidden states (and LoRA gradients) as the full forward indexed afterwards."""
    from rag_tl_domainllm_optimizer_amd.generation import KVCache

    cfg = PRESETS[preset]
    m = models.CausalLM(cfg, dtype=torch.float32, seed=7)
    m.add_lora(4, 8.0, None, seed=2)
    with torch.no_grad():
        for p in m.lora_parameters():
            p.normal_(0, 0.05)
    m.refresh_lora()
    pid, start, resp, rlen, st, rl = _batch(cfg, seed=3)
    B, S = pid.shape
    idx = packed_index(st, np.full(B, S), S, "cpu")[0] if packed else None
    n = idx.numel() if packed else B * S
    rows = torch.tensor(sorted({0, 1, n // 2, n - 3, n - 1, 2}), dtype=torch.long)
    res = []
    for sel in (None, rows):
        for p in m.lora_parameters():
            p.grad = None
        h = m(pid, kv_start=start, packed_idx=idx, out_rows=sel)
        if sel is None:
            h = h[rows]
        (h * torch.linspace(-1, 1, h.shape[1])).sum().backward()
        res.append((h.detach(), [p.grad.clone() for p in m.lora_parameters()]))
    assert res[1][0].shape == (rows.numel(), cfg.hidden_size)
    torch.testing.assert_close(res[0][0], res[1][0], rtol=1e-5, atol=1e-5)
    for ga, gb in zip(res[0][1], res[1][1]):
        # fp32 sums over different row subsets block differently (MKL): ~1e-5 absolute noise
        torch.testing.assert_close(ga, gb, rtol=1e-4, atol=1e-4)
    # prefill: hidden of the last position of every row == the full forward's
    if not packed:
        with torch.no_grad():
            cache = KVCache(cfg.num_layers, B, cfg.num_kv_heads, S + 4, cfg.head_dim, "cpu", torch.float32)
            hp = m.prefill(pid, start, cache)
            hf = m(pid, kv_start=start)
        torch.testing.assert_close(hp, hf[torch.arange(B) * S + S - 1], rtol=1e-5, atol=1e-5)
