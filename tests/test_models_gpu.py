"""Model-level GPU tests: native-kernel forward vs fp32 CPU oracle, graph decode == eager decode,
PPO step, encoder, IVF recall."""
import math

import pytest
import torch

from rag_tl_domainllm_optimizer_amd import models, ops
from rag_tl_domainllm_optimizer_amd.generation import Generator, SamplingParams
from rag_tl_domainllm_optimizer_amd.models.config import PRESETS

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _pair(preset, seed=1):
    cfg = PRESETS[preset]
    cpu = models.CausalLM(cfg, dtype=torch.float32, seed=seed)
    gpu = models.CausalLM(cfg, device=DEV, dtype=torch.bfloat16, init=False)
    with torch.no_grad():
        for (n, a), (_, b) in zip(cpu.named_parameters(), gpu.named_parameters()):
            b.copy_(a.to(torch.bfloat16))
        for (n, a), (_, b) in zip(cpu.named_parameters(), cpu.named_parameters()):
            a.copy_(a.to(torch.bfloat16).float())  # same rounded weights on both sides
    return cpu, gpu


@pytest.mark.parametrize("preset", ["tiny-llama", "tiny-mistral", "tiny-opt"])
def test_decoder_forward_matches_cpu(preset):
    cpu, gpu = _pair(preset)
    ids = torch.randint(3, cpu.cfg.vocab_size, (3, 70))
    start = torch.tensor([0, 11, 40], dtype=torch.int32)
    with torch.no_grad():
        ref = cpu.logits(cpu(ids, kv_start=start)).view(3, 70, -1)
        out = gpu.logits(gpu(ids.to(DEV), kv_start=start.to(DEV))).view(3, 70, -1).float().cpu()
    for b in range(3):
        s = int(start[b])
        err = (out[b, s:] - ref[b, s:]).abs().max().item()
        assert err < 0.05 * ref[b, s:].abs().max().item() + 0.05, (b, err)


@pytest.mark.parametrize("preset", ["tiny-llama", "tiny-opt"])
def test_graph_decode_matches_eager(preset):
    cfg = PRESETS[preset]
    m = models.CausalLM(cfg, device=DEV, dtype=torch.bfloat16, seed=2)
    prompts = [[5, 9, 33, 41, 7, 8], [12, 300, 4], [77] * 11]
    p = SamplingParams(max_new_tokens=12, do_sample=False)
    g1 = Generator(m, 4, 64, DEV, use_graph=True).generate(prompts, p, pad_id=0, eos_ids=[-1])
    g2 = Generator(m, 4, 64, DEV, use_graph=False).generate(prompts, p, pad_id=0, eos_ids=[-1])
    assert torch.equal(g1.tokens, g2.tokens)
    # sampled: graph replay advances the RNG offset on device exactly like eager
    p = SamplingParams(max_new_tokens=12, temperature=0.7, top_k=50, seed=3)
    s1 = Generator(m, 4, 64, DEV, use_graph=True).generate(prompts, p, pad_id=0, eos_ids=[-1])
    s2 = Generator(m, 4, 64, DEV, use_graph=False).generate(prompts, p, pad_id=0, eos_ids=[-1])
    assert torch.equal(s1.tokens, s2.tokens)
    torch.testing.assert_close(s1.logprobs, s2.logprobs)


def test_decode_matches_teacher_forcing():
    cfg = PRESETS["tiny-mistral"]
    m = models.CausalLM(cfg, device=DEV, dtype=torch.bfloat16, seed=4)
    prompts = [[5, 9, 33, 41, 7, 8, 9, 10], [12, 300, 4]]
    p = SamplingParams(max_new_tokens=10, temperature=0.7, top_k=0, seed=5)
    out = Generator(m, 2, 64, DEV).generate(prompts, p, pad_id=0, eos_ids=[-1])
    from rag_tl_domainllm_optimizer_amd.train.common import score_sequences

    with torch.no_grad():
        lp, _, _, _ = score_sequences(m, out.prompt_ids, out.prompt_start, out.tokens, out.lengths, 1 / 0.7)
    torch.testing.assert_close(lp, out.logprobs, rtol=0.0, atol=1e-2)


def test_fused_decode_follows_adapter_updates():
    """Batch-1 decode reads weights derived in place from the adapters (merged W + UB A, then the
    norm fold): after an optimizer-style adapter update + refresh_lora, the next generation must
    score like teacher forcing under the NEW adapter (a stale derived weight would not)."""
    from rag_tl_domainllm_optimizer_amd.train.common import score_sequences

    cfg = PRESETS["tiny-mistral"]
    m = models.CausalLM(cfg, device=DEV, dtype=torch.bfloat16, seed=4)
    m.add_lora(8, 16.0, "all", seed=1)
    gen = Generator(m, 1, 64, DEV)
    p = SamplingParams(max_new_tokens=10, temperature=0.7, top_k=0, seed=5)
    prompts = [[5, 9, 33, 41, 7, 8, 9, 10]]
    for step in range(3):
        with torch.no_grad():
            for q in m.lora_parameters():
                q.normal_(0, 0.08)
        m.refresh_lora()
        out = gen.generate(prompts, p, pad_id=0, eos_ids=[-1])
        # teacher forcing on the same merged bf16 weights the decode engine reads (W + s B A rounded
        # once): what is left is the two engines' numerics (a stale derived weight is off by far more)
        prev = m.set_lora_merged(True)
        try:
            with torch.no_grad():
                lp, _, _, _ = score_sequences(m, out.prompt_ids, out.prompt_start, out.tokens, out.lengths, 1 / 0.7)
        finally:
            m.set_lora_merged(prev)
        err = float((lp - out.logprobs).abs().max())
        assert err <= 1e-2, (step, err)


def test_shuffled_decode_weights_match_row_major(monkeypatch):
    """Batch-1 decode on the tile-ordered weight images (qkv, o, gate_up, down, lm_head) == the
    row-major weights, bitwise at a common split-K, including after an adapter update (the images
    follow the merged / folded sources)."""
    cfg = PRESETS["tiny-mistral"]
    m = models.CausalLM(cfg, device=DEV, dtype=torch.bfloat16, seed=6)
    m.add_lora(8, 16.0, "all", seed=2)
    p = SamplingParams(max_new_tokens=12, temperature=0.7, top_k=0, seed=9)
    prompts = [[5, 9, 33, 41, 7, 8, 9, 10, 11]]
    outs = {}
    ops.native().set_tuning({"decode_split": 2})  # same split-K for both layouts -> bitwise comparable
    for flag in ("1", "0"):
        monkeypatch.setenv("RAGTL_DECODE_SHUF", flag)
        gen = Generator(m, 1, 64, DEV)
        res = []
        for step in range(2):
            with torch.no_grad():
                g = torch.Generator(device=DEV).manual_seed(step)
                for q in m.lora_parameters():
                    q.copy_(torch.randn(q.shape, device=DEV, generator=g, dtype=q.dtype) * 0.05)
            m.refresh_lora()
            out = gen.generate(prompts, p, pad_id=0, eos_ids=[-1])
            res.append((out.tokens.clone(), out.logprobs.clone()))
        outs[flag] = res
    ops.native().set_tuning({"decode_split": 0})
    assert any(len(layer._shufc) for layer in m.layers) and m._head_shuf is not None
    for (t1, l1), (t0, l0) in zip(outs["1"], outs["0"]):
        assert torch.equal(t1, t0)
        assert torch.equal(l1, l0)


def test_encoder_gpu_matches_cpu():
    cfg = PRESETS["tiny-mpnet"]
    cpu = models.SentenceEncoder(cfg, dtype=torch.float32, seed=3)
    gpu = models.SentenceEncoder(cfg, device=DEV, dtype=torch.bfloat16, init=False)
    with torch.no_grad():
        for (_, a), (_, b) in zip(cpu.named_parameters(), gpu.named_parameters()):
            b.copy_(a)
    ids = torch.randint(5, cfg.vocab_size, (4, 40))
    lens = torch.tensor([40, 3, 17, 29])
    e1 = cpu.encode_ids(ids, lens)
    e2 = gpu.encode_ids(ids.to(DEV), lens.to(DEV)).cpu()
    assert (e1 * e2).sum(-1).min().item() > 0.995


def test_ivf_recall_vs_flat():
    from rag_tl_domainllm_optimizer_amd.retrieval import FlatIndex, IVFIndex

    g = torch.Generator().manual_seed(0)
    centers = torch.nn.functional.normalize(torch.randn(64, 384, generator=g), dim=-1)
    x = torch.nn.functional.normalize(centers[torch.randint(0, 64, (20000,), generator=g)] +
                                      0.02 * torch.randn(20000, 384, generator=g), dim=-1)
    q = torch.nn.functional.normalize(x[:200] + 0.005 * torch.randn(200, 384, generator=g), dim=-1)
    flat = FlatIndex(384, device=DEV)
    flat.add(x)
    ivf = IVFIndex(384, nlist=64, device=DEV, nprobe=8)
    ivf.train(x, niter=8)
    ivf.add(x)
    _, fi = flat.search(q, 10)
    _, ii = ivf.search(q, 10)
    # exact search agrees with torch
    sc = q.to(DEV) @ x.to(DEV).t()
    ti = torch.topk(sc, 10).indices
    assert (fi[:, 0] == ti[:, 0]).float().mean() > 0.95
    recall = sum(len(set(a.tolist()) & set(b.tolist())) for a, b in zip(fi, ii)) / fi.numel()
    assert recall > 0.8, recall


def test_ppo_step_gpu():
    from rag_tl_domainllm_optimizer_amd.data import SyntheticCorpus
    from rag_tl_domainllm_optimizer_amd.retrieval import Encoder
    from rag_tl_domainllm_optimizer_amd.rewards import RewardModel
    from rag_tl_domainllm_optimizer_amd.tokenizer import Tokenizer
    from rag_tl_domainllm_optimizer_amd.train.ppo import PPOConfig, PPOTrainer

    cfg = PRESETS["tiny-mistral"]
    tok = Tokenizer.synthetic(cfg.vocab_size, "mistral")
    pol = models.CausalLM(cfg, device=DEV, dtype=torch.bfloat16, seed=1)
    ecfg = PRESETS["tiny-bert"]
    enc = Encoder(models.SentenceEncoder(ecfg, device=DEV, dtype=torch.bfloat16, seed=2).eval(),
                  Tokenizer.synthetic(ecfg.vocab_size, "bert"), max_length=64)
    corpus = SyntheticCorpus(tok.words(), n_docs=50, doc_words=20, seed=3)
    items = corpus.sample_queries(8)
    batch = {"query": [i.query for i in items], "retrieved_docs": [[corpus.docs[i.gold_doc]] for i in items],
             "ground_truth": [i.ground_truth for i in items]}
    tr = PPOTrainer(pol, tok, RewardModel(enc), PPOConfig(max_new_tokens=8, max_prompt_tokens=96,
                                                          minibatch_size=4, lora_r=8), max_batch=8)
    m1 = tr.step(batch)
    m2 = tr.step(batch)
    for m in (m1, m2):
        assert all(math.isfinite(v) for v in m.values() if isinstance(v, float))
    assert 8 <= m1["rollout_tokens"] <= 8 * 8  # rows stop early when the random policy samples EOS


def test_odd_vocab_generation_gpu():
    """A vocabulary that is not a multiple of 8 (OpenChat-3.5: 32002) generates and scores on the
    GPU: the LM head falls back to the library GEMM, the sampler to its generic kernel."""
    import dataclasses

    from rag_tl_domainllm_optimizer_amd.generation import Generator, SamplingParams
    from rag_tl_domainllm_optimizer_amd.train.common import score_sequences

    cfg = dataclasses.replace(PRESETS["tiny-mistral"], vocab_size=514, name="tiny-openchat")
    m = models.CausalLM(cfg, device=DEV, dtype=torch.bfloat16, seed=4)
    prompts = [[5, 9, 33, 41, 7, 8, 9, 513], [12, 300, 4]]
    p = SamplingParams(max_new_tokens=6, temperature=0.7, top_k=20, seed=5)
    out = Generator(m, 2, 64, DEV).generate(prompts, p, pad_id=0, eos_ids=[-1])
    assert out.tokens.shape == (2, 6) and int(out.tokens.max()) < 514 and torch.isfinite(out.logprobs).all()
    with torch.no_grad():
        lp, _, _, _ = score_sequences(m, out.prompt_ids, out.prompt_start, out.tokens, out.lengths, 1 / 0.7)
    torch.testing.assert_close(lp, out.logprobs, rtol=0.0, atol=1e-2)


@pytest.mark.parametrize("merged_lora,batch", [(False, 160), (True, 160), (False, 100)])
def test_batched_decode_deferred_splitk_bitwise(merged_lora, batch):
    """Batch > 64 decode with the split-K reduces fused into their consumers (qkv partials summed in
    the MFMA attention prologue, o / down partials summed inside the RMSNorms) == the same decode
    with separate reduce launches, bitwise; greedy generation on the graph path agrees too."""
    from rag_tl_domainllm_optimizer_amd.models.config import ModelConfig

    cfg = ModelConfig(arch="mistral", vocab_size=512, hidden_size=512, num_layers=2, num_heads=8, num_kv_heads=2,
                      head_dim=128, intermediate_size=1024, max_position=512, norm_eps=1e-5, name="t-d128")
    m = models.CausalLM(cfg, device=DEV, dtype=torch.bfloat16, seed=6)
    if merged_lora:
        m.add_lora(8, 16.0, "all")
        with torch.no_grad():
            for layer in m.layers:
                for g in layer.lora.values():
                    for b in g.b:
                        b.normal_(0, 0.05)
                    g.refresh()
        m.set_lora_merged(True)
    g = torch.Generator().manual_seed(0)
    # batch 160 x 2 kv-heads = 320 pairs: the MFMA attention sums the qkv partials; batch 100 = 200
    # pairs: the VALU kernel, so the partials are reduced first
    prompts = [torch.randint(3, 512, (int(n),), generator=g).tolist() for n in torch.randint(5, 40, (batch,), generator=g)]
    p = SamplingParams(max_new_tokens=6, do_sample=False)
    m.defer_splitk = True
    a = Generator(m, batch, 64, DEV, use_graph=False).generate(prompts, p, pad_id=0, eos_ids=[-1])
    m.defer_splitk = False
    b = Generator(m, batch, 64, DEV, use_graph=False).generate(prompts, p, pad_id=0, eos_ids=[-1])
    assert torch.equal(a.tokens, b.tokens)
    torch.testing.assert_close(a.logprobs, b.logprobs, rtol=0, atol=0)
    m.defer_splitk = True
    c = Generator(m, batch, 64, DEV, use_graph=True).generate(prompts, p, pad_id=0, eos_ids=[-1])
    assert torch.equal(a.tokens, c.tokens)


def test_varlen_packed_scoring_and_prefill_gpu(monkeypatch):
    """Packed (varlen) scoring and prefill on the MI355X kernels agree with the padded forms: the
    same per-token math on fewer GEMM rows — log-probs and values bitwise (the scoring forward is
    batch-invariant), LoRA gradients to fp32-atomic reduction order, greedy prefill continuations
    identical (prefill under ops.batch_invariant: by default its small-M GEMMs pick a split-K per M)."""
    import numpy as np

    from rag_tl_domainllm_optimizer_amd.models import ValueHead
    from rag_tl_domainllm_optimizer_amd.train.common import score_sequences

    cfg = PRESETS["tiny-mistral"]
    m = models.CausalLM(cfg, device=DEV, dtype=torch.bfloat16, seed=11)
    m.add_lora(8, 16.0, None, seed=2)
    with torch.no_grad():
        for p in m.lora_parameters():
            p.normal_(0, 0.02)
    m.refresh_lora()
    vh = ValueHead(cfg.hidden_size, device=DEV, seed=3)
    g = torch.Generator().manual_seed(0)
    B, S, T = 8, 96, 32
    st = np.array([0, 40, 77, 10, 60, 5, 90, 33])
    rl = np.array([32, 5, 17, 1, 30, 12, 8, 25])
    pid = torch.randint(5, cfg.vocab_size, (B, S), generator=g)
    resp = torch.randint(5, cfg.vocab_size, (B, T), generator=g)
    for b in range(B):
        pid[b, :st[b]] = 0
        resp[b, rl[b]:] = 0
    pid, resp = pid.to(DEV), resp.to(DEV)
    start = torch.tensor(st, dtype=torch.int32, device=DEV)
    rlen = torch.tensor(rl, device=DEV)
    outs, grads = [], []
    for lengths in (None, (st, rl)):
        for p in m.lora_parameters():
            p.grad = None
        lp, ent, val, mask = score_sequences(m, pid, start, resp, rlen, 1.0, vh, lengths=lengths)
        ((lp + 0.5 * val) * mask).sum().backward()
        outs.append((lp.detach().float(), val.detach().float(), mask))
        grads.append(torch.cat([p.grad.float().reshape(-1) for p in m.lora_parameters()]))
    (a_lp, a_v, mask), (b_lp, b_v, _) = outs
    assert torch.equal(a_lp * mask, b_lp * mask)
    assert torch.equal(a_v * mask, b_v * mask)
    rel = float((grads[0] - grads[1]).norm() / grads[0].norm().clamp(min=1e-12))
    assert rel < 1e-2, rel
    # prefill: greedy continuations of variable-length prompts, packed vs padded
    prompts = [list(range(7, 7 + n)) for n in (60, 5, 33, 17)]
    toks = []
    for flag in ("0", "1"):
        monkeypatch.setenv("RAGTL_PACK", flag)
        gen = Generator(m, max_batch=4, max_seq=96, device=DEV)
        gen.use_graph = False
        with ops.batch_invariant():
            out = gen.generate(prompts, SamplingParams(max_new_tokens=6, do_sample=False), pad_id=0, eos_ids=[-5])
        toks.append(out.tokens.cpu())
    assert torch.equal(toks[0], toks[1]), toks


def test_graph_replay_eos_after_allocator_churn():
    """Replays of the captured decode graph keep testing the EOS ids they were captured with: the
    second generation on one Generator stops at EOS even after the allocator has recycled the
    first call's small blocks (the graph once read a freed per-call EOS tensor)."""
    cfg = PRESETS["tiny-llama"]
    m = models.CausalLM(cfg, device=DEV, dtype=torch.bfloat16, seed=3)
    gen = Generator(m, max_batch=2, max_seq=64, device=DEV)
    prompts = [[5, 9, 33, 41, 7], [12, 300, 4, 8]]
    ref = gen.generate(prompts, SamplingParams(max_new_tokens=12, do_sample=False), pad_id=0, eos_ids=[-7])
    eos = int(ref.tokens[0, 3])
    first = [t for t in range(4) if int(ref.tokens[0, t]) == eos][0] + 1
    lens = []
    for _ in range(3):
        out = gen.generate(prompts, SamplingParams(max_new_tokens=12, do_sample=False), pad_id=0, eos_ids=[eos])
        lens.append(int(out.lengths[0]))
        assert out.tokens[0, :first].tolist() == ref.tokens[0, :first].tolist()
        # churn: small device blocks of the EOS tensor's size, holding other ids
        junk = [torch.full((1,), 123456 + i, dtype=torch.long, device=DEV) for i in range(64)]
        torch.cuda.synchronize()
        del junk
    assert lens == [first] * 3, (lens, first)


def test_graph_runner_keep_restore_and_shared_pool():
    """runtime.GraphRunner: the warm-up / capture do not advance restored state, replays read the
    kept per-call tensor, a key change recaptures, and two runners share the process graph pool."""
    from rag_tl_domainllm_optimizer_amd import runtime

    acc = torch.zeros(4, device=DEV)
    step = torch.zeros(1, dtype=torch.long, device=DEV)

    def make(delta):
        d = torch.full((4,), float(delta), device=DEV)  # per-call input, captured by address

        def fn():
            acc.add_(d * 2.0)  # intermediate from the graph pool, then accumulate
            step.add_(1)
        return fn, d

    r1, r2 = runtime.GraphRunner(), runtime.GraphRunner()
    fn, d = make(1.5)
    assert r1.needs("a")
    r1.capture(fn, "a", keep=(d,), restore=[acc, step])
    del d, fn
    junk = [torch.full((4,), 9.0, device=DEV) for _ in range(32)]  # recycle small blocks
    del junk
    assert float(acc.sum()) == 0.0 and int(step) == 0  # warm-up and capture restored the state
    for _ in range(3):
        r1.replay()
    torch.cuda.synchronize()
    assert torch.allclose(acc, torch.full((4,), 9.0, device=DEV)) and int(step) == 3
    fn2, d2 = make(-1.0)
    r2.capture(fn2, "b", keep=(d2,), restore=[acc, step])
    r2.replay()
    r1.replay()
    torch.cuda.synchronize()
    assert torch.allclose(acc, torch.full((4,), 10.0, device=DEV)) and int(step) == 5
    assert not r1.needs("a") and r1.needs("c")
    assert runtime.graph_pool() == runtime.graph_pool(DEV)


def test_split_k_tickets_return_to_zero_after_generation():
    """Race detector for the in-launch split-K hand-off: every arrival ticket of every per-stream
    decode workspace is back at zero after graph-replayed generations (a launch that raced another
    on a shared workspace, or lost an arrival, leaves a non-zero count behind)."""
    from rag_tl_domainllm_optimizer_amd.ops import native

    cfg = PRESETS["tiny-llama"]
    m = models.CausalLM(cfg, device=DEV, dtype=torch.bfloat16, seed=3)
    for B in (1, 4, 40):
        gen = Generator(m, max_batch=B, max_seq=96, device=DEV)
        prompts = [[5 + i, 9, 33, 41, 7][: 3 + i % 3] for i in range(B)]
        for _ in range(2):
            gen.generate(prompts, SamplingParams(max_new_tokens=10, temperature=0.9), pad_id=0, eos_ids=[-1])
    torch.cuda.synchronize()
    dirty = native().decode_ws_dirty_tickets()
    assert len(dirty) >= 1 and all(d == 0 for d in dirty), dirty


def test_side_stream_is_high_priority():
    from rag_tl_domainllm_optimizer_amd.runtime import StreamPair

    sp = StreamPair(DEV)
    lo, hi = torch.cuda.Stream.priority_range()
    assert sp.side.priority == hi and hi < lo


def test_continuous_batching_gpu_matches_teacher_forcing():
    """Requests admitted into a running graph-replayed decode batch: every row's behaviour
    log-probs equal a teacher-forced rescoring of its own prompt + tokens (rows independent)."""
    from rag_tl_domainllm_optimizer_amd.generation import ContinuousBatcher
    from rag_tl_domainllm_optimizer_amd.train.common import score_sequences

    cfg = PRESETS["tiny-mistral"]
    m = models.CausalLM(cfg, device=DEV, dtype=torch.bfloat16, seed=4)
    p = SamplingParams(max_new_tokens=10, temperature=0.7, top_k=0, seed=5)
    prompts = [[5, 9, 33, 41, 7, 8, 9, 10], [12, 300, 4], list(range(20, 60)), [7, 7, 7, 7], list(range(100, 130))]
    cb = ContinuousBatcher(Generator(m, 2, 96, DEV), p, pad_id=0, eos_ids=[-1])
    pending, got = list(enumerate(prompts)), {}
    while pending or cb.active_rows():
        if pending and cb.free_rows():
            i, pr = pending.pop(0)
            cb.admit(pr, i)
        cb.step(3)
        for f in cb.collect():
            got[f.tag] = f
    cb.close()
    for i, pr in enumerate(prompts):
        f = got[i]
        assert len(f.tokens) == 10
        ids = torch.tensor([pr], device=DEV)
        resp = torch.tensor([f.tokens], device=DEV)
        with torch.no_grad():
            lp, _, _, _ = score_sequences(m, ids, torch.zeros(1, dtype=torch.long, device=DEV), resp,
                                          torch.tensor([10], device=DEV), 1 / 0.7)
        torch.testing.assert_close(lp[0].cpu(), torch.tensor(f.logprobs), rtol=0.0, atol=1e-2)
