"""Dynamic request batching in front of the RAG pipeline (serve.batching.BatchingEngine)."""
import threading
import time

import pytest
import torch

from rag_tl_domainllm_optimizer_amd.rag import RagAnswer
from rag_tl_domainllm_optimizer_amd.serve.batching import BatchingEngine


class RecordingPipe:
    """Stands in for RagPipeline: records every batch, answers "<query>|k=<top_k>"."""
    docs = ["d0", "d1", "d2"]
    top_k = 2

    def __init__(self, max_batch=8, delay=0.02, fail_on=None):
        self.max_batch, self.delay, self.fail_on = max_batch, delay, fail_on
        self.batches = []

    def answer(self, qs, top_ks=None):
        self.batches.append(list(qs))
        time.sleep(self.delay)
        if self.fail_on and self.fail_on in qs:
            raise ValueError("boom")
        ks = top_ks or [None] * len(qs)
        return [RagAnswer(q, f"{q}|k={k or self.top_k}", [0], ["d0"], [1.0], {"total_s": self.delay})
                for q, k in zip(qs, ks)]


def test_concurrent_requests_are_batched_and_routed():
    pipe = RecordingPipe(max_batch=8, delay=0.05)
    with BatchingEngine(pipe, max_wait_s=0.02) as eng:
        res = {}

        def client(i):
            res[i] = eng.answer(f"q{i}", top_k=(i % 3) or None, timeout=10)

        ts = [threading.Thread(target=client, args=(i,)) for i in range(20)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    assert sorted(res) == list(range(20))
    for i, a in res.items():  # every caller gets its own answer, with its own top_k
        assert a.query == f"q{i}" and a.answer == f"q{i}|k={(i % 3) or 2}"
        assert a.timings["queue_s"] >= 0 and 1 <= a.timings["batch_size"] <= 8
    assert all(len(b) <= 8 for b in pipe.batches)
    assert len(pipe.batches) < 20  # 20 concurrent requests did not run one by one
    assert eng.stats["requests"] == 20 and eng.stats["max_batch_seen"] > 1


def test_batch_error_reaches_every_caller_and_engine_survives():
    pipe = RecordingPipe(max_batch=4, delay=0.0, fail_on="bad")
    with BatchingEngine(pipe, max_wait_s=0.05) as eng:
        f1, f2 = eng.submit("bad"), eng.submit("ok1")
        for f in (f1, f2):
            with pytest.raises(ValueError):
                f.result(10)
        assert eng.answer("ok2", timeout=10).answer == "ok2|k=2"


def test_close_fails_queued_requests_and_rejects_new_ones():
    pipe = RecordingPipe(max_batch=1, delay=0.2)
    eng = BatchingEngine(pipe, max_wait_s=0.0)
    futs = [eng.submit(f"q{i}") for i in range(4)]
    time.sleep(0.05)
    eng.close()
    done = [f for f in futs if f.done() and f.exception() is None]
    assert len(done) >= 1  # the running batch finished
    for f in futs:
        assert f.done()
    with pytest.raises(RuntimeError):
        eng.submit("late")


def test_engine_over_real_pipeline_cpu():
    """Tiny models on the CPU: answers through the engine equal a direct batched call."""
    from rag_tl_domainllm_optimizer_amd import models
    from rag_tl_domainllm_optimizer_amd.generation import SamplingParams
    from rag_tl_domainllm_optimizer_amd.rag import RagPipeline
    from rag_tl_domainllm_optimizer_amd.retrieval import Encoder, FlatIndex
    from rag_tl_domainllm_optimizer_amd.tokenizer import Tokenizer

    torch.manual_seed(0)
    pol = models.CausalLM(models.resolve_preset("tiny-llama"), device="cpu", dtype=torch.float32, seed=1)
    enc_m = models.build_model("tiny-bert", device="cpu", dtype=torch.float32, seed=2).eval()
    tok = Tokenizer.synthetic(pol.cfg.vocab_size, pol.cfg.arch)
    enc = Encoder(enc_m, Tokenizer.synthetic(enc_m.cfg.vocab_size, enc_m.cfg.arch), max_length=32)
    words = tok.words()
    docs = [" ".join(words[(7 * i + j) % len(words)] for j in range(12)) for i in range(30)]
    index = FlatIndex(enc.dim, "ip", "cpu")
    index.add(enc.encode(docs))
    pipe = RagPipeline(enc, index, docs, pol, tok, top_k=2,
                       sampling=SamplingParams(max_new_tokens=4, do_sample=False), max_prompt_tokens=96,
                       max_batch=4, use_graph=False)
    qs = [f"{words[i]} {words[i + 3]}" for i in range(4)]
    direct = pipe.answer(qs)
    with BatchingEngine(pipe, max_wait_s=0.2) as eng:
        futs = [eng.submit(q) for q in qs]
        got = [f.result(60) for f in futs]
    assert [a.answer for a in got] == [a.answer for a in direct]
    assert [a.doc_ids for a in got] == [a.doc_ids for a in direct]


def _tiny_pipe(max_batch=2, new=5):
    from rag_tl_domainllm_optimizer_amd import models
    from rag_tl_domainllm_optimizer_amd.generation import SamplingParams
    from rag_tl_domainllm_optimizer_amd.rag import RagPipeline
    from rag_tl_domainllm_optimizer_amd.retrieval import Encoder, FlatIndex
    from rag_tl_domainllm_optimizer_amd.tokenizer import Tokenizer

    pol = models.CausalLM(models.resolve_preset("tiny-llama"), device="cpu", dtype=torch.float32, seed=1)
    enc_m = models.build_model("tiny-bert", device="cpu", dtype=torch.float32, seed=2).eval()
    tok = Tokenizer.synthetic(pol.cfg.vocab_size, pol.cfg.arch)
    enc = Encoder(enc_m, Tokenizer.synthetic(enc_m.cfg.vocab_size, enc_m.cfg.arch), max_length=32)
    words = tok.words()
    docs = [" ".join(words[(7 * i + j) % len(words)] for j in range(12)) for i in range(30)]
    index = FlatIndex(enc.dim, "ip", "cpu")
    index.add(enc.encode(docs))
    pipe = RagPipeline(enc, index, docs, pol, tok, top_k=2, sampling=SamplingParams(max_new_tokens=new, do_sample=False),
                       max_prompt_tokens=96, max_batch=max_batch, use_graph=False)
    return pipe, words


def test_continuous_batcher_matches_one_at_a_time_greedy():
    """Rows admitted into a running batch (2 rows, 4 requests, staggered) decode exactly what a
    batch-1 generation of the same prompt does."""
    from rag_tl_domainllm_optimizer_amd import models
    from rag_tl_domainllm_optimizer_amd.generation import ContinuousBatcher, Generator, SamplingParams

    m = models.CausalLM(models.resolve_preset("tiny-llama"), device="cpu", dtype=torch.float32, seed=3)
    p = SamplingParams(max_new_tokens=6, do_sample=False)
    prompts = [[5, 9, 33, 41, 7], [12, 300, 4, 8, 9, 10, 11], [20, 21, 22], [100, 200, 300, 400]]
    ref = [Generator(m, 1, 64, "cpu", use_graph=False).generate([pr], p, pad_id=0, eos_ids=[-1]).tokens[0].tolist()
           for pr in prompts]
    cb = ContinuousBatcher(Generator(m, 2, 64, "cpu", use_graph=False), p, pad_id=0, eos_ids=[-1])
    pending, got, admitted_at = list(enumerate(prompts)), {}, {}
    while pending or cb.active_rows():
        if pending and cb.free_rows():  # one admission per step: rows join a batch in flight
            i, pr = pending.pop(0)
            cb.admit(pr, i)
            admitted_at[i] = cb.steps
        cb.step(1)
        for f in cb.collect():
            got[f.tag] = f.tokens
    assert [got[i] for i in range(4)] == ref
    assert admitted_at[1] > admitted_at[0]  # the second request joined after the first had started
    cb.close()


def test_continuous_engine_answers_like_direct_pipeline():
    from rag_tl_domainllm_optimizer_amd.serve import ContinuousEngine

    pipe, words = _tiny_pipe(max_batch=2)
    qs = [f"{words[i]} {words[i + 3]}" for i in range(5)]
    direct = [pipe.answer([q])[0] for q in qs]  # one at a time
    with ContinuousEngine(pipe, chunk=2) as eng:
        futs = [eng.submit(q) for q in qs]
        got = [f.result(120) for f in futs]
        assert eng.stats["finished"] == 5 and eng.stats["max_active"] <= 2
    assert [a.answer for a in got] == [a.answer for a in direct]
    assert [a.doc_ids for a in got] == [a.doc_ids for a in direct]
    assert all(a.timings["new_tokens"] == 5 and a.timings["queue_s"] >= 0 for a in got)
    # mean decode batch over each answer's lifetime: between 1 and the 2 serving rows
    assert all(1.0 <= a.timings["batch_size"] <= 2.0 for a in got), [a.timings["batch_size"] for a in got]


def test_continuous_admit_many_batches_consecutive_rows():
    from rag_tl_domainllm_optimizer_amd import models
    from rag_tl_domainllm_optimizer_amd.generation import ContinuousBatcher, Generator, SamplingParams

    m = models.CausalLM(models.resolve_preset("tiny-llama"), device="cpu", dtype=torch.float32, seed=3)
    p = SamplingParams(max_new_tokens=5, do_sample=False)
    prompts = [[5, 9, 33, 41, 7], [12, 300, 4], [20, 21, 22, 23, 24, 25, 26], [100, 200]]
    ref = [Generator(m, 1, 64, "cpu", use_graph=False).generate([pr], p, pad_id=0, eos_ids=[-1]).tokens[0].tolist()
           for pr in prompts]
    cb = ContinuousBatcher(Generator(m, 4, 64, "cpu", use_graph=False), p, pad_id=0, eos_ids=[-1])
    rows = cb.admit_many(prompts, list(range(4)))  # one left-padded prefill over rows 0..3
    assert rows == [0, 1, 2, 3]
    got = {}
    while cb.active_rows():
        cb.step(2)
        for f in cb.collect():
            got[f.tag] = f.tokens
    assert [got[i] for i in range(4)] == ref


def test_continuous_admit_many_rolls_back_on_failure():
    """A prefill failure in the second run of rows releases the first run's rows too (no row keeps
    decoding for a request whose future the engine is about to fail)."""
    from rag_tl_domainllm_optimizer_amd import models
    from rag_tl_domainllm_optimizer_amd.generation import ContinuousBatcher, Generator, SamplingParams

    m = models.CausalLM(models.resolve_preset("tiny-llama"), device="cpu", dtype=torch.float32, seed=3)
    p = SamplingParams(max_new_tokens=4, do_sample=False)
    cb = ContinuousBatcher(Generator(m, 4, 64, "cpu", use_graph=False), p, pad_id=0, eos_ids=[-1])
    cb.admit([5, 6, 7], "held")  # row 0
    cb.free = [1, 3]  # row 2 withheld: the next admission is two runs of rows, [1] and [3]
    calls = {"n": 0}
    orig = m.prefill

    def flaky(*a, **k):
        calls["n"] += 1
        if calls["n"] == 2:
            raise RuntimeError("boom")
        return orig(*a, **k)

    m.prefill = flaky
    with pytest.raises(RuntimeError, match="boom"):
        cb.admit_many([[9, 10], [11, 12, 13]], ["a", "b"])
    m.prefill = orig
    assert set(cb.rows) == {0} and sorted(cb.free) == [1, 3]
    assert int(cb.gen.active[1]) == 0 and int(cb.gen.active[3]) == 0
    cb.close()


def test_continuous_engine_worker_failure_fails_closed():
    """If the worker loop dies, in-flight and queued requests fail and later submits raise instead of
    returning futures nothing would ever resolve."""
    from rag_tl_domainllm_optimizer_amd.generation import ContinuousBatcher
    from rag_tl_domainllm_optimizer_amd.serve import ContinuousEngine

    pipe, words = _tiny_pipe(max_batch=2)
    orig_step = ContinuousBatcher.step

    def bad_step(self, n=1):
        raise RuntimeError("gpu went away")

    ContinuousBatcher.step = bad_step
    try:
        eng = ContinuousEngine(pipe, chunk=2)
        fut = eng.submit(f"{words[0]} {words[3]}")
        with pytest.raises(RuntimeError, match="gpu went away"):
            fut.result(60)
        eng._worker.join(30)
        assert not eng.alive
        with pytest.raises(RuntimeError, match="worker failed"):
            eng.submit("another")
        eng.close()
    finally:
        ContinuousBatcher.step = orig_step
