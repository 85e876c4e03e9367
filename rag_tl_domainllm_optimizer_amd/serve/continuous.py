"""Continuous (iteration-level) batching for RAG answering.

Where ``BatchingEngine`` forms a batch and runs it to completion, ``ContinuousEngine`` keeps one
decode batch running: between chunks of ``chunk`` graph-replayed decode steps the worker thread
admits queued requests into free rows (one batched retrieval for the newcomers, then a per-row
prefill, ``generation.ContinuousBatcher``) and hands finished rows back to their callers. A new
request waits for at most one chunk plus its prefill instead of a whole in-flight generation, and
the batch stays full under load.

Same client API as ``BatchingEngine``: ``submit`` -> Future[RagAnswer], ``answer``, ``answer_many``,
``close``. ``timings``: ``queue_s`` (submit -> admission), ``total_s`` (submit -> answer),
``retrieve_s``, ``new_tokens``, ``prompt_tokens``, ``decode_steps`` (steps the row was in flight).
"""
from __future__ import annotations

import concurrent.futures as cf
import queue
import threading
import time
from typing import List, Optional

import torch

from ..generation import ContinuousBatcher
from ..rag.pipeline import RagAnswer
from ..rag.prompt import extract_answer


class ContinuousEngine:
    def __init__(self, pipeline, chunk: int = 4):
        self.pipeline = pipeline
        self.chunk = max(1, chunk)
        self._q: "queue.Queue" = queue.Queue()
        self._closed = False
        self._dead: Optional[BaseException] = None  # the error that ended the worker, if any
        self._lock = threading.Lock()  # submit's closed-check + put vs the worker's final drain
        self.stats = {"admitted": 0, "finished": 0, "steps": 0, "max_active": 0}
        self._row_steps = 0  # sum over decode steps of the active rows (an answer's mean batch)
        self._ready = threading.Event()
        self._init_error = None
        self._worker = threading.Thread(target=self._loop, name="rag-continuous", daemon=True)
        self._worker.start()
        self._ready.wait()
        if self._init_error is not None:
            raise self._init_error

    # ---------------------------------------------------------------- client side
    def submit(self, query: str, top_k: Optional[int] = None) -> cf.Future:
        with self._lock:
            if self._closed:
                if self._dead is not None:
                    raise RuntimeError(f"ContinuousEngine worker failed: {self._dead!r}") from self._dead
                raise RuntimeError("ContinuousEngine is closed")
            fut: cf.Future = cf.Future()
            self._q.put((query, top_k, fut, time.perf_counter()))
        return fut

    @property
    def alive(self) -> bool:
        return not self._closed and self._worker.is_alive()

    def answer(self, query: str, top_k: Optional[int] = None, timeout: Optional[float] = None) -> RagAnswer:
        return self.submit(query, top_k).result(timeout)

    def answer_many(self, queries: List[str], timeout: Optional[float] = None) -> List[RagAnswer]:
        futs = [self.submit(q) for q in queries]
        return [f.result(timeout) for f in futs]

    def close(self, timeout: Optional[float] = 60.0):
        with self._lock:
            was_open, self._closed = not self._closed, True
        if was_open:
            self._q.put(None)
        self._worker.join(timeout)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---------------------------------------------------------------- worker
    def _admit(self, cb: ContinuousBatcher, items):
        p = self.pipeline
        live = [it for it in items if it[2].set_running_or_notify_cancel()]
        if not live:
            return
        t0 = time.perf_counter()
        try:
            ks = [it[1] or p.top_k for it in live]
            scores, ids = p.retrieve([it[0] for it in live], max(ks))
            ids_l = [row[:k] for row, k in zip(ids.tolist(), ks)]
            sc_l = [row[:k] for row, k in zip(scores.tolist(), ks)]
        except BaseException as e:  # noqa: BLE001
            for it in live:
                it[2].set_exception(e)
            return
        t1 = time.perf_counter()
        prompts, metas = [], []
        for it, row_ids, row_sc in zip(live, ids_l, sc_l):
            docs = [p.docs[i] for i in row_ids if i >= 0]
            prompt = p._prompt_ids(it[0], docs)
            if len(prompt) + cb.T > p.gen.max_seq:
                it[2].set_exception(ValueError("prompt does not fit the serving cache"))
                continue
            prompts.append(prompt)
            metas.append({"query": it[0], "fut": it[2], "t_submit": it[3], "t_admit": time.perf_counter(),
                          "retrieve_s": t1 - t0, "doc_ids": row_ids, "docs": docs, "scores": row_sc,
                          "rows0": (self._row_steps, self.stats["steps"])})
        if not prompts:
            return
        try:
            cb.admit_many(prompts, metas)  # consecutive free rows share one prefill
        except BaseException as e:  # noqa: BLE001
            for m in metas:
                m["fut"].set_exception(e)
            return
        self.stats["admitted"] += len(prompts)

    def _finish(self, rows):
        p = self.pipeline
        now = time.perf_counter()
        for r in rows:
            m = r.tag
            if m["fut"].done():  # failed or cancelled elsewhere: nothing to deliver
                continue
            text = extract_answer(p.tok.decode(r.tokens))
            rs0, st0 = m["rows0"]
            steps = self.stats["steps"] - st0
            tim = {"queue_s": m["t_admit"] - m["t_submit"], "retrieve_s": m["retrieve_s"],
                   "total_s": now - m["t_submit"], "new_tokens": len(r.tokens), "prompt_tokens": r.prompt_len,
                   "decode_steps": r.steps_waited,
                   "batch_size": (self._row_steps - rs0) / steps if steps > 0 else 0.0}
            m["fut"].set_result(RagAnswer(m["query"], text, m["doc_ids"], m["docs"], m["scores"], tim))
            self.stats["finished"] += 1

    def _loop(self):
        p = self.pipeline
        try:
            cb = ContinuousBatcher(p.gen, p.sampling, pad_id=p.tok.pad_token_id, eos_ids=[p.tok.eos_token_id])
        except BaseException as e:  # noqa: BLE001
            self._init_error = e
            self._ready.set()
            return
        self._ready.set()
        stop = False
        try:
            with torch.no_grad():
                while True:
                    # admissions: block only when nothing is in flight
                    new = []
                    while not stop and len(new) < cb.free_rows():
                        try:
                            item = self._q.get(timeout=0.1) if (cb.active_rows() == 0 and not new) else \
                                self._q.get_nowait()
                        except queue.Empty:
                            break
                        if item is None:
                            stop = True
                            break
                        new.append(item)
                    if new:
                        self._admit(cb, new)
                    if cb.active_rows() == 0:
                        if stop:
                            break
                        continue
                    self.stats["max_active"] = max(self.stats["max_active"], cb.active_rows())
                    self._row_steps += cb.active_rows() * self.chunk
                    cb.step(self.chunk)
                    self.stats["steps"] += self.chunk
                    self._finish(cb.collect())
        except BaseException as e:  # noqa: BLE001 - in-flight callers get the error
            self._dead = e
            for b, (meta, _, _) in list(cb.rows.items()):
                if not meta["fut"].done():
                    meta["fut"].set_exception(e)
            cb.rows.clear()
        finally:
            # the worker is gone for good: later submits raise instead of queueing futures nothing
            # would resolve, and whatever is queued now fails
            with self._lock:
                self._closed = True
                pending = []
                while True:
                    try:
                        pending.append(self._q.get_nowait())
                    except queue.Empty:
                        break
            cb.close()
            err = RuntimeError(f"ContinuousEngine worker failed: {self._dead!r}" if self._dead is not None
                               else "ContinuousEngine closed")
            for item in pending:
                if item is not None and item[2].set_running_or_notify_cancel():
                    item[2].set_exception(err)
