"""HTTP answer service (the README's optional frontend, README.md:9,31: Streamlit / Gradio are not
installed; FastAPI + uvicorn are). POST /answer {"query": "...", "top_k": 3} ->
{"answer", "doc_ids", "docs", "scores", "timings"}; GET /health; GET /stats.

Concurrent requests are batched: the async handler awaits a future while one worker thread owns the
GPU — by default ``serve.continuous.ContinuousEngine`` (requests join the running decode batch
between steps), or ``serve.batching.BatchingEngine`` (batches formed per request group and run to
completion)."""

from typing import Optional

from .batching import BatchingEngine  # noqa: F401
from .continuous import ContinuousEngine  # noqa: F401


def create_app(pipeline, max_wait_s: float = 0.004, continuous: bool = False):
    import asyncio

    from fastapi import FastAPI
    from pydantic import BaseModel

    engine = ContinuousEngine(pipeline) if continuous else BatchingEngine(pipeline, max_wait_s=max_wait_s)
    app = FastAPI(title="rag-tl-domainllm-optimizer-amd")
    app.state.engine = engine

    class Query(BaseModel):
        query: str
        top_k: Optional[int] = None

    @app.get("/health")
    def health():
        return {"status": "ok", "docs": len(pipeline.docs), "max_batch": pipeline.max_batch,
                "batching": "continuous" if continuous else "dynamic"}

    @app.get("/stats")
    def stats():
        return dict(engine.stats)

    @app.post("/answer")
    async def answer(q: Query):
        a = await asyncio.wrap_future(engine.submit(q.query, q.top_k))
        return {"answer": a.answer, "doc_ids": a.doc_ids, "docs": a.docs, "scores": a.scores, "timings": a.timings}

    @app.on_event("shutdown")
    def _shutdown():
        engine.close()

    return app


def serve(cfg, host: str = "127.0.0.1", port: int = 8000, max_batch: int = 16, max_wait_s: float = 0.004,
          continuous: bool = True):
    import uvicorn

    from ..cli import build_stack
    from ..generation import SamplingParams
    from ..parallel import init
    from ..rag import RagPipeline

    di = init()
    st = build_stack(cfg, di.device)
    sp = SamplingParams(max_new_tokens=cfg.ppo.max_new_tokens, temperature=cfg.eval.temperature,
                        do_sample=cfg.eval.do_sample, top_k=cfg.eval.top_k)
    rag = RagPipeline(st["encoder"], st["index"], st["docs"], st["policy"], st["tokenizer"], cfg.retrieval.top_k, sp,
                      cfg.ppo.max_prompt_tokens, max_batch=max_batch)
    uvicorn.run(create_app(rag, max_wait_s, continuous), host=host, port=port)
