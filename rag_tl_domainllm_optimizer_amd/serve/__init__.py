"""Minimal HTTP answer service (the README's optional frontend, README.md:9,31: Streamlit / Gradio
are not installed; FastAPI + uvicorn are). POST /answer {"query": "...", "top_k": 3} ->
{"answer", "doc_ids", "docs", "scores", "timings"}; GET /health."""

from typing import Optional


def create_app(pipeline):
    from fastapi import FastAPI
    from pydantic import BaseModel

    app = FastAPI(title="rag-tl-domainllm-optimizer-amd")

    class Query(BaseModel):
        query: str
        top_k: Optional[int] = None

    @app.get("/health")
    def health():
        return {"status": "ok", "docs": len(pipeline.docs)}

    @app.post("/answer")
    def answer(q: Query):
        if q.top_k:
            pipeline.top_k = q.top_k
        a = pipeline.answer([q.query])[0]
        return {"answer": a.answer, "doc_ids": a.doc_ids, "docs": a.docs, "scores": a.scores, "timings": a.timings}

    return app


def serve(cfg, host: str = "127.0.0.1", port: int = 8000):
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
                      cfg.ppo.max_prompt_tokens)
    uvicorn.run(create_app(rag), host=host, port=port)
