"""FastAPI application — the reference's REST surface (rest_api/src/app/main.py,
controllers/jobs_controller.py, health.py) plus the
OpenAI-compatible LLM endpoints the reference reached on its vLLM pod
(helm/templates/qwen-deployment.yaml; qwen_llm.py:119) and an embeddings
endpoint, all served in-process:

  POST /rag/jobs                 -> {"job_id"}            (C1)
  GET  /rag/jobs/{id}/events     -> text/event-stream     (C2)
  POST /rag/jobs/{id}/cancel     -> {"status":"cancelling","job_id"} (C3)
  GET  /rag/jobs/{id}            -> job status + events so far (new)
  GET  /health, GET /metrics, GET /static/index.html       (C4-C6)
  POST /v1/chat/completions, POST /v1/completions, GET /v1/models,
  POST /v1/embeddings, GET /v1/health                      (C11)
  POST /ingest                   -> background ingest job (new)
"""
from __future__ import annotations

import asyncio
import contextlib
import json
import logging
import time
import uuid
from pathlib import Path

from fastapi import FastAPI, HTTPException, Request, Response
from fastapi.middleware.cors import CORSMiddleware
from fastapi.staticfiles import StaticFiles
from starlette.responses import StreamingResponse

from ..utils.gpu_guard import gpu_shared
from . import metrics as M
from .events import CancelFlags, EventLog
from .health import _get_app_start_time, register_health_endpoints
from .models import ChatCompletionRequest, CompletionRequest, EmbeddingRequest, QueryRequest

log = logging.getLogger(__name__)
STATIC_DIR = Path(__file__).resolve().parent / "static"


class APIState:
    def __init__(self, runtime=None, queue=None, events: EventLog | None = None, flags: CancelFlags | None = None,
                 ping_seconds: float = 15.0):
        self.runtime = runtime
        self.queue = queue
        self.events = events or EventLog()
        self.flags = flags or CancelFlags()
        self.ping_seconds = ping_seconds


def create_app(state: APIState | None = None, runtime_factory=None) -> FastAPI:
    state = state or APIState()

    @contextlib.asynccontextmanager
    async def lifespan(_app):
        await _startup()
        yield

    app = FastAPI(title="RAG API Service", description="MI355X-native code RAG (in-process GPU engine)",
                  version="2.0.0", lifespan=lifespan)
    app.state.api = state
    app.add_middleware(CORSMiddleware, allow_origins=["*"], allow_credentials=True, allow_methods=["*"],
                       allow_headers=["*"])

    @app.middleware("http")
    async def metrics_middleware(request: Request, call_next):
        start = time.perf_counter()
        response: Response = await call_next(request)
        route = request.scope.get("route")
        labels = {"method": request.method, "path": route.path if route else request.url.path,
                  "status": str(response.status_code)}
        M.REQUEST_COUNT.labels(**labels).inc()
        M.REQUEST_LATENCY.labels(**labels).observe(time.perf_counter() - start)
        return response

    async def _startup():  # runtime (built off the event loop), job worker, queue
        _get_app_start_time()
        if state.runtime is None and runtime_factory is not None:
            loop = asyncio.get_running_loop()
            state.runtime = await loop.run_in_executor(None, runtime_factory)
        if state.queue is None and state.runtime is not None:
            from .worker import RAGWorker

            s = state.runtime.settings
            worker = RAGWorker(state.runtime, state.events, state.flags, s.worker_max_jobs, s.job_timeout_s,
                               s.keep_result_s, s.stream_tokens)
            state.queue = worker.queue
        if state.queue is not None and hasattr(state.queue, "start"):
            await state.queue.start()

    @app.get("/metrics")
    async def metrics():
        return Response(M.render(), media_type="text/plain; version=0.0.4; charset=utf-8")

    if STATIC_DIR.exists():
        app.mount("/static", StaticFiles(directory=str(STATIC_DIR)), name="static")

    # ------------------------------------------------------------------ jobs
    @app.post("/rag/jobs")
    async def create_job(req: QueryRequest):
        if state.queue is None:
            raise HTTPException(503, "worker queue not ready")
        job_id = uuid.uuid4().hex
        body = req.model_dump()
        if "top_k" not in req.model_fields_set:
            body["top_k"] = None  # only an explicit top_k caps the retrieved documents
        await state.queue.enqueue_job("run_rag_job", job_id, body, _job_id=job_id)
        return {"job_id": job_id}

    @app.get("/rag/jobs/{job_id}/events")
    async def job_events(job_id: str):
        async def gen():
            async for chunk in state.events.stream(job_id, state.ping_seconds):
                yield chunk

        return StreamingResponse(gen(), media_type="text/event-stream",
                                 headers={"Cache-Control": "no-cache", "X-Accel-Buffering": "no"})

    @app.post("/rag/jobs/{job_id}/cancel")
    async def cancel_job(job_id: str):
        await state.flags.cancel(job_id)
        return {"status": "cancelling", "job_id": job_id}

    @app.get("/rag/jobs/{job_id}")
    async def job_status(job_id: str):
        evs = state.events.events(job_id)
        final = next((e["data"] for e in evs if e["event"] == "final"), None)
        return {"job_id": job_id, "done": final is not None, "final": final, "events": len(evs)}

    register_health_endpoints(app, lambda: state.runtime)

    # ------------------------------------------------------------------ OpenAI-compatible LLM
    def _runner():
        rt = state.runtime
        if rt is None or getattr(rt, "runner", None) is None:
            raise HTTPException(503, "LLM engine not available in this process")
        return rt

    @app.get("/v1/models")
    async def models():
        rt = state.runtime
        name = rt.settings.qwen_model if rt is not None else "unloaded"
        return {"object": "list", "data": [{"id": name, "object": "model", "owned_by": "githubrepostorag_amd"}]}

    @app.get("/v1/health")
    async def llm_health():
        rt = _runner()
        if not rt.runner.healthy:
            raise HTTPException(503, str(rt.runner.last_error))
        return {"status": "ok"}

    def _params(rt, body):
        from ..engine.sequence import SamplingParams

        stop = body.stop if isinstance(body.stop, list) else ([body.stop] if body.stop else [])
        mt = getattr(body, "max_completion_tokens", None) or body.max_tokens
        sp = SamplingParams(max_tokens=int(mt or rt.settings.qwen_max_output), temperature=body.temperature if body.temperature is not None else 0.7,
                              top_p=body.top_p if body.top_p is not None else 1.0,
                              top_k=getattr(body, "top_k", 0) or 0,
                              repetition_penalty=getattr(body, "repetition_penalty", None) or 1.0, stop=stop,
                              seed=getattr(body, "seed", None))
        sp.max_tokens_explicit = bool(mt)  # vLLM: an unset max_tokens means "up to max_model_len"
        return sp

    async def _generate(rt, text, sp, stream: bool, model: str, chat: bool):
        loop = asyncio.get_running_loop()
        # vLLM's contract (reference server flags, helm/templates/qwen-deployment.yaml:30-31): a prompt that
        # does not fit max_model_len is a 400, never a silently shortened prompt
        ids = rt.tokenizer.encode(text)
        eng = getattr(rt.runner, "engine", None)
        mml = getattr(getattr(eng, "cfg", None), "max_model_len", None)
        if mml and len(ids) >= mml:
            from ..engine.llm_engine import PromptTooLongError

            raise HTTPException(400, str(PromptTooLongError(len(ids), mml)))
        if mml:
            if not getattr(sp, "max_tokens_explicit", True):
                sp.max_tokens = mml - len(ids)
            elif len(ids) + sp.max_tokens > mml:  # vLLM's check: prompt + requested completion must fit
                raise HTTPException(400, f"This model's maximum context length is {mml} tokens. However, you "
                                         f"requested {len(ids) + sp.max_tokens} tokens ({len(ids)} in the messages, "
                                         f"{sp.max_tokens} in the completion). Please reduce the length of the "
                                         "messages or completion.")
        text = ids
        rid = f"{'chatcmpl' if chat else 'cmpl'}-{uuid.uuid4().hex}"
        created = int(time.time())
        if not stream:
            c = await loop.run_in_executor(None, lambda: rt.runner.generate(text, sp, timeout=rt.settings.job_timeout_s))
            usage = {"prompt_tokens": c.prompt_tokens, "completion_tokens": len(c.token_ids),
                     "total_tokens": c.prompt_tokens + len(c.token_ids)}
            if chat:
                return {"id": rid, "object": "chat.completion", "created": created, "model": model,
                        "choices": [{"index": 0, "message": {"role": "assistant", "content": c.text},
                                     "finish_reason": c.finish_reason}], "usage": usage}
            return {"id": rid, "object": "text_completion", "created": created, "model": model,
                    "choices": [{"index": 0, "text": c.text, "finish_reason": c.finish_reason}], "usage": usage}
        q: asyncio.Queue = asyncio.Queue()

        def on_tok(delta):
            loop.call_soon_threadsafe(q.put_nowait, ("tok", delta))

        h = rt.runner.submit(text, sp, on_token=on_tok)

        def waiter():
            try:
                c = h.wait(rt.settings.job_timeout_s)
                loop.call_soon_threadsafe(q.put_nowait, ("end", c.finish_reason))
            except Exception as e:  # pragma: no cover
                loop.call_soon_threadsafe(q.put_nowait, ("end", f"error: {e}"))

        loop.run_in_executor(None, waiter)

        async def gen():
            obj = "chat.completion.chunk" if chat else "text_completion"
            while True:
                kind, val = await q.get()
                if kind == "tok":
                    ch = {"index": 0, "delta": {"content": val}} if chat else {"index": 0, "text": val}
                    yield f"data: {json.dumps({'id': rid, 'object': obj, 'created': created, 'model': model, 'choices': [ch]})}\n\n"
                else:
                    ch = {"index": 0, "delta": {}, "finish_reason": val} if chat else \
                        {"index": 0, "text": "", "finish_reason": val}
                    yield f"data: {json.dumps({'id': rid, 'object': obj, 'created': created, 'model': model, 'choices': [ch]})}\n\n"
                    yield "data: [DONE]\n\n"
                    return

        return StreamingResponse(gen(), media_type="text/event-stream")

    @app.post("/v1/chat/completions")
    async def chat_completions(body: ChatCompletionRequest):
        rt = _runner()
        kw = body.chat_template_kwargs or {}
        text = rt.tokenizer.apply_chat_template([m.model_dump() for m in body.messages], True,
                                                kw.get("enable_thinking"))
        return await _generate(rt, text, _params(rt, body), bool(body.stream), body.model or rt.settings.qwen_model,
                               True)

    @app.post("/v1/completions")
    async def completions(body: CompletionRequest):
        rt = _runner()
        return await _generate(rt, body.prompt, _params(rt, body), False, body.model or rt.settings.qwen_model, False)

    @app.post("/v1/embeddings")
    async def embeddings(body: EmbeddingRequest):
        rt = state.runtime
        if rt is None:
            raise HTTPException(503, "runtime not ready")
        texts = [body.input] if isinstance(body.input, str) else list(body.input)
        loop = asyncio.get_running_loop()
        def _embed():
            with gpu_shared():  # the .cpu() sync must not land inside an engine graph capture
                return rt.embedder.embed_documents(texts).float().cpu().tolist()

        vecs = await loop.run_in_executor(None, _embed)
        return {"object": "list", "model": rt.settings.embed_model,
                "data": [{"object": "embedding", "index": i, "embedding": v} for i, v in enumerate(vecs)]}

    # ------------------------------------------------------------------ ingest trigger
    # The reference exposes no HTTP ingest (its ingest is a batch Job); this
    # route is OFF unless HTTP_INGEST=1, and a `local` source is confined to
    # INGEST_ROOT (checked after resolve(), so `..` and symlinks cannot escape).
    @app.post("/ingest")
    async def ingest(payload: dict):
        from ..config import settings as _settings

        cfg = _settings()
        if not cfg.http_ingest:
            raise HTTPException(403, "HTTP ingest is disabled (set HTTP_INGEST=1 to enable)")
        rt = state.runtime
        if rt is None:
            raise HTTPException(503, "runtime not ready")
        source = payload.get("source", "synthetic")
        if source not in ("synthetic", "github", "local"):
            raise HTTPException(400, f"unknown ingest source {source!r}")
        path = payload.get("path")
        if source == "local":
            if not cfg.ingest_root or not path:
                raise HTTPException(403, "local ingest needs INGEST_ROOT and a path under it")
            root = Path(cfg.ingest_root).resolve()
            target = (root / path).resolve()
            if target != root and root not in target.parents:
                raise HTTPException(403, "path escapes INGEST_ROOT")
            path = str(target)
        from ..ingest.controller import IngestController

        job_id = uuid.uuid4().hex
        loop = asyncio.get_running_loop()

        def run():
            ctl = IngestController(rt)
            try:
                res = ctl.ingest_many(payload.get("components") or [], source=source, path=path)
                state.events.emit_sync(job_id, "final", {"results": res})
            except Exception as e:
                state.events.emit_sync(job_id, "error", {"message": str(e)})
                state.events.emit_sync(job_id, "final", {"results": None, "error": True})

        loop.run_in_executor(None, run)
        return {"job_id": job_id}

    return app
