"""REST/SSE contract on CPU (reference: rest_api/tests/test_jobs_controller.py,
test_health.py, rag_worker/tests/test_worker.py): job creation, replayable SSE
event order, cancel, job status, health UP/DOWN (503), uptime formatting,
metrics, OpenAI-compatible endpoints against a real tiny in-process engine."""
import asyncio
import json
import time

import pytest
import torch
from fastapi.testclient import TestClient

from githubrepostorag_amd.agent.llm import ScriptedLLM
from githubrepostorag_amd.config import Settings
from githubrepostorag_amd.embed.service import Embedder
from githubrepostorag_amd.index.store import VectorStore
from githubrepostorag_amd.service.api import APIState, create_app
from githubrepostorag_amd.service.events import CancelFlags, EventLog
from githubrepostorag_amd.service.health import _format_uptime
from githubrepostorag_amd.service.runtime import RAGRuntime
from githubrepostorag_amd.service.worker import JobQueue


def _router(p):
    if p.startswith("Choose the best search scope"):
        return '{"scope": "code"}'
    if "Judge if the retrieved" in p:
        return '{"coverage": 0.9, "needs_more": false}'
    if p.startswith("Generate 3-4"):
        return '["alt query"]'
    return "Widgets are handled in [1]."


@pytest.fixture(scope="module")
def embedder():
    return Embedder.from_name("encoder-tiny", device="cpu", seed=3)


def _runtime(embedder, llm=None, **kw):
    s = Settings(index_dir=None, data_dir=None, worker_max_jobs=4, job_timeout_s=30.0, **kw)
    store = VectorStore(embedder.dim, "cpu")
    vecs = embedder.embed_documents(["widgets code", "gadget service", "billing module"])
    store.table("chunk").upsert(["a", "b", "c"], ["widgets code", "gadget service", "billing module"], vecs,
                                [{"namespace": "default", "repo": "r", "module": "m", "file_path": f"{x}.py"}
                                 for x in "abc"])
    return RAGRuntime(s, device="cpu", llm=llm or ScriptedLLM(_router), embedder=embedder, store=store,
                      build_engine=False)


def _sse(client, job_id):
    """Parse the reference wire format: ``data: {"event": E, "data": D}`` frames."""
    events = []
    with client.stream("GET", f"/rag/jobs/{job_id}/events") as r:
        assert r.headers["content-type"].startswith("text/event-stream")
        for line in r.iter_lines():
            if line.startswith("data:"):
                msg = json.loads(line.split(":", 1)[1])
                events.append((msg["event"], msg["data"]))
                if msg["event"] == "final":
                    break
    return events


def test_job_lifecycle_and_event_order(embedder):
    rt = _runtime(embedder)
    with TestClient(create_app(APIState(runtime=rt))) as client:
        r = client.post("/rag/jobs", json={"query": "how are widgets handled?"})
        assert r.status_code == 200
        job_id = r.json()["job_id"]
        evs = _sse(client, job_id)
        kinds = [k for k, _ in evs]
        assert kinds[0] == "started" and kinds[1] == "iteration" and kinds[-1] == "final"
        for k in ("turn", "token", "retrieval", "timing"):
            assert k in kinds, kinds
        assert kinds.index("retrieval") < kinds.index("final")
        timing = next(d for k, d in evs if k == "timing")
        names = [sp["name"] for sp in timing["spans"]]
        for n in ("queue_wait", "plan", "retrieve", "search", "judge", "synthesize", "llm"):
            assert n in names, names
        llm_purposes = {sp.get("purpose") for sp in timing["spans"] if sp["name"] == "llm"}
        assert {"plan", "judge", "synthesize"} <= llm_purposes
        assert timing["totals_ms"]["synthesize"] >= 0 and timing["trace_id"] == job_id
        assert b"grag_span_seconds_bucket" in client.get("/metrics").content
        final = evs[-1][1]
        assert final["answer"] == "Widgets are handled in [1]."
        assert final["sources"] and final["sources"][0]["metadata"]["repo"] == "r"
        toks = "".join(d["text"] for k, d in evs if k == "token")
        assert toks.split() == final["answer"].split()
        # replay: a second subscriber sees the same stream from the start
        assert [k for k, _ in _sse(client, job_id)] == kinds
        st = client.get(f"/rag/jobs/{job_id}").json()
        assert st["done"] and st["final"]["answer"] == final["answer"]


def test_cancel_before_start(embedder):
    rt = _runtime(embedder)
    state = APIState(runtime=rt)
    with TestClient(create_app(state)) as client:
        # cancel a job id first, then enqueue with that id through the queue
        client.post("/rag/jobs/abc/cancel")
        r = client.post("/rag/jobs/abc/cancel")
        assert r.json() == {"status": "cancelling", "job_id": "abc"}
        client.portal.call(state.queue.enqueue_job, "run_rag_job", "abc", {"query": "q"})
        evs = _sse(client, "abc")
        assert [k for k, _ in evs] == ["started", "final"] and evs[-1][1]["cancelled"] is True


def test_cancel_mid_run(embedder):
    started = {"t": None}

    def slow(p):
        if "Judge if the retrieved" in p:
            started["t"] = time.time()
            time.sleep(0.5)
        return _router(p)

    rt = _runtime(embedder, llm=ScriptedLLM(slow))
    with TestClient(create_app(APIState(runtime=rt))) as client:
        job_id = client.post("/rag/jobs", json={"query": "q"}).json()["job_id"]
        for _ in range(200):
            if started["t"]:
                break
            time.sleep(0.01)
        client.post(f"/rag/jobs/{job_id}/cancel")
        evs = _sse(client, job_id)
        assert evs[-1][0] == "final" and evs[-1][1].get("cancelled") is True


def test_agent_error_emits_error_then_final(embedder):
    rt = _runtime(embedder)
    rt.agent = lambda: (_ for _ in ()).throw(RuntimeError("agent exploded"))
    with TestClient(create_app(APIState(runtime=rt))) as client:
        job_id = client.post("/rag/jobs", json={"query": "q"}).json()["job_id"]
        evs = _sse(client, job_id)
        assert [k for k, _ in evs][-2:] == ["error", "final"]
        assert evs[-1][1]["error"] is True and "exploded" in evs[-2][1]["message"]


def test_create_job_validation(embedder):
    with TestClient(create_app(APIState(runtime=_runtime(embedder)))) as client:
        assert client.post("/rag/jobs", json={}).status_code == 422


def test_health_up_and_down(embedder):
    rt = _runtime(embedder)
    with TestClient(create_app(APIState(runtime=rt))) as client:
        r = client.get("/health")
        assert r.status_code == 200
        h = r.json()
        assert h["status"] == "UP"
        assert set(h["components"]) >= {"vector_store", "qwen", "vector_index", "gpu", "cassandra"}
        assert h["components"]["vector_store"]["details"]["embeddings_count"] == 3
        assert h["components"]["vector_index"]["details"]["test_results_count"] >= 1
        assert "uptime_human_readable" in h["details"]["application"]
    with TestClient(create_app(APIState(runtime=None))) as client:
        r = client.get("/health")
        assert r.status_code == 503 and r.json()["status"] == "DOWN"


def test_health_remote_llm_probe(embedder):
    class Resp:
        status_code = 500

        class elapsed:
            @staticmethod
            def total_seconds():
                return 0.01

    class Req:
        @staticmethod
        def get(url, timeout):
            assert url == "http://llm:8000/health"
            return Resp()

    from fastapi import FastAPI

    from githubrepostorag_amd.service.health import register_health_endpoints

    rt = _runtime(embedder, qwen_endpoint="http://llm:8000")
    app = FastAPI()
    register_health_endpoints(app, lambda: rt, Req)
    with TestClient(app) as client:
        r = client.get("/health")
        assert r.status_code == 503 and r.json()["components"]["qwen"]["status"] == "DOWN"


@pytest.mark.parametrize("secs,expect", [(5.25, "5.2 seconds"), (61, "1 minute, 1 second"),
                                         (3600, "1 hour"), (90061, "1 day, 1 hour, 1 minute, 1 second"),
                                         (172800 + 7200, "2 days, 2 hours")])
def test_format_uptime(secs, expect):
    assert _format_uptime(secs) == expect


def test_metrics_endpoint(embedder):
    with TestClient(create_app(APIState(runtime=_runtime(embedder)))) as client:
        client.get("/health")
        body = client.get("/metrics").text
        assert 'rest_api_requests_total{method="GET",path="/health",status="200"}' in body
        assert "rest_api_health_checks_total" in body and "rest_api_health_status 1.0" in body


def test_embeddings_endpoint(embedder):
    with TestClient(create_app(APIState(runtime=_runtime(embedder)))) as client:
        r = client.post("/v1/embeddings", json={"input": ["a", "b"]})
        data = r.json()["data"]
        assert len(data) == 2 and len(data[0]["embedding"]) == embedder.dim
        v = torch.tensor(data[0]["embedding"])
        assert abs(float(v.norm()) - 1.0) < 1e-2


def test_v1_requires_engine(embedder):
    with TestClient(create_app(APIState(runtime=_runtime(embedder)))) as client:
        assert client.post("/v1/completions", json={"prompt": "hi"}).status_code == 503


def test_ingest_endpoint(embedder, monkeypatch):
    from githubrepostorag_amd.config import settings

    monkeypatch.setenv("HTTP_INGEST", "1")
    settings(reload=True)
    try:
        rt = _runtime(embedder)
        state = APIState(runtime=rt)
        with TestClient(create_app(state)) as client:
            job = client.post("/ingest", json={"components": [{"repo": "demo", "namespace": "default"}]}).json()
            evs = _sse(client, job["job_id"])
            res = evs[-1][1]["results"]
            assert res[0]["repo"] == "demo" and res[0]["nodes_written"] > 0
            assert rt.store.counts()["embeddings_catalog"] >= 1
    finally:
        monkeypatch.delenv("HTTP_INGEST")
        settings(reload=True)


def test_ingest_endpoint_locked_down(embedder, monkeypatch, tmp_path):
    """POST /ingest is off by default; when on, a `local` source may not leave INGEST_ROOT."""
    from githubrepostorag_amd.config import settings

    rt = _runtime(embedder)
    try:
        settings(reload=True)
        with TestClient(create_app(APIState(runtime=rt))) as client:
            assert client.post("/ingest", json={"source": "local", "path": "/etc"}).status_code == 403
        root = tmp_path / "repos"
        (root / "ok").mkdir(parents=True)
        monkeypatch.setenv("HTTP_INGEST", "1")
        monkeypatch.setenv("INGEST_ROOT", str(root))
        settings(reload=True)
        with TestClient(create_app(APIState(runtime=rt))) as client:
            for bad in ("/etc", "../../etc", "ok/../../"):
                r = client.post("/ingest", json={"source": "local", "path": bad})
                assert r.status_code == 403, bad
            assert client.post("/ingest", json={"source": "ftp"}).status_code == 400
    finally:
        monkeypatch.delenv("HTTP_INGEST", raising=False)
        monkeypatch.delenv("INGEST_ROOT", raising=False)
        settings(reload=True)


def test_job_queue_timeout():
    async def run():
        hits = []

        async def slow(ctx, job_id):
            await asyncio.sleep(5)

        async def on_timeout(job_id, *a):
            hits.append(job_id)

        q = JobQueue({"slow": slow}, max_jobs=2, job_timeout=0.1)
        q.ctx["on_timeout"] = on_timeout
        await q.start()
        await q.enqueue_job("slow", "j1")
        for _ in range(50):
            if hits:
                break
            await asyncio.sleep(0.05)
        await q.stop()
        return hits

    assert asyncio.run(run()) == ["j1"]


def test_event_log_replay_and_gc():
    async def run():
        ev = EventLog(keep_seconds=0.0)
        await ev.emit("j", "started", {"a": 1})
        await ev.emit("j", "final", {"answer": "x"})
        chunks = [c async for c in ev.stream("j", ping_seconds=0.05)]
        return ev, chunks

    ev, chunks = asyncio.run(run())
    body = "".join(chunks)
    assert body.index('"event": "started"') < body.index('"event": "final"')
    time.sleep(0.01)
    assert ev.gc() == 1


def test_cancel_flags_callbacks():
    f = CancelFlags()
    seen = []
    f.on_cancel("x", lambda: seen.append(1))
    f.cancel_sync("x")
    assert f.is_cancelled_sync("x") and seen == [1]
    assert not f.is_cancelled_sync("y")


def test_static_ui_served():
    from fastapi.testclient import TestClient

    from githubrepostorag_amd.service.api import APIState, create_app

    with TestClient(create_app(APIState())) as c:
        r = c.get("/static/index.html")
        assert r.status_code == 200 and "text/html" in r.headers["content-type"]
        body = r.text
        for needle in ("/rag/jobs", "EventSource", "/cancel", '"token"', '"final"'):
            assert needle in body
