"""Job runtime: the reference's ARQ worker (rag_worker/src/worker/worker.py)
as an in-process asyncio job queue with the same knobs (``max_jobs=10``,
``job_timeout=300``, ``keep_result=3600``, worker.py:182-187) and the same
event sequence per job:

  started -> [final{cancelled}] -> iteration -> turn* -> [token*] -> retrieval
  -> final{answer, sources}        (or error{message} -> final{error:true})

The agent runs as a coroutine on the worker's event loop (``GraphAgent.arun``:
its LLM calls await engine futures, its index searches run on a small shared
executor), so a running job holds no thread and thousands can wait on the
engine at once; ``AGENT_ASYNC=0`` keeps the thread-per-job mode.  Its progress
callback is bound per job (no shared singleton state) and publishes into the
job's replayable event log.  Cancellation
is checked before every agent node and aborts the job's in-flight LLM
requests (the reference checked once, before any work).
"""
from __future__ import annotations

import asyncio
import concurrent.futures
import logging
import time
import uuid

from ..agent.graph_agent import Cancelled
from ..index.sharded_store import round_health
from . import metrics as M
from ..utils.tracing import Trace
from .events import CancelFlags, EventLog

log = logging.getLogger(__name__)


class JobQueue:
    """ARQ-equivalent: named job functions, bounded concurrency, per-job
    timeout, result retention."""

    def __init__(self, functions: dict, max_jobs: int = 10, job_timeout: float = 300.0, keep_result: float = 3600.0):
        self.functions = functions
        self.max_jobs = max_jobs
        self.job_timeout = job_timeout
        self.keep_result = keep_result
        self.results: dict[str, dict] = {}
        self._q: asyncio.Queue | None = None
        self._tasks: list[asyncio.Task] = []
        self.ctx: dict = {}

    async def start(self) -> None:
        if self._q is not None:
            return
        self._loop = asyncio.get_running_loop()
        self._q = asyncio.Queue()
        self._tasks = [asyncio.create_task(self._consume(i)) for i in range(self.max_jobs)]

    def set_max_jobs(self, n: int) -> None:
        """Raise the concurrency bound (thread-safe; e.g. the front door's queue follows the sum of its
        replicas' slots).  Consumers are only added: a smaller bound leaves the extra ones idle-waiting
        on the queue, and the hub's job function waits for a replica slot anyway."""
        self.max_jobs = max(1, int(n))
        loop = getattr(self, "_loop", None)
        if loop is None or self._q is None:
            return
        try:
            loop.call_soon_threadsafe(self._grow)
        except RuntimeError:  # loop closed
            pass

    def _grow(self) -> None:
        while self._q is not None and len(self._tasks) < self.max_jobs:
            self._tasks.append(asyncio.create_task(self._consume(len(self._tasks))))

    async def stop(self) -> None:
        for t in self._tasks:
            t.cancel()
        self._tasks = []
        self._q = None

    async def enqueue_job(self, function: str, *args, _job_id: str | None = None):
        if self._q is None:
            await self.start()
        jid = _job_id or uuid.uuid4().hex
        self.results[jid] = {"status": "queued", "enqueued": time.time(), "function": function}
        await self._q.put((jid, function, args))
        return jid

    async def _consume(self, idx: int) -> None:
        while True:
            jid, fn, args = await self._q.get()
            self.results[jid]["status"] = "running"
            try:
                res = await asyncio.wait_for(self.functions[fn](self.ctx, *args), timeout=self.job_timeout)
                self.results[jid].update(status="complete", result=res)
            except asyncio.TimeoutError:
                self.results[jid].update(status="timeout")
                on_to = self.ctx.get("on_timeout")
                if on_to:
                    await on_to(*args)
            except asyncio.CancelledError:
                raise
            except Exception as e:  # job functions report their own errors as events
                log.exception("job %s failed", jid)
                self.results[jid].update(status="failed", error=str(e))
            finally:
                self.results[jid]["finished"] = time.time()
                self._gc()
                self._q.task_done()

    def _gc(self) -> None:
        now = time.time()
        for k in [k for k, v in self.results.items() if v.get("finished") and now - v["finished"] > self.keep_result]:
            self.results.pop(k, None)


class RAGWorker:
    def __init__(self, runtime, events: EventLog, flags: CancelFlags, max_jobs: int = 10,
                 job_timeout: float = 300.0, keep_result: float = 3600.0, stream_tokens: bool = True,
                 agent_async: bool | None = None):
        self.runtime = runtime
        self.events = events
        self.flags = flags
        self.stream_tokens = stream_tokens
        s = getattr(runtime, "settings", None)
        # coroutine agent (GraphAgent.arun): a running job holds no thread; its searches share a small pool
        self.agent_async = bool(getattr(s, "agent_async", True)) if agent_async is None else agent_async
        n_exec = max(1, int(getattr(s, "search_threads", 16))) if self.agent_async else max_jobs
        self.executor = concurrent.futures.ThreadPoolExecutor(max_workers=n_exec,
                                                              thread_name_prefix="rag-search" if self.agent_async
                                                              else "rag-job")
        self.queue = JobQueue({"run_rag_job": self.run_rag_job}, max_jobs, job_timeout, keep_result)
        self.queue.ctx["on_timeout"] = self._on_timeout

    async def _on_timeout(self, job_id: str, req: dict) -> None:
        self.flags.cancel_sync(job_id)
        M.WORKER_JOBS_TOTAL.labels(status="error").inc()
        await self.events.emit(job_id, "error", {"message": f"job timed out after {self.queue.job_timeout}s"})
        await self.events.emit(job_id, "final", {"answer": "", "sources": None, "error": True})

    async def run_rag_job(self, ctx, job_id: str, req: dict) -> dict | None:
        t_job = time.perf_counter()
        queue_wait = max(0.0, time.time() - float((self.queue.results.get(job_id) or {}).get("enqueued", time.time())))
        query = (req.get("query") or "").strip()
        forced = req.get("force_level")
        s = self.runtime.settings
        namespace = req.get("namespace") or s.default_namespace
        await self.events.emit(job_id, "started", {"query": query, "force_level": forced,
                                                   "max_attempts": s.max_rag_attempts})
        try:
            if await self.flags.is_cancelled(job_id):
                await self.events.emit(job_id, "final", {"answer": "", "sources": None, "cancelled": True})
                M.WORKER_JOBS_TOTAL.labels(status="cancelled").inc()
                return None
            await self.events.emit(job_id, "iteration", {"attempt": 0, "query": query, "force_level": forced,
                                                         "namespace": namespace})
            agent = self.runtime.agent()
            n_tok = [0]

            def progress(payload):
                self.events.emit_threadsafe(job_id, "turn", payload)

            def on_token(delta):
                self.events.emit_threadsafe(job_id, "token", {"text": delta, "index": n_tok[0]})
                n_tok[0] += 1

            loop = asyncio.get_running_loop()
            t_rag = time.perf_counter()
            trace = Trace(job_id, observer=M.observe_span)
            trace.add("queue_wait", queue_wait)
            def run_agent():
                # the job's shard rounds run on this thread: record whether any lost a shard
                with round_health() as health:
                    res = agent.run(query, namespace=namespace, progress_cb=progress,
                                    cancel_check=lambda: self.flags.is_cancelled_sync(job_id),
                                    force_level=forced, on_answer_token=on_token if self.stream_tokens else None,
                                    trace=trace, repo=req.get("repo_name") or None,
                                    top_k=req.get("top_k") or None)
                return res, health

            if self.agent_async:
                health = {"rounds": 0, "degraded_rounds": 0, "missing_shards": set()}
                result = await agent.arun(query, namespace=namespace, progress_cb=progress,
                                          cancel_check=lambda: self.flags.is_cancelled_sync(job_id),
                                          force_level=forced,
                                          on_answer_token=on_token if self.stream_tokens else None, trace=trace,
                                          repo=req.get("repo_name") or None, top_k=req.get("top_k") or None,
                                          search_executor=self.executor, health=health)
            else:
                result, health = await loop.run_in_executor(self.executor, run_agent)
            M.WORKER_RETRIEVAL_DURATION.observe(time.perf_counter() - t_rag)
            sources = result.get("sources") or []
            debug = result.get("debug") or {}
            retrieval = {"attempt": 0, "scope": result.get("scope", ""), "sources_found": len(sources),
                         "turns": debug.get("turns", []), "final_ctx_blocks": debug.get("final_ctx_blocks", 0)}
            if health["rounds"]:  # sharded index: were all shards heard in every round?
                retrieval.update(degraded=health["degraded_rounds"] > 0, shard_rounds=health["rounds"],
                                 degraded_rounds=health["degraded_rounds"],
                                 missing_shards=sorted(health["missing_shards"]))
            await self.events.emit(job_id, "retrieval", retrieval)
            await self.events.emit(job_id, "timing", {"job_s": round(time.perf_counter() - t_job, 4),
                                                      "agent_s": round(time.perf_counter() - t_rag, 4),
                                                      "trace_id": trace.trace_id, "totals_ms": trace.totals(),
                                                      "spans": trace.to_list()})
            await self.events.emit(job_id, "final", {"answer": result.get("answer", ""), "sources": sources or None})
            M.WORKER_JOBS_TOTAL.labels(status="success").inc()
            return {"answer": result.get("answer", ""), "n_sources": len(sources)}
        except Cancelled:
            await self.events.emit(job_id, "final", {"answer": "", "sources": None, "cancelled": True})
            M.WORKER_JOBS_TOTAL.labels(status="cancelled").inc()
            return None
        except Exception as e:
            log.exception("worker job failed")
            M.WORKER_JOBS_TOTAL.labels(status="error").inc()
            await self.events.emit(job_id, "error", {"message": str(e)})
            await self.events.emit(job_id, "final", {"answer": "", "sources": None, "error": True})
            return None
        finally:
            M.WORKER_JOB_DURATION.observe(time.perf_counter() - t_job)
