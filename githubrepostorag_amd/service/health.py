"""Actuator-style ``GET /health`` (rest_api/src/app/health.py:32-142).

Same JSON shape and semantics: ``status`` UP/DOWN, ``components`` with
per-component status/details, ``details.application`` (name, version,
uptime), ``details.system`` (cpu/memory/disk via psutil), response time;
HTTP 503 whenever a component is DOWN.  Components map to this design:
``vector_store`` (the in-HBM tables; also reported under the reference's
``cassandra`` key for dashboards), ``qwen`` (the in-process engine, or an
HTTP probe of ``QWEN_ENDPOINT`` when the LLM is remote), ``vector_index``
(a one-row retrieval smoke test), and ``gpu`` (device + HBM usage).
"""
from __future__ import annotations

import time
from datetime import datetime, timezone

import psutil
from fastapi import FastAPI
from fastapi.responses import JSONResponse

from . import metrics as M

_app_start_time: float | None = None


def _get_app_start_time() -> float:
    global _app_start_time
    if _app_start_time is None:
        _app_start_time = time.time()
    return _app_start_time


def _format_uptime(uptime_seconds: float) -> str:
    if uptime_seconds < 60:
        return f"{uptime_seconds:.1f} seconds"
    days = int(uptime_seconds // 86400)
    hours = int((uptime_seconds % 86400) // 3600)
    minutes = int((uptime_seconds % 3600) // 60)
    seconds = int(uptime_seconds % 60)
    parts = []
    if days:
        parts.append(f"{days} day{'s' if days != 1 else ''}")
    if hours:
        parts.append(f"{hours} hour{'s' if hours != 1 else ''}")
    if minutes:
        parts.append(f"{minutes} minute{'s' if minutes != 1 else ''}")
    if seconds or not parts:
        parts.append(f"{seconds} second{'s' if seconds != 1 else ''}")
    return ", ".join(parts)


def _probe_store(runtime) -> dict:
    counts = runtime.store.counts()
    return {"status": "UP", "details": {"kind": "gpu-vector-store", "device": str(runtime.store.device),
                                        "tables": counts, "embeddings_count": counts.get("embeddings", 0)}}


def _probe_llm(runtime, requests_mod) -> dict:
    if getattr(runtime, "runner", None) is not None:
        st = runtime.runner.stats()
        ok = runtime.runner.healthy and runtime.runner._thread.is_alive()
        return {"status": "UP" if ok else "DOWN",
                "details": {"endpoint": "in-process", "running": st.get("running"), "waiting": st.get("waiting"),
                            "kv_cache_usage": round(st.get("kv_usage", 0.0), 4),
                            **({"error": str(runtime.runner.last_error)} if not ok else {})}}
    endpoint = runtime.settings.qwen_endpoint
    if endpoint in ("", "inproc"):
        return {"status": "UP", "details": {"endpoint": "injected-client"}}
    r = requests_mod.get(f"{endpoint.rstrip('/')}/health", timeout=5)
    return {"status": "UP" if r.status_code == 200 else "DOWN",
            "details": {"endpoint": endpoint, "response_time_ms": r.elapsed.total_seconds() * 1000}}


def _probe_index(runtime) -> dict:
    tab = runtime.store.table("chunk")
    if tab.count() == 0:
        return {"status": "UP", "details": {"initialized": False}}
    hits = runtime.retrievers.for_chunk(k=1, start_k=1, max_depth=0).invoke("health check")
    return {"status": "UP", "details": {"initialized": True, "test_results_count": len(hits)}}


def _probe_replicas(view, component: str) -> dict:
    """At a front door every component lives on the replicas: UP while at least one replica is connected
    (and, for the LLM, its engine reports healthy); details list each replica's last health report."""
    h = view.hub.health()
    reps = h["replicas"]
    if not reps:
        return {"status": "DOWN", "details": {"error": "no replica connected"}}
    if component == "qwen":
        ok = [r for r in reps if (r.get("engine") or {}).get("healthy", True)]
        return {"status": "UP" if ok else "DOWN",
                "details": {"endpoint": "replicas", "healthy": len(ok), "replicas": len(reps)}}
    if component == "vector_store":
        if any(r.get("shard", "full") != "full" for r in reps):  # row-sharded index: every shard's rows
            return {"status": "UP", "details": {"shards": {r.get("shard"): r.get("tables", {}) for r in reps},
                                                "replicas": len(reps)}}
        return {"status": "UP", "details": {"tables": reps[0].get("tables", {}), "replicas": len(reps)}}
    if component == "gpu":
        return {"status": "UP", "details": {"devices": [r.get("device") for r in reps]}}
    return {"status": "UP", "details": {"replicas": [{"rank": r["rank"], "inflight": r["inflight"],
                                                      "capacity": r["capacity"], "shard": r.get("shard", "full")}
                                                     for r in reps]}}


def _probe_gpu() -> dict:
    try:
        import torch

        if not torch.cuda.is_available():
            return {"status": "UP", "details": {"device": "cpu"}}
        free, total = torch.cuda.mem_get_info()
        return {"status": "UP", "details": {"device": torch.cuda.get_device_name(0), "hbm_total_gb": round(total / 2**30, 1),
                                            "hbm_free_gb": round(free / 2**30, 1)}}
    except Exception as e:  # pragma: no cover
        return {"status": "DOWN", "details": {"error": str(e)}}


def register_health_endpoints(app: FastAPI, runtime_getter, requests_mod=None) -> None:
    import requests as _requests

    req = requests_mod or _requests

    @app.get("/health")
    async def detailed_health():
        t0 = time.perf_counter()
        M.HEALTH_CHECKS_TOTAL.inc()
        start = _get_app_start_time()
        up = time.time() - start
        h = {"status": "UP", "components": {},
             "details": {"application": {"name": "RAG API Service", "version": "2.0.0",
                                         "uptime_human_readable": _format_uptime(up), "uptime_ms": up * 1000.0,
                                         "timestamp": datetime.now(timezone.utc).isoformat()},
                         "system": {"cpu_percent": psutil.cpu_percent(), "memory_percent": psutil.virtual_memory().percent,
                                    "disk_usage": psutil.disk_usage("/").percent}}}
        runtime = runtime_getter()
        if hasattr(runtime, "hub"):  # front door over replica processes (service/cluster.py)
            probes = [(name, lambda name=name: _probe_replicas(runtime, name))
                      for name in ("vector_store", "qwen", "vector_index", "gpu")]
        else:
            probes = [("vector_store", lambda: _probe_store(runtime)), ("qwen", lambda: _probe_llm(runtime, req)),
                      ("vector_index", lambda: _probe_index(runtime)), ("gpu", _probe_gpu)]
        for name, fn in probes:
            try:
                if runtime is None and name != "gpu":
                    raise RuntimeError("runtime not initialised")
                h["components"][name] = fn()
            except Exception as e:
                h["components"][name] = {"status": "DOWN", "details": {"error": str(e)}}
            if h["components"][name]["status"] != "UP":
                h["status"] = "DOWN"
        h["components"]["cassandra"] = dict(h["components"]["vector_store"],
                                            details={**h["components"]["vector_store"].get("details", {}),
                                                     "replaced_by": "vector_store"})
        dur = time.perf_counter() - t0
        h["details"]["response_time_ms"] = dur * 1000.0
        M.HEALTH_STATUS_GAUGE.set(1.0 if h["status"] == "UP" else 0.0)
        M.HEALTH_LATENCY.observe(dur)
        return JSONResponse(status_code=503 if h["status"] == "DOWN" else 200, content=h)
