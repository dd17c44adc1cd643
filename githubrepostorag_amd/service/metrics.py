"""Prometheus metrics — the reference's metric names (drop-in dashboards,
SURVEY §5.5) plus engine/index metrics of the new design.

All metrics live in one module-level registry so the API, worker and ingest
paths of a single process share them; ``/metrics`` renders it.
"""
from __future__ import annotations

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest

REGISTRY = CollectorRegistry(auto_describe=True)

# rest_api/src/app/main.py:22-32
REQUEST_COUNT = Counter("rest_api_requests_total", "Total HTTP requests", ["method", "path", "status"],
                        registry=REGISTRY)
REQUEST_LATENCY = Histogram("rest_api_request_duration_seconds", "Request duration in seconds",
                            buckets=(0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2, 5),
                            labelnames=["method", "path", "status"], registry=REGISTRY)
# rest_api/src/app/health.py:17-19
HEALTH_CHECKS_TOTAL = Counter("rest_api_health_checks_total", "Total health checks", registry=REGISTRY)
HEALTH_STATUS_GAUGE = Gauge("rest_api_health_status", "1=UP, 0=DOWN", registry=REGISTRY)
HEALTH_LATENCY = Histogram("rest_api_health_duration_seconds", "Health endpoint duration in seconds",
                           registry=REGISTRY)
# rag_worker/src/worker/worker.py:43-47
WORKER_JOBS_TOTAL = Counter("rag_worker_jobs_total", "Total RAG jobs processed", ["status"], registry=REGISTRY)
WORKER_JOB_DURATION = Histogram("rag_worker_job_duration_seconds", "Duration of RAG jobs", registry=REGISTRY)
WORKER_LLM_CALLS_TOTAL = Counter("rag_worker_llm_calls_total", "Total LLM calls from worker", ["result"],
                                 registry=REGISTRY)
WORKER_LLM_DURATION = Histogram("rag_worker_llm_duration_seconds", "Duration of LLM calls in worker",
                                registry=REGISTRY)
WORKER_RETRIEVAL_DURATION = Histogram("rag_worker_retrieval_seconds", "Time spent in GraphRAG retrieval+planning",
                                      registry=REGISTRY)
# ingest_controller.py:82-152 (pushed to a gateway there; exposed directly here)
INGEST_STAGE_SECONDS = Gauge("ingest_stage_run_seconds", "Duration (seconds) of an ingest stage",
                             ["level", "repo", "namespace", "branch", "run_id"], registry=REGISTRY)
INGEST_RUN_SECONDS = Gauge("ingest_run_seconds", "Total duration (seconds) of a single ingest run",
                           ["repo", "namespace", "branch", "run_id"], registry=REGISTRY)
# new: engine / index
ENGINE_TTFT = Histogram("grag_llm_ttft_seconds", "LLM time to first token",
                        buckets=(0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2, 5, 10), registry=REGISTRY)
ENGINE_TOKENS = Counter("grag_llm_generated_tokens_total", "Generated tokens", registry=REGISTRY)
ENGINE_PROMPT_TOKENS = Counter("grag_llm_prompt_tokens_total", "Prompt tokens processed", registry=REGISTRY)
ENGINE_CACHED_TOKENS = Counter("grag_llm_prefix_cached_tokens_total", "Prompt tokens served from the prefix cache",
                               registry=REGISTRY)
ENGINE_RUNNING = Gauge("grag_llm_running_seqs", "Sequences in the running batch", registry=REGISTRY)
ENGINE_WAITING = Gauge("grag_llm_waiting_seqs", "Queued sequences", registry=REGISTRY)
ENGINE_KV_USAGE = Gauge("grag_llm_kv_cache_usage", "Fraction of KV blocks in use", registry=REGISTRY)
INDEX_SEARCH_SECONDS = Histogram("grag_index_search_seconds", "Vector search latency", ["scope"],
                                 buckets=(0.0005, 0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.5),
                                 registry=REGISTRY)
INDEX_ROWS = Gauge("grag_index_rows", "Rows per scope table", ["table"], registry=REGISTRY)
EMBED_TEXTS = Counter("grag_embed_texts_total", "Texts embedded", registry=REGISTRY)
INGEST_DOCS = Counter("grag_ingest_documents_total", "Source files fully ingested", registry=REGISTRY)
SPAN_SECONDS = Histogram("grag_span_seconds", "Per-stage span durations of RAG jobs (utils.tracing)", ["span"],
                         buckets=(0.001, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10, 30),
                         registry=REGISTRY)
ENGINE_HEALTHY = Gauge("grag_engine_healthy", "1 when the engine loop is stepping normally, 0 after a fault/hang",
                       registry=REGISTRY)
GPU_MEM_USED = Gauge("grag_gpu_memory_used_bytes", "HBM bytes allocated by this process", ["device"],
                     registry=REGISTRY)


def observe_span(name: str, seconds: float) -> None:
    SPAN_SECONDS.labels(span=name).observe(seconds)


def render() -> bytes:
    try:
        import torch

        if torch.cuda.is_available():
            for i in range(torch.cuda.device_count()):
                GPU_MEM_USED.labels(device=str(i)).set(torch.cuda.memory_allocated(i))
    except Exception:
        pass
    return generate_latest(REGISTRY)

# front door over N replicas (service/cluster.py)
CLUSTER_REPLICAS = Gauge("grag_cluster_replicas_live", "Replicas connected to the front door", registry=REGISTRY)
CLUSTER_INFLIGHT = Gauge("grag_cluster_replica_inflight_jobs", "Jobs running on a replica", ["replica"],
                         registry=REGISTRY)
CLUSTER_DISPATCH = Counter("grag_cluster_dispatched_jobs_total", "Jobs dispatched to a replica", ["replica"],
                           registry=REGISTRY)
# sharded index rounds (index/sharded_store.py, service/mesh.py)
INDEX_DEGRADED_ROUNDS = Counter("rag_index_degraded_rounds_total",
                                "Sharded retrieval rounds answered without every shard (recall dropped)", ["table"],
                                registry=REGISTRY)
PROMPT_TRUNCATIONS = Counter("grag_llm_prompt_truncations_total",
                             "Agent / ingest prompts whose middle context was cut to fit max_model_len",
                             registry=REGISTRY)
