"""One typed configuration, read from the environment once.

Keeps every env name the reference reads (rag_shared/config.py:1-47,
ingest/src/app/config.py:13-47, ingest/src/app/llm_init.py:21-24) so existing
deployments keep working, resolves the reference's duplicate definitions
(REDIS_URL, MAX_RAG_ATTEMPTS, … were defined up to 3x; the last one won, so
those are the defaults here) and adds the engine / index knobs of the
MI355X design.  Cassandra settings are accepted for compatibility; the store
is the in-HBM index (``INDEX_DIR`` snapshots replace the Cassandra PVC).
"""
from __future__ import annotations

import os
from dataclasses import asdict, dataclass, field


def _env(name, default):
    return os.environ.get(name, default)


def _bool(name, default: bool) -> bool:
    v = os.environ.get(name)
    if v is None:
        return default
    return v.strip().lower() in {"1", "true", "t", "yes", "y", "on"}


def _int(name, default: int) -> int:
    return int(os.environ.get(name, str(default)))


def _float(name, default: float) -> float:
    return float(os.environ.get(name, str(default)))


@dataclass
class Settings:
    # --- shared (rag_shared/config.py)
    redis_url: str = field(default_factory=lambda: _env("REDIS_URL", "redis://redis-master:6379/0"))
    sse_ping_seconds: int = field(default_factory=lambda: _int("SSE_PING_SECONDS", 15))
    max_rag_attempts: int = field(default_factory=lambda: _int("MAX_RAG_ATTEMPTS", 3))
    min_source_nodes: int = field(default_factory=lambda: _int("MIN_SOURCE_NODES", 1))
    log_level: str = field(default_factory=lambda: _env("LOG_LEVEL", "INFO"))
    cassandra_host: str = field(default_factory=lambda: _env("CASSANDRA_HOST", "rag-demo-cassandra"))
    cassandra_port: int = field(default_factory=lambda: _int("CASSANDRA_PORT", 9042))
    cassandra_keyspace: str = field(default_factory=lambda: _env("CASSANDRA_KEYSPACE", "vector_store"))
    embed_model: str = field(default_factory=lambda: _env("EMBED_MODEL", "sentence-transformers/all-MiniLM-L6-v2"))
    embed_dim: int = field(default_factory=lambda: _int("EMBED_DIM", 384))
    qwen_endpoint: str = field(default_factory=lambda: _env("QWEN_ENDPOINT", "inproc"))
    qwen_model: str = field(default_factory=lambda: _env("QWEN_MODEL", "Qwen/Qwen2.5-3B-Instruct"))
    qwen_max_output: int = field(default_factory=lambda: _int("QWEN_MAX_OUTPUT", 4096))
    qwen_temperature: float = field(default_factory=lambda: _float("QWEN_TEMPERATURE", 0.7))
    qwen_top_p: float = field(default_factory=lambda: _float("QWEN_TOP_P", 0.9))
    router_top_k: int = field(default_factory=lambda: _int("ROUTER_TOP_K", 5))
    # token cap of the agent's synthesize call (0: QWEN_MAX_OUTPUT like every other agent call)
    synth_max_tokens: int = field(default_factory=lambda: _int("SYNTH_MAX_TOKENS", 0))
    default_namespace: str = field(default_factory=lambda: _env("DEFAULT_NAMESPACE", "default"))
    metrics_port: int = field(default_factory=lambda: _int("METRICS_PORT", 9000))
    allow_thinking: bool = field(default_factory=lambda: _bool("ALLOW_THINKING", True))
    # --- ingest (ingest/src/app/config.py)
    github_token: str = field(default_factory=lambda: _env("GITHUB_TOKEN", ""))
    github_user: str = field(default_factory=lambda: _env("GITHUB_USER", "jasonbuchanan145"))
    data_dir: str | None = field(default_factory=lambda: os.environ.get("DATA_DIR"))
    default_branch: str = field(default_factory=lambda: _env("DEFAULT_BRANCH", "main"))
    default_collection: str = field(default_factory=lambda: _env("DEFAULT_COLLECTION", "misc"))
    dev_force_standalone: bool = field(default_factory=lambda: _bool("DEV_MODE", False))
    table_catalog: str = field(default_factory=lambda: _env("EMBEDDINGS_TABLE_CATALOG", "embeddings_catalog"))
    table_repo: str = field(default_factory=lambda: _env("EMBEDDINGS_TABLE_REPO", "embeddings_repo"))
    table_module: str = field(default_factory=lambda: _env("EMBEDDINGS_TABLE_MODULE", "embeddings_module"))
    table_file: str = field(default_factory=lambda: _env("EMBEDDINGS_TABLE_FILE", "embeddings_file"))
    table_chunk: str = field(default_factory=lambda: _env("EMBEDDINGS_TABLE_CHUNK",
                                                          _env("EMBEDDINGS_TABLE", "embeddings")))
    pushgateway_address: str = field(default_factory=lambda: _env("PUSHGATEWAY_ADDRESS", "pushgateway:9091"))
    # --- MI355X engine / index knobs (new)
    # repositories ingest_many runs at once on the one engine (the reference: one after another,
    # ingest_controller.py:506-516): repo N+1's extractor waves fill repo N's roll-up tail
    ingest_concurrency: int = field(default_factory=lambda: _int("INGEST_CONCURRENCY", 4))
    model_dir: str | None = field(default_factory=lambda: os.environ.get("MODEL_DIR"))
    encoder_dir: str | None = field(default_factory=lambda: os.environ.get("ENCODER_DIR"))
    index_dir: str | None = field(default_factory=lambda: os.environ.get("INDEX_DIR"))
    device: str = field(default_factory=lambda: _env("DEVICE", "auto"))
    tp: int = field(default_factory=lambda: _int("TP", 1))
    dp: int = field(default_factory=lambda: _int("DP", 1))  # serve: replicas behind one front door
    # serve --replicas N: "shard" = each replica holds 1/N of every table, searches fan out through the
    # front door's hub (index/sharded_store.py); "mirror" = full copies, ingest writes broadcast
    index_sharding: str = field(default_factory=lambda: _env("INDEX_SHARDING", "shard"))
    max_num_seqs: int = field(default_factory=lambda: _int("MAX_NUM_SEQS", 64))
    max_model_len: int = field(default_factory=lambda: _int("MAX_MODEL_LEN", 11712))
    max_num_batched_tokens: int = field(default_factory=lambda: _int("MAX_NUM_BATCHED_TOKENS", 16384))
    kv_block: int = field(default_factory=lambda: _int("KV_BLOCK", 16))
    kv_cache_gb: float = field(default_factory=lambda: _float("KV_CACHE_GB", 0.0))
    cuda_graphs: bool = field(default_factory=lambda: _bool("CUDA_GRAPHS", True))
    prefix_caching: bool = field(default_factory=lambda: _bool("PREFIX_CACHING", True))
    mixed_batches: bool = field(default_factory=lambda: _bool("MIXED_BATCHES", False))
    index_kind: str = field(default_factory=lambda: _env("INDEX_KIND", "flat"))
    nlist: int = field(default_factory=lambda: _int("NLIST", 1024))
    nprobe: int = field(default_factory=lambda: _int("NPROBE", 16))
    worker_max_jobs: int = field(default_factory=lambda: _int("WORKER_MAX_JOBS", 10))
    job_timeout_s: int = field(default_factory=lambda: _int("JOB_TIMEOUT", 300))
    engine_watchdog_s: int = field(default_factory=lambda: _int("ENGINE_WATCHDOG_S", 120))
    keep_result_s: int = field(default_factory=lambda: _int("KEEP_RESULT", 3600))
    llm_timeout_s: float = field(default_factory=lambda: _float("LLM_TIMEOUT", 60.0))  # remote (HTTP) LLM calls
    llm_retries: int = field(default_factory=lambda: _int("LLM_RETRIES", 1))
    stream_tokens: bool = field(default_factory=lambda: _bool("STREAM_TOKENS", True))
    # the agent runs as a coroutine on the worker's event loop (LLM calls await engine futures; searches on a
    # small executor) instead of one thread per running job (AGENT_ASYNC=0: the thread-per-job mode)
    agent_async: bool = field(default_factory=lambda: _bool("AGENT_ASYNC", True))
    search_threads: int = field(default_factory=lambda: _int("SEARCH_THREADS", 16))
    # coalesce concurrent jobs' query embeddings into one encoder pass (0 disables)
    embed_batch_window_ms: float = field(default_factory=lambda: _float("EMBED_BATCH_WINDOW_MS", 1.0))
    # POST /ingest is off by default; `local` sources must resolve under INGEST_ROOT
    http_ingest: bool = field(default_factory=lambda: _bool("HTTP_INGEST", False))
    ingest_root: str | None = field(default_factory=lambda: os.environ.get("INGEST_ROOT"))
    seed: int = field(default_factory=lambda: _int("SEED", 0))

    def table_names(self) -> dict:
        return {"catalog": self.table_catalog, "repo": self.table_repo, "module": self.table_module,
                "file": self.table_file, "chunk": self.table_chunk}

    def resolved_device(self) -> str:
        if self.device != "auto":
            return self.device
        try:
            import torch

            return "cuda" if torch.cuda.is_available() else "cpu"
        except Exception:
            return "cpu"

    def to_dict(self) -> dict:
        d = asdict(self)
        d.pop("github_token", None)
        return d


_SETTINGS: Settings | None = None


def settings(reload: bool = False) -> Settings:
    global _SETTINGS
    if _SETTINGS is None or reload:
        _SETTINGS = Settings()
    return _SETTINGS
