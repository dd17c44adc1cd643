"""Process-wide runtime: one GPU (or TP group) hosting the LLM engine, the
encoder, the five-table vector store and the retrievers, shared by the API,
the job workers and ingest.  Replaces the reference's five pods (api, worker,
vLLM, Cassandra, Redis) with one process per GPU."""
from __future__ import annotations

import logging
import os
import sys
import time
from pathlib import Path

import torch

from ..agent.graph_agent import GraphAgent
from ..agent.llm import EngineLLM, HTTPLLM, MeteredLLM
from ..config import Settings, settings as get_settings
from ..embed.service import Embedder
from ..engine.llm_engine import EngineConfig, LLMEngine
from ..engine.runner import EngineRunner
from ..engine.tokenizer import WordPieceTokenizer, load_tokenizer
from ..index.store import VectorStore
from ..models.configs import decoder_config, encoder_config
from ..models.encoder import BertEncoder
from ..models import build_decoder
from ..models.weights import load_state_dict
from ..retrieval.graph import RetrieverFactory

log = logging.getLogger(__name__)


class RAGRuntime:
    def __init__(self, settings: Settings | None = None, device: str | None = None, llm=None, ingest_llm=None,
                 embedder: Embedder | None = None, store: VectorStore | None = None, build_engine: bool = True,
                 shard: tuple[int, int] | None = None):
        self.settings = s = settings or get_settings()
        # TP serving (TP=N under torchrun): one process per GPU, the engine's
        # weights sharded over the TP group, replicated scheduling
        # (engine/runner.py); TP rank 0 of each group serves the API.
        self.tp_group = self.dp_group = None
        if s.tp > 1 and build_engine and llm is None:
            from ..parallel import comm
            from ..parallel.custom_ar import enable_for_group

            info = comm.init_distributed()
            if device is None and torch.cuda.is_available():
                device = f"cuda:{info.local_rank}"
            self.tp_group, self.dp_group = comm.make_tp_dp_groups(s.tp)
            enable_for_group(self.tp_group, device or s.resolved_device())
        self.device = torch.device(device or s.resolved_device())
        if self.device.type == "cuda" and self.device.index is None:  # threads pin it with set_device
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.started = time.time()
        dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        # encoder
        if embedder is None:
            ecfg = encoder_config(s.embed_model)
            sd = load_state_dict(s.encoder_dir) if s.encoder_dir else None
            vocab = str(Path(s.encoder_dir) / "vocab.txt") if s.encoder_dir else None
            enc = BertEncoder(ecfg, device=self.device, dtype=dtype, seed=s.seed + 2, state_dict=sd)
            embedder = Embedder(enc, WordPieceTokenizer(ecfg.vocab_size, vocab))
        self.embedder = embedder
        if s.embed_batch_window_ms > 0 and hasattr(embedder, "enable_batching"):
            embedder.enable_batching(s.embed_batch_window_ms / 1000.0)
        # store
        if store is None and shard is not None and shard[1] > 1 and s.index_dir:
            # replica r of N with a sharded index: its own shard snapshot, or the full one cut down
            from ..index.sharded_store import load_shard

            store = load_shard(s.index_dir, shard[0], shard[1], self.device, nprobe=s.nprobe)
        if store is None:
            if s.index_dir and (Path(s.index_dir) / "manifest.json").exists():
                store = VectorStore.load(s.index_dir, self.device, nprobe=s.nprobe)
            else:  # INDEX_KIND / NLIST / NPROBE select the per-table index (flat | ivf)
                store = VectorStore(embedder.dim, self.device, s.table_names(), index_kind=s.index_kind,
                                    nlist=s.nlist, nprobe=s.nprobe)
        self.store = store
        self.retrievers = RetrieverFactory(store, embedder)
        # LLM engine
        self.engine = self.runner = None
        self.tokenizer = None
        remote = s.qwen_endpoint.startswith(("http://", "https://"))
        if llm is None and remote:
            # remote mode (the reference's worker -> vLLM split, qwen_llm.py:104-148): an OpenAI-compatible
            # server elsewhere (e.g. another node's `serve`) answers the agent's and ingest's LLM calls
            llm = MeteredLLM(HTTPLLM(s.qwen_endpoint, s.qwen_model, max_tokens=s.qwen_max_output,
                                     timeout_s=s.llm_timeout_s, allow_thinking=s.allow_thinking))
            ingest_llm = HTTPLLM(s.qwen_endpoint, s.qwen_model, max_tokens=2048, mode="ingest",
                                 timeout_s=s.llm_timeout_s, allow_thinking=s.allow_thinking)
        elif llm is None and build_engine:
            dcfg = decoder_config(s.qwen_model)
            sd = load_state_dict(s.model_dir, device=self.device) if s.model_dir else None
            model = build_decoder(dcfg, device=self.device, dtype=dtype, seed=s.seed + 1, state_dict=sd,
                                  tp=self.tp_group)
            self.tokenizer = load_tokenizer(s.model_dir, dcfg.vocab_size, dcfg.arch)
            ecfg = EngineConfig(max_num_seqs=s.max_num_seqs, max_num_batched_tokens=s.max_num_batched_tokens,
                                max_model_len=s.max_model_len, block_size=s.kv_block,
                                kv_cache_gb=s.kv_cache_gb or None, use_cuda_graph=s.cuda_graphs,
                                enable_prefix_caching=s.prefix_caching, mixed_batches=s.mixed_batches, seed=s.seed)
            self.engine = LLMEngine(model, self.tokenizer, ecfg)
            from . import metrics as M

            M.ENGINE_HEALTHY.set(1)
            # the engine thread shares the interpreter with the API / job / retrieval threads: a 0.5 ms GIL
            # switch interval (Python's default is 5 ms) bounds how long it waits at a step boundary
            # (same-box A/B in profiles/ab_switch_r3.txt; the bench runs the same setting)
            sys.setswitchinterval(float(os.environ.get("GRAG_SWITCH_INTERVAL_MS", "0.5")) / 1000.0)
            self.runner = EngineRunner(self.engine, watchdog_s=s.engine_watchdog_s,
                                       on_health=lambda ok: M.ENGINE_HEALTHY.set(1 if ok else 0),
                                       tp=self.tp_group)
            llm = MeteredLLM(EngineLLM(self.runner, self.tokenizer, max_tokens=s.qwen_max_output,
                                       timeout_s=s.job_timeout_s, retries=s.llm_retries))
            ingest_llm = EngineLLM(self.runner, self.tokenizer, max_tokens=2048, mode="ingest",
                                   allow_thinking=s.allow_thinking, timeout_s=s.job_timeout_s,
                                   retries=s.llm_retries)
        self.llm = llm
        self.ingest_llm = ingest_llm or llm

    @property
    def tp_leader(self) -> bool:
        """True on the rank that owns the request queue (always without TP)."""
        return self.runner is None or self.runner.leader

    def warmup(self, contexts=(1024, 2048, 4096), windows=(1, 2, 4, 8)) -> int:
        """Capture the decode graphs a serving mix needs at startup (batch
        buckets up to MAX_NUM_SEQS x decode windows x split plans of the
        given context lengths), as vLLM does, so no capture stalls a live
        request.  The engine thread must be idle (call before serving)."""
        eng = self.engine
        if eng is None or not eng.on_gpu:
            return 0
        from ..engine.sequence import SamplingParams

        if self.tp_group is not None and not self.tp_group.trivial:
            return self._warmup_tp()

        # admit one request with the worker's sampling knobs first: graphs are keyed on the sampler chain
        eng.generate([[1, 2, 3, 4]], SamplingParams(max_tokens=2, temperature=0.4, top_p=0.8,
                                                     repetition_penalty=1.2, ignore_eos=True))
        buckets = [b for b in eng.cfg.graph_batch_sizes if b <= max(1, eng.cfg.max_num_seqs)]
        n = 0
        for ctx in contexts:
            if ctx <= eng.cfg.max_model_len:
                n += eng.warmup_graphs(buckets, ctx, windows, cascade=(False, True))
        return n

    def _warmup_tp(self) -> int:
        """TP: every rank's engine thread already steps in lockstep (the followers mirror the leader), so
        the leader warms the decode graphs by serving one batch per graph bucket through the runner —
        each bucket's graph (with its all-reduces) is captured by all TP ranks in the same step."""
        if not self.runner.leader:
            return 0
        from ..engine.sequence import SamplingParams

        eng = self.engine
        before = eng.stats["graph_captures"]
        sp = SamplingParams(max_tokens=3, temperature=0.4, top_p=0.8, repetition_penalty=1.2, ignore_eos=True)
        for B in [b for b in eng.cfg.graph_batch_sizes if b <= max(1, eng.cfg.max_num_seqs)]:
            hs = [self.runner.submit([1, 2, 3, 4 + i], sp) for i in range(B)]
            for h in hs:
                h.wait(self.settings.job_timeout_s)
        return eng.stats["graph_captures"] - before

    def agent(self) -> GraphAgent:
        """A fresh agent per job (cheap: it only holds references)."""
        s = self.settings
        return GraphAgent(self.llm, self.retrievers.scope_retrievers(), namespace=s.default_namespace,
                          max_iters=s.max_rag_attempts, router_top_k=s.router_top_k,
                          synth_max_tokens=s.synth_max_tokens or None)

    def health(self) -> dict:
        out = {"device": str(self.device), "tables": self.store.counts()}
        if self.tp_group is not None and not self.tp_group.trivial:
            out["tp"] = {"size": self.tp_group.size, "rank": self.tp_group.rank,
                         "custom_allreduce": self.tp_group.custom_ar is not None}
        if self.runner is not None:
            out["engine"] = {"healthy": self.runner.healthy, **{k: v for k, v in self.runner.stats().items()
                                                                 if isinstance(v, (int, float))}}
        return out

    def save_index(self, path: str | None = None) -> None:
        p = path or self.settings.index_dir
        if p:
            self.store.save(p)

    def close(self) -> None:
        if self.runner is not None:
            self.runner.shutdown()
        if hasattr(self.embedder, "close"):
            self.embedder.close()
