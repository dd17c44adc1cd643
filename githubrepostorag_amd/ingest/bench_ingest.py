"""Ingest throughput benchmark (BASELINE.json secondary metric: ingest
docs/sec).  Runs the FULL ingest_component pipeline on a synthetic repository
of ``n_files`` source files: filter/transform -> code split -> LLM summary /
title / keyword waves -> catalog (README check or code-summary catalog) ->
file / module / repo roll-ups (+ their extractor passes) -> embedding of
every scope -> upsert into the GPU store.

Random-init weights essentially never emit EOS, so every LLM call would run
to its token cap; caps are therefore set to the lengths real Qwen outputs
have for these prompts (code summary 128, keywords 64, title 32, roll-ups
256 tokens) and ``ignore_eos`` is not used.
"""
from __future__ import annotations

import logging
import time

import torch


from ..agent.llm import EngineLLM
from ..config import Settings
from ..engine.llm_engine import EngineConfig, LLMEngine
from ..engine.sequence import SamplingParams
from ..engine.runner import EngineRunner
from ..index.store import VectorStore
from ..utils.synthetic import synthetic_repo
from .controller import IngestController
from .readers import Document

log = logging.getLogger(__name__)


def run_ingest_bench(model, tok, emb, n_files: int, seed: int = 0, max_num_seqs: int = 256,
                     max_model_len: int = 8192, use_graph: bool = True, summary_tokens: int = 128,
                     mixed_batches: bool = False, tp=None, token_cap: int | None = None,
                     kv_cache_gb: float | None = None, runner: EngineRunner | None = None
                     ) -> tuple[int, float, dict]:
    """Returns (documents ingested, seconds, per-stage seconds).

    ``token_cap``: one generation cap for every LLM call instead of the per-call lengths above (the
    reference's 2048, ingest/src/app/llm_init.py:56; random weights run every call to the cap).

    ``tp`` (a tensor-parallel group the model is sharded over): the group's TP
    rank 0 runs the pipeline and owns the request queue; the other ranks mirror
    its engine in lockstep (engine/runner.py ``follow``) until it shuts down, and
    report 0 documents (one ingest per TP group).

    ``runner``: run on this (already warmed) engine runner instead of an engine of its own -- ingest sharing
    one engine with interactive serving traffic (BASELINE config 4's concurrent ingest + query streams); the
    runner is left running."""
    dev = torch.device(getattr(model, "device", "cpu"))
    if runner is not None:
        return _ingest_on(runner, runner.engine, tok, emb, n_files, seed, summary_tokens, token_cap, dev)
    sizes = tuple(sorted({*EngineConfig.graph_batch_sizes, *range(256, max_num_seqs + 1, 128), max_num_seqs}))
    eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=max_num_seqs, max_num_batched_tokens=16384,
                                             max_model_len=max_model_len, use_cuda_graph=use_graph, seed=seed,
                                             mixed_batches=mixed_batches, kv_cache_gb=kv_cache_gb,
                                             graph_batch_sizes=tuple(b for b in sizes if b <= max_num_seqs)))
    if use_graph and dev.type == "cuda":
        # the decode graphs the ingest will replay, captured before timing: every batch bucket x decode
        # window x the split plans of short / medium / long contexts, for the ingest sampling chain (top-p)
        ctxs = sorted({c for c in (2048, 4096, max_model_len) if c <= max_model_len})
        t_w = time.perf_counter()
        n_w = eng.warmup_graphs(max_ctx=ctxs, windows=(1, 2, 4, 8),
                                params=SamplingParams(temperature=EngineLLM.INGEST["temperature"],
                                                      top_p=EngineLLM.INGEST["top_p"]),
                                cascade=(False, True))
        log.info("ingest engine: %d decode graphs captured in %.1fs", n_w, time.perf_counter() - t_w)
    tp = tp if tp is not None and not tp.trivial else None
    runner = EngineRunner(eng, tp=tp)
    if tp is not None and not runner.leader:
        t0 = time.perf_counter()
        runner.join()  # lockstep follower until the leader's runner stops
        del eng
        if dev.type == "cuda":
            torch.cuda.empty_cache()
        return 0, time.perf_counter() - t0, {"tp_follower": True}
    try:
        return _ingest_on(runner, eng, tok, emb, n_files, seed, summary_tokens, token_cap, dev)
    finally:
        runner.shutdown()
        del eng
        if dev.type == "cuda":
            torch.cuda.empty_cache()


def _ingest_on(runner, eng, tok, emb, n_files, seed, summary_tokens, token_cap, dev):
    """The timed ingest_component pass over a synthetic repo, on ``runner``'s engine."""
    llm = EngineLLM(runner, tok, max_tokens=token_cap or summary_tokens, mode="ingest", timeout_s=3600.0,
                    retries=0)
    store = VectorStore(emb.dim, dev)
    ctl = IngestController(llm=llm, store=store, embedder=emb, settings=Settings(data_dir=None),
                           summary_tokens=summary_tokens, token_cap=token_cap)
    _, files = synthetic_repo(seed, n_files, f"bench-repo-{seed}")
    docs = [Document(f["text"], {"file_path": f["file_path"], "file_name": f["file_path"].split("/")[-1]})
            for f in files]
    if dev.type == "cuda":
        torch.cuda.synchronize()
    own_trace = eng.trace is None  # a caller's trace (bench.py concurrent phase) is kept and shared
    if own_trace:
        eng.trace = []  # per-step timeline for the critical-path summary below
    trace = eng.trace
    i0 = len(trace)
    t0 = time.perf_counter()
    res = ctl.ingest_component(repo=f"bench-repo-{seed}", namespace="bench", documents=docs, force=True)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = dict(res["stage_seconds"])
    st["engine"] = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in eng.stats.items()
                    if isinstance(v, (int, float))}
    st["llm_calls"] = ctl.extractors.wave.calls + ctl.hier.wave.calls + ctl.hier.extract.wave.calls
    st["timeline"] = critical_path(trace[i0:], t0, dt)
    if own_trace:
        eng.trace = None
    return res["documents"], dt, st


def run_ingest_multi(model, tok, emb, n_repos: int, n_files: int, seed: int = 0, concurrency: int | None = None,
                     max_num_seqs: int = 256, max_model_len: int = 8192, use_graph: bool = True,
                     summary_tokens: int = 128, kv_cache_gb: float | None = None) -> dict:
    """Multi-repository ingest (the reference's DEV_MODE batch: every repo of a user) through
    ``IngestController.ingest_many`` on ONE engine: ``n_repos`` synthetic repositories of ``n_files`` files,
    ``concurrency`` of them at once (default: all).  Returns docs/s with the sequential figure's setup."""
    dev = torch.device(getattr(model, "device", "cpu"))
    sizes = tuple(sorted({*EngineConfig.graph_batch_sizes, *range(256, max_num_seqs + 1, 128), max_num_seqs}))
    eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=max_num_seqs, max_num_batched_tokens=16384,
                                             max_model_len=max_model_len, use_cuda_graph=use_graph, seed=seed,
                                             kv_cache_gb=kv_cache_gb,
                                             graph_batch_sizes=tuple(b for b in sizes if b <= max_num_seqs)))
    if use_graph and dev.type == "cuda":
        ctxs = sorted({c for c in (2048, 4096, max_model_len) if c <= max_model_len})
        eng.warmup_graphs(max_ctx=ctxs, windows=(1, 2, 4, 8),
                          params=SamplingParams(temperature=EngineLLM.INGEST["temperature"],
                                                top_p=EngineLLM.INGEST["top_p"]),
                          cascade=(False, True))
    runner = EngineRunner(eng)
    try:
        llm = EngineLLM(runner, tok, max_tokens=summary_tokens, mode="ingest", timeout_s=3600.0, retries=0)
        store = VectorStore(emb.dim, dev)
        ctl = IngestController(llm=llm, store=store, embedder=emb, settings=Settings(data_dir=None),
                               summary_tokens=summary_tokens)
        items, n_docs = [], 0
        for r in range(n_repos):
            name = f"bench-multi-{seed}-{r}"
            _, files = synthetic_repo(seed * 1000 + r, n_files, name)
            docs = [Document(f["text"], {"file_path": f["file_path"], "file_name": f["file_path"].split("/")[-1]})
                    for f in files]
            n_docs += len(docs)
            items.append({"repo": name, "namespace": "bench", "documents": docs, "force": True})
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = ctl.ingest_many(items, concurrency=concurrency or n_repos)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        return {"repos": n_repos, "files_per_repo": n_files, "concurrency": concurrency or n_repos,
                "docs": n_docs, "seconds": round(dt, 2), "docs_per_s": round(n_docs / dt, 3),
                "ok": all(r.get("ok") for r in res),
                "engine": {k: (round(v, 4) if isinstance(v, float) else v) for k, v in eng.stats.items()
                           if isinstance(v, (int, float))}}
    finally:
        runner.shutdown()
        del eng
        if dev.type == "cuda":
            torch.cuda.empty_cache()


def critical_path(trace: list, t0: float, total: float, bucket: float = 1.0) -> dict:
    """Where the ingest wall time went, from the engine's per-step trace (engine/llm_engine.py ``trace``):
    totals per step kind, the engine-idle remainder (host work, waits between dependent waves), and a
    per-``bucket`` timeline of prefill / decode / capture seconds and mean decode rows — the decode-step
    count is the length of the dependent generation chain (file -> module -> repo summaries -> extractors)."""
    tot = {"prefill_s": 0.0, "decode_s": 0.0, "capture_s": 0.0, "prefill_tokens": 0, "decode_steps": 0,
           "decode_tokens": 0}
    nb = max(1, int(total / bucket) + 1)
    tl = [{"t": round(i * bucket, 1), "prefill_s": 0.0, "decode_s": 0.0, "capture_s": 0.0, "rows": 0, "steps": 0}
          for i in range(nb)]
    for ts, kind, rows, toks, sec in trace:
        b = tl[min(nb - 1, max(0, int((ts - t0) / bucket)))]
        if kind == "capture":
            tot["capture_s"] += sec
            b["capture_s"] += sec
        elif kind == "decode":
            tot["decode_s"] += sec
            tot["decode_steps"] += 1
            tot["decode_tokens"] += toks
            b["decode_s"] += sec
            b["rows"] += rows
            b["steps"] += 1
        else:
            tot["prefill_s"] += sec
            tot["prefill_tokens"] += toks
            b["prefill_s"] += sec
    busy = tot["prefill_s"] + tot["decode_s"]  # decode_s includes captures made inside a decode step
    out = {k: round(v, 3) if isinstance(v, float) else v for k, v in tot.items()}
    out["engine_idle_s"] = round(max(0.0, total - busy), 3)
    out["mean_decode_step_ms"] = round(1000 * tot["decode_s"] / max(1, tot["decode_steps"]), 2)
    out["buckets"] = [{"t": b["t"], "prefill_s": round(b["prefill_s"], 2), "decode_s": round(b["decode_s"], 2),
                       "capture_s": round(b["capture_s"], 2),
                       "mean_rows": round(b["rows"] / b["steps"], 1) if b["steps"] else 0} for b in tl]
    return out
