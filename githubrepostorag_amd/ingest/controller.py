"""Ingest controller (ingest/src/app/ingest_controller.py:164-542).

``ingest_component`` runs the same stages as the reference, each under a
``stage_timer`` that records ``ingest_stage_run_seconds`` (and pushes it to a
Prometheus push-gateway when one is configured and reachable):

  preprocess -> code_nodes -> catalog -> file_summaries -> module_summaries
  -> repo_summaries -> vector_write -> audit_and_clean

The LLM stages go through the in-process engine (batched waves, see
extractors.py) instead of an HTTP vLLM pod; vectors land in the GPU store.
Additions: content-hash resume markers under ``DATA_DIR/repos/<repo>/``
(an unchanged repo is skipped unless ``force``), audit rows appended to the
store manifest and ``DATA_DIR/ingest_runs.jsonl`` (replaces the Cassandra
``ingest_runs`` table), and source selection (github / local / synthetic).
"""
from __future__ import annotations

import hashlib
import json
import logging
import math
import os
import time
import uuid
from concurrent.futures import ThreadPoolExecutor
from datetime import datetime, timezone
from pathlib import Path

from ..config import settings as get_settings
from ..service import metrics as M
from .extractors import ExtractorPipeline
from .hierarchy import ROLLUP_PRIORITY, HierarchyBuilder
from .preprocess import infer_component_kind, prepare_repo_documents, top_directory
from .readers import GithubReader, LocalDirReader, SyntheticRepoReader, fetch_repositories
from .splitters import DynamicCodeSplitter
from .writer import VectorWriter

log = logging.getLogger(__name__)
CATALOG_HEAD = 16  # chunks extracted first: the catalog uses the first 10 summaries (> 20 chars)

DOC_TYPE_TO_SCOPE = {"catalog": "catalog", "repo": "repo", "module": "module", "file": "file"}


class stage_timer:
    def __init__(self, level: str, *, repo: str, namespace: str, branch: str, run_id: str, timings: dict,
                 push_addr: str | None = None, on_stage=None):
        self.level, self.labels = level, dict(repo=repo, namespace=namespace, branch=branch, run_id=run_id)
        self.timings, self.push_addr, self.on_stage = timings, push_addr, on_stage

    def __enter__(self):
        self.t0 = time.perf_counter()
        if self.on_stage:
            self.on_stage(self.level, self.labels)
        return self

    def __exit__(self, exc_type, exc, tb):
        self.record(time.perf_counter() - self.t0)
        return False

    def record(self, dt: float) -> None:
        """Report a stage duration measured elsewhere (a stage that overlaps another)."""
        if not math.isfinite(dt):
            return
        self.timings[self.level] = dt
        M.INGEST_STAGE_SECONDS.labels(level=self.level, **self.labels).set(dt)
        _push("ingest_stage_run_seconds", "Duration (seconds) of a single ingest stage for a single run",
              {"level": self.level, **self.labels}, dt, self.push_addr)


def _push(name: str, help_text: str, labels: dict, value: float, addr: str | None) -> None:
    if not addr or os.environ.get("PUSHGATEWAY_ADDRESS") is None:
        return  # only push when explicitly configured
    try:
        from prometheus_client import CollectorRegistry, Gauge, push_to_gateway

        reg = CollectorRegistry()
        g = Gauge(name, help_text, list(labels), registry=reg)
        g.labels(**labels).set(value)
        push_to_gateway(addr, job="ingest_component", registry=reg, grouping_key={"run_id": labels.get("run_id", "")},
                        timeout=2)
    except Exception:
        log.debug("push-gateway push failed", exc_info=True)


def attach_common_metadata(nodes, *, namespace, repo, branch, collection, component_kind, is_standalone, run_id,
                           dev_forced, doc_type) -> None:
    for n in nodes:
        md = n.metadata
        md.update(namespace=namespace, repo=repo, branch=branch, collection=collection, component_kind=component_kind,
                  is_standalone=is_standalone, dev_forced_standalone=dev_forced, ingest_run_id=str(run_id))
        md.setdefault("doc_type", doc_type)
        md.setdefault("path", md.get("file_path"))
        if md.get("file_path") and "module" not in md:
            # chunks get their module too (the reference never sets it, so its
            # module edge/filter is empty at code scope: SURVEY §2.11-10)
            md["module"] = top_directory(md["file_path"], 1)
        md["scope"] = DOC_TYPE_TO_SCOPE.get(doc_type, "chunk")


def docs_digest(docs) -> str:
    h = hashlib.sha1()
    for d in sorted(docs, key=lambda d: d.metadata.get("file_path", "")):
        h.update(d.metadata.get("file_path", "").encode())
        h.update(hashlib.sha1(d.text.encode("utf-8", "replace")).digest())
    return h.hexdigest()


class IngestController:
    def __init__(self, runtime=None, *, llm=None, store=None, embedder=None, settings=None, extract: bool = True,
                 summary_tokens: int | None = None, on_event=None, token_cap: int | None = None):
        self.s = settings or (runtime.settings if runtime is not None else get_settings())
        self.llm = llm or runtime.ingest_llm
        self.store = store or runtime.store
        self.embedder = embedder or runtime.embedder
        self.runtime = runtime
        self.on_event = on_event or (lambda kind, data: None)
        toks = summary_tokens or 256
        # token_cap: ONE generation cap for every ingest LLM call (summaries, titles, keywords, roll-ups) —
        # the reference's ingest LLM runs every call with max_new_tokens=2048 (ingest/src/app/llm_init.py:56)
        caps = dict(keyword_tokens=token_cap, title_tokens=token_cap) if token_cap else {}
        self.extractors = ExtractorPipeline(self.llm, title_nodes=5, summary_tokens=token_cap or toks,
                                            enabled=extract, **caps)
        self.hier = HierarchyBuilder(self.llm, ExtractorPipeline(self.llm, title_nodes=3,
                                                                 summary_tokens=token_cap or toks, enabled=extract,
                                                                 **caps), summary_tokens=token_cap or 2 * toks)
        self.writer = VectorWriter(self.store, self.embedder)
        self.splitter = DynamicCodeSplitter()

    # ---- sources ---------------------------------------------------------
    def _reader(self, source: str, path: str | None):
        if source == "github":
            return GithubReader(self.s.github_user, self.s.github_token)
        if source == "local":
            if not path:
                raise ValueError("source=local needs a path")
            return LocalDirReader(path)
        return SyntheticRepoReader()

    def _data_dir(self) -> Path | None:
        return Path(self.s.data_dir) if self.s.data_dir else None

    # ---- one component ---------------------------------------------------
    def ingest_component(self, *, repo: str, namespace: str, branch: str | None = None, layer: str | None = None,
                         collection: str | None = None, component_kind: str | None = None,
                         dev_force_standalone: bool | None = None, source: str = "synthetic",
                         path: str | None = None, documents=None, force: bool = False) -> dict:
        t_run = time.perf_counter()
        branch = branch or self.s.default_branch
        collection = collection or self.s.default_collection
        forced = bool(dev_force_standalone)
        run_id = uuid.uuid4()
        started = datetime.now(timezone.utc)
        timings: dict = {}
        self.on_event("ingest_start", {"repo": repo, "namespace": namespace, "branch": branch,
                                       "collection": collection, "force": forced})

        def timer(level):
            return stage_timer(level, repo=repo, namespace=namespace, branch=branch, run_id=str(run_id),
                               timings=timings, push_addr=self.s.pushgateway_address,
                               on_stage=lambda lv, lab: self.on_event("step", {"stage": lv, **lab}))

        with timer("preprocess"):
            raw = documents if documents is not None else self._reader(source, path).load_data(repo, branch)
            docs = prepare_repo_documents(raw)
            kind = "standalone" if forced else (component_kind or infer_component_kind(docs))
            is_sa = kind == "standalone"
            digest = docs_digest(docs)
            dd = self._data_dir()
            marker = dd / "repos" / repo / f".ingested_{branch}" if dd else None
            if marker is not None and marker.exists() and not force and marker.read_text().strip() == digest:
                log.info("%s@%s unchanged since last ingest; skipping", repo, branch)
                return {"repo": repo, "namespace": namespace, "branch": branch, "skipped": True,
                        "nodes_written": 0, "component_kind": kind}
            if dd:
                (dd / "repos" / repo).mkdir(parents=True, exist_ok=True)
                with open(dd / "repos" / repo / f"raw_documents_{branch}.json", "w") as f:
                    json.dump([{"id": d.id, "text": d.text, "metadata": d.metadata} for d in docs], f)
        common = dict(namespace=namespace, repo=repo, branch=branch, collection=collection, component_kind=kind,
                      is_standalone=is_sa, dev_forced=forced)
        # Stage DAG (the reference ran these 6 stages strictly in sequence,
        # ingest_controller.py:249-389): the chunk extractors + catalog branch
        # and the file -> module -> repo roll-up branch only share the split
        # chunks, and each level's extractor passes run beside the next level's
        # summary wave, so the engine sees a few large batches instead of many
        # small serial ones.  Stage timers overlap accordingly.
        with timer("split"):
            split_nodes = self.splitter.get_nodes_from_documents(docs)
        pool = ThreadPoolExecutor(max_workers=5)
        try:
            def code_branch():
                # the catalog reads the first <= 10 code-chunk summaries
                # (catalog_builder.py:140-194): extract those first, at roll-up
                # priority, and build the catalog while the bulk extractor
                # waves over the remaining chunks run
                head, rest = split_nodes[:CATALOG_HEAD], split_nodes[CATALOG_HEAD:]
                with timer("code_nodes"):
                    self.extractors.run(head, priority=ROLLUP_PRIORITY)
                    f_rest = pool.submit(self.extractors.run, rest)
                    with timer("catalog"):
                        cat = self.hier.catalog_nodes(repo, docs, split_nodes, collection, kind, layer)
                    f_rest.result()
                return split_nodes, cat

            f_code = pool.submit(code_branch)
            # file -> module roll-ups pipelined per module (a module's summary starts when its own files
            # are summarised); stage marks record when the last file / module summary finished
            marks: dict = {}
            with timer("module_summaries"):
                file_nodes, module_nodes = self.hier.file_module_pipeline(split_nodes, repo, namespace, branch, kind,
                                                                          marks=marks)
            timer("file_summaries").record(marks.get("file_summaries", 0.0))
            f_file_ext = pool.submit(self.hier.extract.run, file_nodes)
            f_mod_ext = pool.submit(self.hier.extract.run, module_nodes)
            with timer("repo_summaries"):
                repo_nodes = self.hier.extract.run(
                    self.hier.repo_summary_nodes(docs, module_nodes, repo, namespace, branch, kind),
                    priority=ROLLUP_PRIORITY)
            with timer("extract_wait"):
                code_nodes, catalog_nodes = f_code.result()
                f_file_ext.result()
                f_mod_ext.result()
        finally:
            pool.shutdown(wait=True)
        attach_common_metadata(code_nodes, run_id=run_id, doc_type="code", **common)
        attach_common_metadata(catalog_nodes, run_id=uuid.UUID(int=0), doc_type="catalog", **common)
        attach_common_metadata(file_nodes, run_id=run_id, doc_type="file", **common)
        attach_common_metadata(module_nodes, run_id=run_id, doc_type="module", **common)
        attach_common_metadata(repo_nodes, run_id=run_id, doc_type="repo", **common)
        with timer("vector_write"):
            written = self.writer.write_nodes_per_scope(catalog_nodes=catalog_nodes, repo_nodes=repo_nodes,
                                                        module_nodes=module_nodes, file_nodes=file_nodes,
                                                        chunk_nodes=code_nodes)
        with timer("audit_and_clean"):
            row = {"run_id": str(run_id), "namespace": namespace, "repo": repo, "branch": branch,
                   "collection": collection, "component_kind": kind, "started_at": started.isoformat(),
                   "finished_at": datetime.now(timezone.utc).isoformat(), "node_count": len(code_nodes),
                   "nodes_per_scope": written}
            self.store.audit.append(row)
            if dd:
                with open(dd / "ingest_runs.jsonl", "a") as f:
                    f.write(json.dumps(row) + "\n")
                marker.write_text(digest)
            if self.runtime is not None and self.s.index_dir:
                self.runtime.save_index()
        total = time.perf_counter() - t_run
        M.INGEST_RUN_SECONDS.labels(repo=repo, namespace=namespace, branch=branch, run_id=str(run_id)).set(total)
        M.INGEST_DOCS.inc(len(docs))
        _push("ingest_run_seconds", "Total duration (seconds) of a single ingest run",
              {"repo": repo, "namespace": namespace, "branch": branch, "run_id": str(run_id)}, total,
              self.s.pushgateway_address)
        res = {"ok": True, "run_id": str(run_id), "repo": repo, "namespace": namespace, "collection": collection,
               "component_kind": kind,
               "branch": branch, "nodes_written": len(code_nodes), "is_standalone": is_sa,
               "dev_forced_standalone": forced, "documents": len(docs), "nodes_per_scope": written,
               "stage_seconds": {k: round(v, 4) for k, v in timings.items()}, "run_seconds": round(total, 4)}
        self.on_event("ingest_done", res)
        return res

    # ---- batch driver (ingest_controller.py:490-542) ---------------------
    def ingest_many(self, components, *, branch: str | None = None, dev_force_standalone: bool | None = None,
                    source: str = "synthetic", path: str | None = None, concurrency: int | None = None) -> list[dict]:
        """Every component of the batch (the reference's DEV_MODE: every public repo of the user), up to
        ``concurrency`` (settings INGEST_CONCURRENCY) at once on the one engine: each repository's pipeline
        ends in a dependent roll-up chain (file -> module -> repo -> catalog) of small decode batches, and
        the next repository's extractor waves fill those steps (the reference ingests one repository after
        another, ingest_controller.py:506-516).  Results in input order; a failed component raises after
        the others finished, as the sequential loop would have stopped at it."""
        default_branch = branch or self.s.default_branch
        items = []
        if dev_force_standalone and source == "github":
            for repo in fetch_repositories(self.s.github_user, self.s.github_token):
                items.append({"repo": repo, "namespace": "default", "branch": default_branch,
                              "dev_force_standalone": True})
        else:
            for it in components:
                if isinstance(it, dict):
                    p = dict(it)
                    p.setdefault("branch", default_branch)
                    p.setdefault("dev_force_standalone", dev_force_standalone)
                else:
                    it = list(it)
                    p = {"repo": it[0], "namespace": it[1], "layer": it[2] if len(it) > 2 else None,
                         "collection": it[3] if len(it) > 3 else None,
                         "component_kind": it[4] if len(it) > 4 else None,
                         "dev_force_standalone": it[5] if len(it) > 5 else dev_force_standalone,
                         "branch": default_branch}
                items.append(p)
        for p in items:
            p.setdefault("source", source)
            p.setdefault("path", path)
        R = max(1, int(concurrency if concurrency is not None else getattr(self.s, "ingest_concurrency", 1)))
        if R == 1 or len(items) <= 1:
            return [self.ingest_component(**p) for p in items]
        with ThreadPoolExecutor(max_workers=min(R, len(items)), thread_name_prefix="ingest-repo") as ex:
            futs = [ex.submit(self.ingest_component, **p) for p in items]
            return [f.result() for f in futs]
