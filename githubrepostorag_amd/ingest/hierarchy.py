"""Hierarchical roll-up summaries file -> module -> repo and the catalog
document (ingest/src/app/services/hierarchy_summary_service.py:13-202,
catalog/catalog_builder.py:8-194, services/catalog_service.py:12-39).

Each level is one batched LLM wave (every file summary of a repo at once,
then every module summary; the ingest controller pipelines the two per module,
``file_module_pipeline``), then the "catalog pipeline"
(SentenceSplitter(1500,100) + Summary + Title(3) + Keyword extractors,
pipelines/catalog_pipeline.py:10-23) runs over the produced documents.
Truncation semantics match the reference: 25 000 chars per roll-up input,
40 files per module, 3 READMEs + 10 modules for the repo overview, README
quality check on the first 1 000 chars, <= 10 code summaries for the catalog.
"""
from __future__ import annotations

import logging
import threading
import time
from concurrent.futures import ThreadPoolExecutor

from ..agent import prompts
from .extractors import ExtractorPipeline, LLMWave
from .preprocess import group_files_by_module, group_nodes_by_file, top_directory
from .readers import Document, Node
from .splitters import SentenceSplitter

log = logging.getLogger(__name__)
# the file -> module -> repo chain is the ingest critical path: its waves are
# admitted ahead of the bulk extractor waves running beside them
ROLLUP_PRIORITY = 1


class HierarchyBuilder:
    def __init__(self, llm, extractors: ExtractorPipeline | None = None, summary_tokens: int = 512):
        self.wave = LLMWave(llm)
        self.extract = extractors or ExtractorPipeline(llm, title_nodes=3)
        self.summary_tokens = summary_tokens
        self.splitter = SentenceSplitter(1500, 100)

    def _catalog_pipeline(self, docs: list[Document]) -> list[Node]:
        # the catalog sits on the ingest critical path: its extractor pass jumps the bulk chunk waves
        return self.extract.run(self.splitter.get_nodes_from_documents(docs), priority=ROLLUP_PRIORITY)

    def file_nodes(self, code_nodes: list[Node], repo: str, namespace: str, branch: str, kind: str) -> list[Node]:
        return self.extract.run(self.file_summary_nodes(code_nodes, repo, namespace, branch, kind))

    def module_nodes(self, file_nodes: list[Node], repo: str, namespace: str, branch: str, kind: str,
                     depth: int = 1, max_files: int = 40) -> list[Node]:
        return self.extract.run(self.module_summary_nodes(file_nodes, repo, namespace, branch, kind, depth, max_files))

    def repo_nodes(self, docs: list[Document], module_nodes: list[Node], repo: str, namespace: str, branch: str,
                   kind: str, readme_limit: int = 3, module_limit: int = 10) -> list[Node]:
        return self.extract.run(self.repo_summary_nodes(docs, module_nodes, repo, namespace, branch, kind,
                                                        readme_limit, module_limit))

    # The *_summary_nodes steps produce a level's split nodes WITHOUT the
    # extractor passes: the next level reads only the summary text, so the
    # controller runs a level's extractors concurrently with the next level.
    def file_summary_nodes(self, code_nodes: list[Node], repo: str, namespace: str, branch: str,
                           kind: str) -> list[Node]:
        files = [(fp, ns) for fp, ns in group_nodes_by_file(code_nodes).items() if fp]
        concat = ["\n\n".join(n.get_content() for n in ns)[:25000] for _, ns in files]
        texts = self.wave.map([prompts.file_summary_prompt(fp, c) for (fp, _), c in zip(files, concat)],
                              max_tokens=self.summary_tokens, priority=ROLLUP_PRIORITY)
        docs = []
        for (fp, ns), t in zip(files, texts):
            t = t or f"{fp} summary unavailable."
            docs.append(Document(t, {"namespace": namespace, "repo": repo, "branch": branch, "file_path": fp,
                                     "module": top_directory(fp, 1), "component_kind": kind, "doc_type": "file",
                                     "rollup_of": [n.id for n in ns], "rollup_count": len(ns)}))
        return self.splitter.get_nodes_from_documents(docs)

    def module_summary_nodes(self, file_nodes: list[Node], repo: str, namespace: str, branch: str, kind: str,
                             depth: int = 1, max_files: int = 40) -> list[Node]:
        summaries, ids = {}, {}
        for n in file_nodes:
            fp = (n.metadata.get("file_path") or "").strip()
            if fp:
                summaries.setdefault(fp, n.get_content())
                ids.setdefault(fp, n.id)
        mods = [(m, fs) for m, fs in group_files_by_module(list(summaries), depth).items() if m]
        joined = ["\n\n".join(summaries[f] for f in fs[:max_files])[:25000] for _, fs in mods]
        texts = self.wave.map([prompts.module_summary(m, repo) + "\n\n" + j for (m, _), j in zip(mods, joined)],
                              max_tokens=self.summary_tokens, priority=ROLLUP_PRIORITY)
        docs = [Document(t or f"{m} module summary unavailable.",
                         {"namespace": namespace, "repo": repo, "branch": branch, "module": m, "component_kind": kind,
                          "doc_type": "module", "rollup_of": [ids[f] for f in fs[:max_files] if f in ids],
                          "constituent_files": fs[:max_files]})
                for (m, fs), t in zip(mods, texts)]
        return self.splitter.get_nodes_from_documents(docs)

    def file_module_pipeline(self, code_nodes: list[Node], repo: str, namespace: str, branch: str, kind: str,
                             depth: int = 1, max_files: int = 40, marks: dict | None = None
                             ) -> tuple[list[Node], list[Node]]:
        """file_summary_nodes then module_summary_nodes, pipelined per module: a module's summary is
        submitted as soon as ITS files' summaries are back, not after the slowest file of the repo, so
        the file -> module -> repo chain costs about one file wave + one module wave on its slowest
        module instead of two full waves (same prompts, same outputs as the two level functions).
        ``marks`` receives the wall times when the last file / module summary finished."""
        files = [(fp, ns) for fp, ns in group_nodes_by_file(code_nodes).items() if fp]
        by_mod = group_files_by_module([fp for fp, _ in files], depth)
        nodes_of = dict(files)
        t0 = time.perf_counter()
        done_files = [0.0]
        lock = threading.Lock()

        def one_module(item):
            m, fps = item
            concat = ["\n\n".join(n.get_content() for n in nodes_of[fp])[:25000] for fp in fps]
            texts = self.wave.map([prompts.file_summary_prompt(fp, c) for fp, c in zip(fps, concat)],
                                  max_tokens=self.summary_tokens, priority=ROLLUP_PRIORITY)
            with lock:
                done_files[0] = max(done_files[0], time.perf_counter() - t0)
            fdocs = [Document(t or f"{fp} summary unavailable.",
                              {"namespace": namespace, "repo": repo, "branch": branch, "file_path": fp,
                               "module": top_directory(fp, 1), "component_kind": kind, "doc_type": "file",
                               "rollup_of": [n.id for n in nodes_of[fp]], "rollup_count": len(nodes_of[fp])})
                     for fp, t in zip(fps, texts)]
            fnodes = self.splitter.get_nodes_from_documents(fdocs)
            if not m:  # root-level files have no module roll-up
                return fnodes, []
            first = {}
            for n in fnodes:
                first.setdefault(n.metadata.get("file_path"), n)
            keep = [fp for fp in fps if fp in first][:max_files]
            joined = "\n\n".join(first[fp].get_content() for fp in keep)[:25000]
            t = self.wave.map([prompts.module_summary(m, repo) + "\n\n" + joined], max_tokens=self.summary_tokens,
                              priority=ROLLUP_PRIORITY)[0]
            mdoc = Document(t or f"{m} module summary unavailable.",
                            {"namespace": namespace, "repo": repo, "branch": branch, "module": m,
                             "component_kind": kind, "doc_type": "module",
                             "rollup_of": [first[fp].id for fp in keep], "constituent_files": keep})
            return fnodes, self.splitter.get_nodes_from_documents([mdoc])

        items = list(by_mod.items())
        with ThreadPoolExecutor(max_workers=max(1, min(64, len(items)))) as ex:
            res = list(ex.map(one_module, items))
        if marks is not None:
            marks["file_summaries"] = done_files[0]
            marks["module_summaries"] = time.perf_counter() - t0
        return [n for f, _ in res for n in f], [n for _, mn in res for n in mn]

    def repo_summary_nodes(self, docs: list[Document], module_nodes: list[Node], repo: str, namespace: str,
                           branch: str, kind: str, readme_limit: int = 3, module_limit: int = 10) -> list[Node]:
        readmes = [d.text for d in docs if d.metadata.get("file_path", "").lower().endswith("readme.md")][:readme_limit]
        mods = module_nodes[:module_limit]
        seeds = "\n\n".join(readmes + [m.get_content() for m in mods])[:25000]
        text = self.wave.map([prompts.repo_overview(repo) + "\n\n" + seeds], max_tokens=self.summary_tokens,
                             priority=ROLLUP_PRIORITY)[0]
        doc = Document(text or f"{repo}: overview unavailable.",
                       {"namespace": namespace, "repo": repo, "branch": branch, "component_kind": kind,
                        "doc_type": "repo", "rollup_of": [m.id for m in mods],
                        "constituent_modules": [m.metadata.get("module", "") for m in mods if m.metadata.get("module")]})
        return self.splitter.get_nodes_from_documents([doc])

    # ---- catalog (catalog_builder.make_catalog_document) ------------------
    def catalog_nodes(self, repo: str, docs: list[Document], code_nodes: list[Node], collection: str, kind: str,
                      layer: str | None = None) -> list[Node]:
        readme = "\n\n".join(d.text for d in docs
                             if d.metadata.get("file_path", "").lower().endswith(("readme.md", "readme.txt"))
                             or d.metadata.get("file_path", "").lower() == "readme")
        good = False
        if readme and len(readme.strip()) >= 50:
            verdict = self.wave.map([prompts.readme_quality(readme)], max_tokens=8, priority=ROLLUP_PRIORITY)[0]
            if verdict.startswith("Error"):
                good = len(readme.strip()) > 200 and "todo" not in readme.lower()
            else:
                good = verdict.strip().upper() == "GOOD"
        if readme and good:
            text = f"# PROJECT OVERVIEW\n{readme}"
        elif code_nodes:
            sums, exts = [], set()
            for n in code_nodes:
                s = n.metadata.get("section_summary", "") or n.get_content()[:200]
                fp = n.metadata.get("file_path", "unknown")
                if s and len(s.strip()) > 20:
                    sums.append(f"File: {fp}\nSummary: {s}")
                if fp != "unknown" and "." in fp:
                    exts.add(fp.rsplit(".", 1)[-1].lower())
            tech = ", ".join(sorted(exts)) or "unknown"
            text = self.wave.map([prompts.catalog_from_summaries(repo, tech, "\n\n---\n\n".join(sums[:10]))],
                                 max_tokens=self.summary_tokens, priority=ROLLUP_PRIORITY)[0]
        else:
            text = f"# PROJECT OVERVIEW\n{readme}" if readme else f"Component summary placeholder for {repo}."
        doc = Document(text, {"doc_type": "catalog", "repo": repo, "layer": layer or "unspecified",
                              "collection": collection, "component_kind": kind,
                              "generated_from_code_summaries": bool(code_nodes) and not (readme and good)})
        return self._catalog_pipeline([doc])
