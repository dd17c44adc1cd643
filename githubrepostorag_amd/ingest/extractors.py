"""LLM metadata extractors as batched waves (SURVEY §2.4, Appendix D:
LlamaIndex SummaryExtractor / TitleExtractor / KeywordExtractor used at
ingest/src/app/services/code_pipeline_service.py:23-51 and
pipelines/catalog_pipeline.py:19-21).

The reference issued these calls one after another against a vLLM pod with
``--max-num-seqs 4``; ingest was LLM-bound.  Here every wave
(all summaries of a repo, then all keyword prompts, ...) is submitted at once
and the engine's continuous batching runs them together.  Prompts put the
chunk text first ("Here is the content of the section: ...") for every
extractor so the summary and keyword prompts of one chunk share a KV prefix
(prefix cache hit on the second one).  Failures are isolated per extractor
like the reference's try/except blocks.
"""
from __future__ import annotations

import logging
from collections import defaultdict
from concurrent.futures import ThreadPoolExecutor

from ..agent import prompts
from .readers import Node

log = logging.getLogger(__name__)


class LLMWave:
    """Run many completions concurrently through one LLM client."""

    def __init__(self, llm, max_parallel: int = 256):
        self.llm = llm
        self.max_parallel = max_parallel
        self.calls = 0

    def map(self, prompt_list: list[str], **kw) -> list[str]:
        if not prompt_list:
            return []
        self.calls += len(prompt_list)
        many = getattr(self.llm, "complete_many", None)
        if many is not None:  # engine client: one submission of the whole wave
            try:
                return [r.text.strip() for r in many(prompt_list, **kw)]
            except Exception as e:  # extractor failures never abort ingest
                log.warning("extractor wave failed: %s", e)
                return [f"Error: {e}"] * len(prompt_list)

        def one(p):
            try:
                return self.llm.complete(p, **kw).text.strip()
            except Exception as e:  # extractor failures never abort ingest
                log.warning("extractor call failed: %s", e)
                return f"Error: {e}"

        with ThreadPoolExecutor(max_workers=min(self.max_parallel, len(prompt_list))) as ex:
            return list(ex.map(one, prompt_list))


def _shared_prefix(context: str) -> str:
    return f"Here is the content of the section:\n{context}\n\n"


def extract_summaries(nodes: list[Node], wave: LLMWave, max_tokens: int = 256, **kw) -> None:
    outs = wave.map([prompts.summary_extract(n.get_content()) for n in nodes], max_tokens=max_tokens, **kw)
    for n, o in zip(nodes, outs):
        n.metadata["section_summary"] = o


def extract_keywords(nodes: list[Node], wave: LLMWave, n_keywords: int = 10, max_tokens: int = 64, **kw) -> None:
    ps = [_shared_prefix(n.get_content()) + f"Give {n_keywords} unique keywords for this document. "
          "Format as comma separated. Keywords: " for n in nodes]
    outs = wave.map(ps, max_tokens=max_tokens, **kw)
    for n, o in zip(nodes, outs):
        n.metadata["excerpt_keywords"] = o


def extract_titles(nodes: list[Node], wave: LLMWave, nodes_per_doc: int = 5, max_tokens: int = 32, **kw) -> None:
    by_doc = defaultdict(list)
    for n in nodes:
        by_doc[n.metadata.get("source_doc_id") or n.metadata.get("file_path") or ""].append(n)
    docs = list(by_doc.items())
    cand_prompts, owners = [], []
    for key, ns in docs:
        for n in ns[:nodes_per_doc]:
            cand_prompts.append(_shared_prefix(n.get_content()) + "Give a title that summarizes all of the unique "
                                "entities, titles or themes found in the context. Title: ")
            owners.append(key)
    cands = wave.map(cand_prompts, max_tokens=max_tokens, **kw)
    per_doc = defaultdict(list)
    for k, c in zip(owners, cands):
        per_doc[k].append(c)
    keys = [k for k, _ in docs]
    combined = wave.map([prompts.title_combine(per_doc[k]) for k in keys], max_tokens=max_tokens, **kw)
    for (k, ns), t in zip(docs, combined):
        for n in ns:
            n.metadata["document_title"] = t


class ExtractorPipeline:
    """Summary -> Title(nodes=N) -> Keywords, each guarded."""

    def __init__(self, llm, title_nodes: int = 5, summary_tokens: int = 256, keyword_tokens: int = 64,
                 title_tokens: int = 32, enabled: bool = True):
        self.wave = LLMWave(llm)
        self.title_nodes = title_nodes
        self.summary_tokens = summary_tokens
        self.keyword_tokens = keyword_tokens
        self.title_tokens = title_tokens
        self.enabled = enabled

    def run(self, nodes: list[Node], priority: int = 0) -> list[Node]:
        """The three extractors are independent reads of the same nodes (each
        writes its own metadata key), so their waves are submitted together:
        one engine batch instead of three back-to-back ones (the reference ran
        them sequentially, code_pipeline_service.py:23-51).  ``priority``:
        engine admission priority of the waves (critical-path passes)."""
        if not self.enabled or not nodes:
            return nodes
        kw = {"priority": priority} if priority else {}
        jobs = (("summary", lambda: extract_summaries(nodes, self.wave, self.summary_tokens, **kw)),
                ("title", lambda: extract_titles(nodes, self.wave, self.title_nodes, self.title_tokens, **kw)),
                ("keywords", lambda: extract_keywords(nodes, self.wave, 10, self.keyword_tokens, **kw)))

        def guarded(item):
            name, fn = item
            try:
                fn()
            except Exception:
                log.exception("%s extraction failed", name)

        with ThreadPoolExecutor(max_workers=len(jobs)) as ex:
            list(ex.map(guarded, jobs))
        return nodes
