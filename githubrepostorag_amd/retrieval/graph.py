"""Metadata-edge graph retrieval ("GraphRAG", Eager strategy) over the GPU
vector tables — the reference's ``GraphRetriever(store, edges,
Eager(k, start_k, adjacent_k, max_depth))`` (rag_worker/src/worker/services/
graph_rag_retrievers.py:82-134) re-designed for the GPU:

1. seeds: the ``start_k`` most similar rows passing the caller's filter;
2. each traversal depth expands EVERY newly reached node along every edge
   ``(src_field, dst_field)``: nodes whose ``dst_field`` equals the node's
   ``src_field`` value, similarity-ranked against the same query, up to
   ``adjacent_k`` per (edge, value).  The reference issued one filtered ANN
   query per (edge, value) pair; here all pairs of a depth are ONE launch of
   the fused score+top-k kernel with per-query predicates (the query vector
   repeated, each copy carrying its own ``column == value`` test), so a
   two-hop traversal costs two kernel launches regardless of fan-out;
3. stop at ``max_depth``; return up to ``k`` nodes in discovery order with
   ``_depth`` and ``_similarity_score`` metadata (what the reference UI's
   ``score`` field should have shown).
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field

import torch

from ..index.store import Hit, VectorTable
from ..utils.gpu_guard import side_stream


@dataclass
class Document:
    page_content: str
    metadata: dict = field(default_factory=dict)
    id: str = ""
    score: float | None = None


EDGES = {
    "project": [("namespace", "namespace"), ("repo", "repo")],
    "package": [("namespace", "namespace"), ("repo", "repo"), ("module", "module")],
    "file": [("namespace", "namespace"), ("repo", "repo"), ("module", "module"), ("file_path", "file_path")],
    "code": [("namespace", "namespace"), ("repo", "repo"), ("module", "module"), ("file_path", "file_path")],
}


class GraphRetriever:
    def __init__(self, table: VectorTable, embedder, edges, k: int = 10, start_k: int = 2, adjacent_k: int = 10,
                 max_depth: int = 2):
        self.table = table
        self.embedder = embedder
        self.edges = list(edges)
        self.k, self.start_k, self.adjacent_k, self.max_depth = k, start_k, adjacent_k, max_depth
        self.last_stats: dict = {}

    def _doc(self, h: Hit, depth: int) -> Document:
        md = dict(h.metadata)
        md["_depth"] = depth
        md["_similarity_score"] = h.score
        return Document(h.text, md, h.row_id, h.score)

    def invoke(self, query: str, filter: dict | None = None, qvec: torch.Tensor | None = None) -> list[Document]:
        # the embed + every traversal hop share one side stream (utils/gpu_guard.py)
        with side_stream(self.table.device, wait_caller=qvec is not None):
            return self._invoke(query, filter, qvec)

    def _invoke(self, query: str, filter: dict | None, qvec: torch.Tensor | None) -> list[Document]:
        t0 = time.perf_counter()
        tab = self.table
        if qvec is None:
            qvec = self.embedder.embed_query(query)
        q = qvec.reshape(1, -1)
        seeds = tab.search(q, self.start_k, filter)[0]
        out: list[Document] = []
        seen: set[str] = set()
        for h in seeds:
            if h.row_id not in seen:
                seen.add(h.row_id)
                out.append(self._doc(h, 0))
        frontier = list(seeds)
        visited_edges: set[tuple[str, str]] = set()
        launches = 1
        for depth in range(1, self.max_depth + 1):
            if len(out) >= self.k or not frontier:
                break
            pairs = []
            for h in frontier:
                for src, dst in self.edges:
                    v = h.metadata.get(src)
                    if v in (None, ""):
                        continue
                    key = (dst, str(v))
                    if key in visited_edges:
                        continue
                    visited_edges.add(key)
                    pairs.append(key)
            if not pairs:
                break
            found = self._adjacent(q, pairs, filter)
            launches += 1
            nxt = []
            for hits in found:
                for h in hits:
                    if h.row_id in seen:
                        continue
                    seen.add(h.row_id)
                    out.append(self._doc(h, depth))
                    nxt.append(h)
            frontier = nxt
        self.last_stats = {"launches": launches, "seconds": time.perf_counter() - t0, "found": len(out)}
        return out[: self.k]

    def _adjacent(self, q: torch.Tensor, pairs, base_filter) -> list[list[Hit]]:
        """All (dst_field, value) lookups of one depth: one fused launch on a local
        table (``VectorTable.search_pairs``), one fan-out round on a sharded one
        (``index/sharded_store.py``)."""
        return self.table.search_pairs(q, pairs, self.adjacent_k, base_filter)


class RetrieverFactory:
    """The four scope retrievers of the reference agent (agent_graph.py:158-176)."""

    def __init__(self, store, embedder):
        self.store = store
        self.embedder = embedder

    def for_repo(self, k=10, start_k=2, max_depth=2, adjacent_k=10):
        return GraphRetriever(self.store.table("repo"), self.embedder, EDGES["project"], k, start_k, adjacent_k,
                              max_depth)

    def for_module(self, k=8, start_k=2, adjacent_k=6, max_depth=2):
        return GraphRetriever(self.store.table("module"), self.embedder, EDGES["package"], k, start_k, adjacent_k,
                              max_depth)

    def for_file(self, k=8, start_k=2, adjacent_k=6, max_depth=2):
        return GraphRetriever(self.store.table("file"), self.embedder, EDGES["file"], k, start_k, adjacent_k,
                              max_depth)

    def for_chunk(self, k=10, start_k=3, adjacent_k=8, max_depth=2):
        return GraphRetriever(self.store.table("chunk"), self.embedder, EDGES["code"], k, start_k, adjacent_k,
                              max_depth)

    def for_catalog(self, k=5, start_k=2, adjacent_k=4, max_depth=1):
        return GraphRetriever(self.store.table("catalog"), self.embedder, EDGES["project"], k, start_k, adjacent_k,
                              max_depth)

    def scope_retrievers(self) -> dict:
        return {"project": self.for_repo(k=10, start_k=2, max_depth=2),
                "package": self.for_module(k=8, start_k=2, adjacent_k=6, max_depth=2),
                "file": self.for_file(k=8, start_k=2, adjacent_k=6, max_depth=2),
                "code": self.for_chunk(k=10, start_k=3, adjacent_k=8, max_depth=2)}
