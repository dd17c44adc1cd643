"""Embed + write nodes per scope into the GPU vector store
(ingest/src/app/services/vector_write_service.py:19-209).

Same per-scope allow-lists and keep-always set as the reference's
``_sanitize_doc_metadata`` (values flattened to text, lists comma-joined,
dicts JSON-encoded, None dropped).  List-valued traversal fields
(topics/imports/labels) are "shredded" into the table's multi-valued bloom
column instead of one row per element (store.py).  Differences by design:

* row ids are content hashes of (scope, namespace, repo, module, file_path,
  start/end, text) so a re-ingest of unchanged content overwrites instead of
  duplicating;
* embeddings for ALL scopes are computed in one length-sorted batched pass
  (Embedder.embed_documents) before any table is touched.
"""
from __future__ import annotations

import hashlib
import json
import logging

import torch

from .readers import Node

log = logging.getLogger(__name__)

ALLOW_FIELDS_BY_SCOPE = {
    "catalog": ("namespace", "repo", "owner", "language", "topics", "labels", "component_kind"),
    "repo": ("namespace", "repo", "owner", "language", "topics", "labels"),
    "module": ("namespace", "repo", "module", "language", "topics", "imports", "labels"),
    "file": ("namespace", "repo", "module", "file_path", "language", "topics", "imports", "labels"),
    "chunk": ("namespace", "repo", "module", "file_path", "symbol", "language", "topics", "imports"),
}
KEEP_ALWAYS = ("scope", "namespace", "repo", "module", "file_path", "symbol", "owner", "component_kind", "branch",
               "language", "row_id")
# extra descriptive fields we keep for the answer "sources" (not indexed in the reference either)
KEEP_EXTRA = ("doc_type", "collection", "document_title", "excerpt_keywords", "file_name")
MULTI = ("topics", "imports", "labels")
SCOPE_ORDER = ("catalog", "repo", "module", "file", "chunk")


def to_text(v):
    if v is None:
        return None
    if isinstance(v, str):
        return v
    if isinstance(v, (bool, int, float)):
        return str(v)
    if isinstance(v, (list, tuple, set)):
        return ",".join(map(str, v))
    try:
        return json.dumps(v, ensure_ascii=False, separators=(",", ":"))
    except Exception:
        return str(v)


def sanitize_metadata(md: dict, scope: str) -> dict:
    md = dict(md or {})
    md.setdefault("scope", scope)
    if "path" in md and "file_path" not in md:
        md["file_path"] = md["path"]
    keep = set(ALLOW_FIELDS_BY_SCOPE[scope]) | set(KEEP_ALWAYS) | set(KEEP_EXTRA)
    out = {}
    for k, v in md.items():
        k = str(k)
        if k not in keep:
            continue
        t = to_text(v)
        if t is not None:
            out[k] = t
    return out


def row_id_for(scope: str, node: Node) -> str:
    md = node.metadata
    seed = "|".join(str(md.get(k, "")) for k in ("namespace", "repo", "module", "file_path", "start_char_idx",
                                                 "end_char_idx", "doc_type"))
    h = hashlib.sha1(f"{scope}|{seed}|".encode())
    h.update(node.get_content().encode("utf-8", "replace"))
    return h.hexdigest()


class VectorWriter:
    def __init__(self, store, embedder, batch_size: int = 256):
        self.store = store
        self.embedder = embedder
        self.batch_size = batch_size

    def write_nodes_per_scope(self, *, catalog_nodes=(), repo_nodes=(), module_nodes=(), file_nodes=(),
                              chunk_nodes=()) -> dict:
        per = dict(zip(SCOPE_ORDER, (list(catalog_nodes), list(repo_nodes), list(module_nodes), list(file_nodes),
                                     list(chunk_nodes))))
        texts, owners = [], []
        for s in SCOPE_ORDER:
            for n in per[s]:
                texts.append(n.get_content())
                owners.append(s)
        if not texts:
            return {s: 0 for s in SCOPE_ORDER}
        vecs = self.embedder.embed_documents(texts)
        written, off = {}, 0
        for s in SCOPE_ORDER:
            nodes = per[s]
            if not nodes:
                written[s] = 0
                continue
            v = vecs[off:off + len(nodes)]
            off += len(nodes)
            ids = [row_id_for(s, n) for n in nodes]
            mds = [sanitize_metadata(n.metadata, s) for n in nodes]
            for i in range(0, len(nodes), self.batch_size):
                sl = slice(i, i + self.batch_size)
                self.store.table(s).upsert(ids[sl], [n.get_content() for n in nodes[sl]], v[sl], mds[sl])
            written[s] = len(nodes)
            log.info("wrote %d %s nodes to %s", len(nodes), s, self.store.table_names[s])
        if isinstance(vecs, torch.Tensor) and vecs.is_cuda:
            torch.cuda.current_stream().synchronize()
        return written
