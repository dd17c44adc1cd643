"""GPU-resident vector store — replaces the reference's Cassandra 5 SAI vector
tables (helm/templates/cassandra-initdb-configmap.yaml:13-102) and the
LangChain ``Cassandra`` store (vector_write_service.py:136-159,
graph_rag_retrievers.py:68-80).

Layout per scope table (catalog / repo / module / file / chunk):
  * vectors  bf16 [capacity, d] in HBM, L2-normalised (cosine == dot), grown
    geometrically; the live prefix [0, n) is what the kernels scan;
  * metadata columns: every filterable field (the reference's allow-lists,
    vector_write_service.py:28-34, plus scope/namespace/…) is
    dictionary-encoded to int32 on device, so equality filters run inside the
    fused score+top-k kernel instead of a secondary index;
    multi-valued fields (topics/labels/imports — the reference "shreds" them,
    vector_write_service.py:118,153) use a 31-bit bloom bitset column with an
    exact host re-check;
  * a live-row bitmap (deletes / re-ingest tombstones);
  * host side: row_id primary key -> row, body text, full metadata dict.

Upserts are idempotent on ``row_id`` (the reference re-ingest duplicated rows,
SURVEY §2.11 quirk 13): ids are content hashes chosen by the writer.
"""
from __future__ import annotations

import json
import threading
from dataclasses import dataclass
from pathlib import Path

import numpy as np
import torch

from ..ops.topk import OP_BITAND, OP_EQ, Predicate, score_topk
from ..utils.gpu_guard import guarded, side_stream

SCOPES = ("catalog", "repo", "module", "file", "chunk")
DEFAULT_TABLES = {"catalog": "embeddings_catalog", "repo": "embeddings_repo", "module": "embeddings_module",
                  "file": "embeddings_file", "chunk": "embeddings"}
FILTER_FIELDS = ("scope", "namespace", "repo", "module", "file_path", "language", "component_kind", "branch",
                 "owner", "symbol", "doc_type", "collection")
MULTI_FIELDS = ("topics", "labels", "imports")


@dataclass
class Hit:
    row_id: str
    text: str
    metadata: dict
    score: float
    row: int = -1


def _split_multi(v) -> list[str]:
    if v is None:
        return []
    if isinstance(v, (list, tuple, set)):
        return [str(x).strip() for x in v if str(x).strip()]
    return [x.strip() for x in str(v).split(",") if x.strip()]


class VectorTable:
    def __init__(self, name: str, dim: int, device="cpu", capacity: int = 1024, dtype=torch.bfloat16):
        self.name = name
        self.dim = dim
        self.device = torch.device(device)
        self.dtype = dtype
        self.n = 0
        self._cap = max(16, capacity)
        self.vectors = torch.zeros(self._cap, dim, dtype=dtype, device=self.device)
        self.columns = {f: torch.full((self._cap,), -1, dtype=torch.int32, device=self.device)
                        for f in FILTER_FIELDS + MULTI_FIELDS}
        self.dicts: dict[str, dict[str, int]] = {f: {} for f in FILTER_FIELDS + MULTI_FIELDS}
        self.live = torch.zeros((self._cap + 31) // 32, dtype=torch.int32, device=self.device)
        self.row_ids: list[str] = []
        self.texts: list[str] = []
        self.metas: list[dict] = []
        self.key_to_row: dict[str, int] = {}
        self.deleted = 0
        self.lock = threading.RLock()

    # ------------------------------------------------------------------ storage
    def _grow(self, need: int) -> None:
        if need <= self._cap:
            return
        cap = self._cap
        while cap < need:
            cap *= 2
        v = torch.zeros(cap, self.dim, dtype=self.dtype, device=self.device)
        v[: self.n] = self.vectors[: self.n]
        self.vectors = v
        for f, c in self.columns.items():
            nc = torch.full((cap,), -1, dtype=torch.int32, device=self.device)
            nc[: self.n] = c[: self.n]
            self.columns[f] = nc
        lv = torch.zeros((cap + 31) // 32, dtype=torch.int32, device=self.device)
        lv[: self.live.numel()] = self.live
        self.live = lv
        self._cap = cap

    def _code(self, field: str, value) -> int:
        d = self.dicts[field]
        s = str(value)
        if s not in d:
            d[s] = len(d)
        return d[s]

    def _multi_bits(self, field: str, values) -> int:
        bits = 0
        for v in _split_multi(values):
            bits |= 1 << (self._code(field, v) % 31)
        return bits

    def _set_live(self, rows: np.ndarray, alive: bool) -> None:
        words = self.live.cpu().numpy().view(np.uint32).copy()
        for r in rows.tolist():
            if alive:
                words[r >> 5] |= np.uint32(1 << (r & 31))
            else:
                words[r >> 5] &= np.uint32(~(1 << (r & 31)) & 0xFFFFFFFF)
        self.live.copy_(torch.from_numpy(words.view(np.int32)).to(self.device))
        if self.device.type == "cuda":  # searches read the table from other (side) streams
            torch.cuda.current_stream(self.device).synchronize()

    @guarded
    def upsert(self, row_ids: list[str], texts: list[str], vectors: torch.Tensor, metadatas: list[dict]) -> int:
        """Insert or overwrite rows keyed by row_id. vectors [n, d] (any float
        dtype; normalised here).  Returns the number of new rows."""
        n = len(row_ids)
        if n == 0:
            return 0
        vecs = vectors.to(self.device, torch.float32)
        vecs = vecs / vecs.norm(dim=-1, keepdim=True).clamp_min(1e-12)
        with self.lock:
            rows = np.empty(n, dtype=np.int64)
            new = 0
            for i, rid in enumerate(row_ids):
                r = self.key_to_row.get(rid)
                if r is None:
                    r = self.n + new
                    new += 1
                rows[i] = r
            self._grow(self.n + new)
            for i, rid in enumerate(row_ids):
                r = int(rows[i])
                md = dict(metadatas[i] or {})
                if r >= len(self.row_ids):
                    self.row_ids.append(rid)
                    self.texts.append(texts[i])
                    self.metas.append(md)
                    self.key_to_row[rid] = r
                else:
                    self.texts[r] = texts[i]
                    self.metas[r] = md
            self.n += new
            ridx = torch.from_numpy(rows).to(self.device)
            self.vectors[ridx] = vecs.to(self.dtype)
            for f in FILTER_FIELDS:
                codes = [self._code(f, m[f]) if m.get(f) not in (None, "") else -1 for m in metadatas]
                self.columns[f][ridx] = torch.tensor(codes, dtype=torch.int32).to(self.device)
            for f in MULTI_FIELDS:
                codes = [self._multi_bits(f, m.get(f)) for m in metadatas]
                self.columns[f][ridx] = torch.tensor(codes, dtype=torch.int32).to(self.device)
            self._set_live(rows, True)
            return new

    @guarded
    def delete(self, row_ids: list[str]) -> int:
        with self.lock:
            rows = np.asarray([self.key_to_row[r] for r in row_ids if r in self.key_to_row], dtype=np.int64)
            for r in row_ids:
                self.key_to_row.pop(r, None)
            if rows.size:
                self._set_live(rows, False)
                self.deleted += rows.size
            return int(rows.size)

    def count(self) -> int:
        return self.n - self.deleted

    # ------------------------------------------------------------------ filters
    def predicates(self, flt: dict | None):
        """filter dict -> (fused predicates, host checks) or None if a value is
        unknown (nothing can match)."""
        preds, checks = [], []
        for k, v in (flt or {}).items():
            if v is None or v == "":
                continue
            if k in FILTER_FIELDS:
                code = self.dicts[k].get(str(v))
                if code is None:
                    return None
                preds.append(Predicate(self.columns[k], code, OP_EQ))
            elif k in MULTI_FIELDS:
                vals = _split_multi(v)
                for val in vals:
                    code = self.dicts[k].get(val)
                    if code is None:
                        return None
                    preds.append(Predicate(self.columns[k], 1 << (code % 31), OP_BITAND))
                    checks.append((k, val))
            else:  # unindexed field: host-side check only
                checks.append((k, str(v)))
        return preds, checks

    def _host_ok(self, row: int, checks) -> bool:
        md = self.metas[row]
        for k, v in checks:
            if k in MULTI_FIELDS:
                if v not in _split_multi(md.get(k)):
                    return False
            elif str(md.get(k, "")) != v:
                return False
        return True

    # ------------------------------------------------------------------ search
    @guarded
    def search(self, qvecs: torch.Tensor, k: int, flt: dict | None = None, qpred=None) -> list[list[Hit]]:
        """Batched filtered top-k by cosine. qvecs [nq, d]."""
        nq = qvecs.shape[0]
        with self.lock, side_stream(self.device, wait_caller=qvecs.is_cuda):
            if self.n == 0:
                return [[] for _ in range(nq)]
            pc = self.predicates(flt)
            if pc is None:
                return [[] for _ in range(nq)]
            preds, checks = pc
            extra = []
            if len(preds) > 4:
                # AND the overflow predicates into a row bitmap with one torch pass
                m = torch.ones(self.n, dtype=torch.bool, device=self.device)
                for p in preds[4:]:
                    c = p.column[: self.n]
                    m &= (c == p.value) if p.op == OP_EQ else ((c & p.value) != 0)
                extra = m
                preds = preds[:4]
            bitmap = self.live
            if isinstance(extra, torch.Tensor):
                bitmap = _and_bitmap(self.live, extra)
            q = qvecs.to(self.device, self.dtype)
            kk = min(32, k + (8 if checks else 0))
            scores, ids = score_topk(self.vectors[: self.n], q, kk, preds=preds, bitmap=bitmap, qpred=qpred)
            scores, ids = scores.cpu().tolist(), ids.cpu().tolist()
            out = []
            for qi in range(nq):
                hits = []
                for s, r in zip(scores[qi], ids[qi]):
                    if r < 0 or s == float("-inf"):
                        continue
                    if checks and not self._host_ok(r, checks):
                        continue
                    hits.append(Hit(self.row_ids[r], self.texts[r], self.metas[r], float(s), r))
                    if len(hits) >= k:
                        break
                out.append(hits)
            return out

    # ------------------------------------------------------------------ persistence
    def save(self, path: str | Path) -> None:
        path = Path(path)
        path.mkdir(parents=True, exist_ok=True)
        with self.lock:
            from safetensors.torch import save_file

            tensors = {"vectors": self.vectors[: self.n].contiguous().cpu(), "live": self.live.cpu()}
            for f, c in self.columns.items():
                tensors[f"col.{f}"] = c[: self.n].contiguous().cpu()
            tmp = path / "table.safetensors.tmp"
            save_file(tensors, str(tmp))
            tmp.replace(path / "table.safetensors")
            meta = {"name": self.name, "dim": self.dim, "n": self.n, "deleted": self.deleted,
                    "row_ids": self.row_ids, "texts": self.texts, "metas": self.metas, "dicts": self.dicts}
            tmpj = path / "rows.json.tmp"
            tmpj.write_text(json.dumps(meta, ensure_ascii=False))
            tmpj.replace(path / "rows.json")

    @classmethod
    def load(cls, path: str | Path, device="cpu") -> "VectorTable":
        from safetensors.torch import load_file

        path = Path(path)
        meta = json.loads((path / "rows.json").read_text())
        t = load_file(str(path / "table.safetensors"))
        tab = cls(meta["name"], meta["dim"], device=device, capacity=max(16, meta["n"]))
        n = meta["n"]
        tab.n = n
        tab.vectors[:n] = t["vectors"].to(tab.device)
        for f in tab.columns:
            if f"col.{f}" in t:
                tab.columns[f][:n] = t[f"col.{f}"].to(tab.device)
        lv = t["live"].to(tab.device)
        tab.live[: lv.numel()] = lv[: tab.live.numel()]
        tab.row_ids, tab.texts, tab.metas = meta["row_ids"], meta["texts"], meta["metas"]
        tab.dicts = {f: dict(d) for f, d in meta["dicts"].items()}
        tab.deleted = meta.get("deleted", 0)
        tab.key_to_row = {r: i for i, r in enumerate(tab.row_ids)}
        return tab


def _and_bitmap(live: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    n = mask.numel()
    pad = (-n) % 32
    m = torch.cat([mask, torch.zeros(pad, dtype=torch.bool, device=mask.device)]).view(-1, 32).to(torch.int64)
    w = (m << torch.arange(32, device=mask.device, dtype=torch.int64)).sum(1)
    w = torch.where(w >= (1 << 31), w - (1 << 32), w).to(torch.int32)
    out = live.clone()
    out[: w.numel()] &= w
    return out


class VectorStore:
    """The five per-scope tables of the reference schema."""

    def __init__(self, dim: int, device="cpu", table_names: dict | None = None, capacity: int = 1024):
        self.dim = dim
        self.device = torch.device(device)
        self.table_names = dict(DEFAULT_TABLES, **(table_names or {}))
        self.tables = {s: VectorTable(self.table_names[s], dim, device, capacity) for s in SCOPES}
        self.audit: list[dict] = []

    def table(self, scope: str) -> VectorTable:
        return self.tables[scope]

    def counts(self) -> dict:
        return {self.table_names[s]: t.count() for s, t in self.tables.items()}

    def save(self, path: str | Path) -> None:
        path = Path(path)
        path.mkdir(parents=True, exist_ok=True)
        for s, t in self.tables.items():
            t.save(path / s)
        manifest = {"dim": self.dim, "tables": self.table_names, "counts": self.counts(), "audit": self.audit}
        tmp = path / "manifest.json.tmp"
        tmp.write_text(json.dumps(manifest, indent=1))
        tmp.replace(path / "manifest.json")

    @classmethod
    def load(cls, path: str | Path, device="cpu") -> "VectorStore":
        path = Path(path)
        man = json.loads((path / "manifest.json").read_text())
        st = cls(man["dim"], device, man["tables"])
        for s in SCOPES:
            if (path / s / "rows.json").exists():
                st.tables[s] = VectorTable.load(path / s, device)
        st.audit = man.get("audit", [])
        return st
