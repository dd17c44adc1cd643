"""GPU-resident vector store — replaces the reference's Cassandra 5 SAI vector
tables (helm/templates/cassandra-initdb-configmap.yaml:13-102) and the
LangChain ``Cassandra`` store (vector_write_service.py:136-159,
graph_rag_retrievers.py:68-80).

Per scope table (catalog / repo / module / file / chunk), two index kinds
(``INDEX_KIND``):

* ``flat``: every live row scanned by the fused score + filter + top-k kernel
  (exact; the right choice up to a few million rows);
* ``ivf`` (``NLIST`` lists, ``NPROBE`` probes): rows live in *slots*; the
  clustered region [0, nc) is ordered by inverted list, new rows go to an
  append region [nc, n) that every query scans flat, and ``compact()``
  (automatic once the append region outgrows ``compact_frac`` of the
  clustered one) trains/assigns and re-sorts every live slot by list,
  dropping tombstones.  A query = coarse top-nprobe over the centroids, the
  device-built probe plan (``grag_ivf_plan``: no sort/scatter glue, no host
  sync), ONE ``grag_score_topk_work`` launch over the probed lists and one
  flat launch over the append region, both with the metadata predicates and
  the live bitmap inside the scan, and the device merge
  (``grag_topk_merge``).

Device columns per slot: bf16 vectors (L2-normalised, cosine == dot),
dictionary-encoded int32 filter columns (the reference's allow-listed
metadata, vector_write_service.py:28-34, plus scope/namespace/...), 31-bit
bloom columns for multi-valued fields with an exact host re-check, a live
bitmap (updated in place by ``grag_bitmap_update``), and slot -> logical row.

Host rows (``RowStore``) are columnar byte arenas — row_id / text / JSON
metadata + int64 offsets — so tens of millions of rows cost their bytes,
not a Python object each; bulk synthetic corpora are virtual segments
generated on demand (utils/synthetic.py).

Upserts are idempotent on ``row_id`` (the reference re-ingest duplicated
rows): ids are content hashes chosen by the writer.
"""
from __future__ import annotations

import json
import threading
from dataclasses import dataclass
from pathlib import Path

import numpy as np
import torch

from ..ops.topk import (OP_BITAND, OP_EQ, Predicate, bitmap_update, ivf_plan, merge_fits, merge_partials,
                        num_waves, score_topk, score_topk_work)
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


# ---------------------------------------------------------------------------- host rows
class _Arena:
    """Append-only byte strings: one bytearray + int64 end offsets."""

    def __init__(self):
        self.data = bytearray()
        self.ends = np.zeros(1024, dtype=np.int64)
        self.n = 0

    def extend(self, items: list[bytes]) -> None:
        need = self.n + len(items)
        if need > self.ends.shape[0]:
            cap = self.ends.shape[0]
            while cap < need:
                cap *= 2
            e = np.zeros(cap, dtype=np.int64)
            e[: self.n] = self.ends[: self.n]
            self.ends = e
        pos = len(self.data)
        for i, b in enumerate(items):
            self.data += b
            pos += len(b)
            self.ends[self.n + i] = pos
        self.n = need

    def get(self, i: int) -> bytes:
        e = self.ends
        a = int(e[i - 1]) if i > 0 else 0
        return bytes(self.data[a:int(e[i])])

    def save(self, path: Path, stem: str) -> None:
        (path / f"{stem}.bin.tmp").write_bytes(bytes(self.data))
        (path / f"{stem}.bin.tmp").replace(path / f"{stem}.bin")
        np.save(path / f"{stem}.ends.npy", self.ends[: self.n])

    @classmethod
    def load(cls, path: Path, stem: str) -> "_Arena":
        a = cls()
        a.data = bytearray((path / f"{stem}.bin").read_bytes())
        ends = np.load(path / f"{stem}.ends.npy", allow_pickle=False)
        a.n = int(ends.shape[0])
        a.ends = np.zeros(max(1024, a.n), dtype=np.int64)
        a.ends[: a.n] = ends
        return a


class RowStore:
    """Logical rows (append-only; row = insertion index): row_id, text, metadata.
    Materialised rows live in byte arenas; a virtual segment [r0, r1) is served by a
    provider (``row_id(i)``, ``text(i)``, ``meta(i)``, ``index_of(row_id)``, ``spec()``)."""

    def __init__(self):
        self.ids, self.texts, self.metas = _Arena(), _Arena(), _Arena()
        self.key_to_row: dict[str, int] = {}
        self.n = 0
        self.row_arena = np.full(1024, -1, dtype=np.int64)  # row -> arena index (-1: virtual row)
        self.virtual: list[tuple[int, int, object]] = []
        self.overrides: dict[int, tuple[str, dict]] = {}
        self.lock = threading.Lock()

    def append(self, row_ids: list[str], texts: list[str], metas: list[dict]) -> int:
        with self.lock:
            r0 = self.n
            a0 = self.ids.n
            self.ids.extend([r.encode() for r in row_ids])
            self.texts.extend([(t or "").encode() for t in texts])
            self.metas.extend([json.dumps(m or {}, ensure_ascii=False).encode() for m in metas])
            self._arena_grow(r0 + len(row_ids))
            self.row_arena[r0:r0 + len(row_ids)] = np.arange(a0, a0 + len(row_ids))
            for i, rid in enumerate(row_ids):
                self.key_to_row[rid] = r0 + i
            self.n += len(row_ids)
            return r0

    def _arena_grow(self, need: int) -> None:
        if need > self.row_arena.shape[0]:
            cap = self.row_arena.shape[0]
            while cap < need:
                cap *= 2
            ra = np.full(cap, -1, dtype=np.int64)
            ra[: self.row_arena.shape[0]] = self.row_arena
            self.row_arena = ra

    def append_virtual(self, provider, n: int) -> int:
        with self.lock:
            r0 = self.n
            self.virtual.append((r0, r0 + n, provider))
            self.n += n
            self._arena_grow(self.n)
            return r0

    def update(self, row: int, text: str, meta: dict) -> None:
        self.overrides[row] = (text, dict(meta or {}))

    def lookup(self, row_id: str) -> int | None:
        r = self.key_to_row.get(row_id)
        if r is not None:
            return r
        for r0, r1, pv in self.virtual:
            i = pv.index_of(row_id)
            if i is not None and 0 <= i < r1 - r0:
                return r0 + i
        return None

    def _virtual(self, row: int):
        for r0, r1, pv in self.virtual:
            if r0 <= row < r1:
                return pv, row - r0
        return None, -1

    def _arena_of(self, row: int) -> int:
        ra = self.row_arena
        return int(ra[row]) if row < ra.shape[0] else -1

    def row_id(self, row: int) -> str:
        a = self._arena_of(row)
        if a >= 0:
            return self.ids.get(a).decode()
        pv, i = self._virtual(row)
        return pv.row_id(i)

    def get(self, row: int) -> tuple[str, str, dict]:
        rid = self.row_id(row)
        ov = self.overrides.get(row)
        if ov is not None:
            return rid, ov[0], ov[1]
        a = self._arena_of(row)
        if a >= 0:
            return rid, self.texts.get(a).decode(), json.loads(self.metas.get(a))
        pv, i = self._virtual(row)
        return rid, pv.text(i), pv.meta(i)

    def save(self, path: Path) -> None:
        for stem, ar in (("ids", self.ids), ("texts", self.texts), ("metas", self.metas)):
            ar.save(path, stem)
        np.save(path / "row_arena.npy", self.row_arena[: self.n])
        side = {"n": self.n, "virtual": [(r0, r1, pv.spec()) for r0, r1, pv in self.virtual],
                "overrides": {str(r): v for r, v in self.overrides.items()}}
        (path / "rows_meta.json.tmp").write_text(json.dumps(side))
        (path / "rows_meta.json.tmp").replace(path / "rows_meta.json")

    @classmethod
    def load(cls, path: Path) -> "RowStore":
        from ..utils.synthetic import provider_from_spec

        rs = cls()
        rs.ids, rs.texts, rs.metas = (_Arena.load(path, s) for s in ("ids", "texts", "metas"))
        ra = np.load(path / "row_arena.npy", allow_pickle=False)
        side = json.loads((path / "rows_meta.json").read_text())
        rs.n = side["n"]
        rs._arena_grow(max(1, rs.n))
        rs.row_arena[: ra.shape[0]] = ra
        for r in np.nonzero(ra >= 0)[0].tolist():
            rs.key_to_row[rs.ids.get(int(ra[r])).decode()] = r
        rs.virtual = [(r0, r1, provider_from_spec(sp)) for r0, r1, sp in side["virtual"]]
        rs.overrides = {int(r): (v[0], v[1]) for r, v in side["overrides"].items()}
        return rs


# ---------------------------------------------------------------------------- table
class VectorTable:
    def __init__(self, name: str, dim: int, device="cpu", capacity: int = 1024, dtype=torch.bfloat16,
                 index_kind: str = "flat", nlist: int = 1024, nprobe: int = 16, compact_frac: float = 0.1,
                 compact_min: int = 1 << 16):
        if index_kind not in ("flat", "ivf"):
            raise ValueError(f"index_kind must be flat or ivf, not {index_kind!r}")
        self.name = name
        self.dim = dim
        self.device = torch.device(device)
        self.dtype = dtype
        self.index_kind = index_kind
        self.nlist, self.nprobe = int(nlist), int(nprobe)
        self.compact_frac, self.compact_min = compact_frac, compact_min
        self.rows = RowStore()
        self.n = 0        # slots in use
        self.nc = 0       # clustered slots (ivf)
        self._cap = max(16, capacity)
        self.vectors = torch.zeros(self._cap, dim, dtype=dtype, device=self.device)
        self.columns = {f: torch.full((self._cap,), -1, dtype=torch.int32, device=self.device)
                        for f in FILTER_FIELDS + MULTI_FIELDS}
        self.dicts: dict[str, dict[str, int]] = {f: {} for f in FILTER_FIELDS + MULTI_FIELDS}
        self.live = torch.zeros((self._cap + 31) // 32, dtype=torch.int32, device=self.device)
        # ivf: slot -> logical row (device, fed to the kernels) and row -> slot (host)
        self.slot_row = torch.full((self._cap,), -1, dtype=torch.int64, device=self.device) if self.ivf else None
        self.slot_list = torch.full((self._cap,), -1, dtype=torch.int32, device=self.device) if self.ivf else None
        self.row_slot = np.full(1024, -1, dtype=np.int64)
        self.centroids: torch.Tensor | None = None
        self.offsets: torch.Tensor | None = None
        self.deleted = 0
        self.lock = threading.RLock()
        self.stats = {"searches": 0, "compactions": 0}
        # filtered IVF: probe more lists when the filter is selective (nprobe * min(max_boost,
        # selectivity^-1/2)); selectivity from cached per-column code counts
        self.max_probe_boost = 8.0
        self._version = 0
        self._counts: dict = {}
        # write hook (service/cluster.py mirrors ingest writes to the other replicas): fn(op, args)
        self.on_write = None
        # searches launch under the lock and read their results back after releasing it; a writer
        # (which may reallocate or re-sort the device arrays) first waits for every launched search
        self._readers: list = []

    def _track_read(self) -> None:
        """Under the lock, after a search's launches: remember its completion event."""
        if self.device.type != "cuda":
            return
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        if len(self._readers) >= 64:
            self._readers = [e for e in self._readers if not e.query()]
        self._readers.append(ev)

    def _drain_readers(self) -> None:
        """Under the lock, before mutating device arrays: no in-flight search may still read them."""
        readers, self._readers = self._readers, []
        for ev in readers:
            ev.synchronize()

    @property
    def ivf(self) -> bool:
        return self.index_kind == "ivf"

    # back-compat accessors (row-ordered host views)
    @property
    def key_to_row(self) -> dict:
        return self.rows.key_to_row

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
        if self.ivf:
            sr = torch.full((cap,), -1, dtype=torch.int64, device=self.device)
            sr[: self.n] = self.slot_row[: self.n]
            self.slot_row = sr
            sl = torch.full((cap,), -1, dtype=torch.int32, device=self.device)
            sl[: self.n] = self.slot_list[: self.n]
            self.slot_list = sl
        self._cap = cap

    def _row_slot_grow(self, need: int) -> None:
        if need > self.row_slot.shape[0]:
            cap = self.row_slot.shape[0]
            while cap < need:
                cap *= 2
            rs = np.full(cap, -1, dtype=np.int64)
            rs[: self.row_slot.shape[0]] = self.row_slot
            self.row_slot = rs

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

    def _set_live(self, slots, alive: bool) -> None:
        t = torch.as_tensor(np.asarray(slots, dtype=np.int64)).to(self.device)
        bitmap_update(self.live, t, alive)

    def _write_slots(self, slots: np.ndarray, vecs: torch.Tensor, metadatas: list[dict], rows: np.ndarray) -> None:
        sidx = torch.from_numpy(slots).to(self.device)
        self.vectors[sidx] = vecs.to(self.dtype)
        for f in FILTER_FIELDS:
            codes = [self._code(f, m[f]) if (m or {}).get(f) not in (None, "") else -1 for m in metadatas]
            self.columns[f][sidx] = torch.tensor(codes, dtype=torch.int32).to(self.device)
        for f in MULTI_FIELDS:
            codes = [self._multi_bits(f, (m or {}).get(f)) for m in metadatas]
            self.columns[f][sidx] = torch.tensor(codes, dtype=torch.int32).to(self.device)
        if self.ivf:
            self.slot_row[sidx] = torch.from_numpy(rows).to(self.device)
            self.slot_list[sidx] = -1
        self._set_live(slots, True)

    @guarded
    def upsert(self, row_ids: list[str], texts: list[str], vectors: torch.Tensor, metadatas: list[dict]) -> int:
        """Insert or overwrite rows keyed by row_id. vectors [n, d] (any float
        dtype; normalised here).  Returns the number of new rows."""
        n = len(row_ids)
        if n == 0:
            return 0
        vecs = vectors.to(self.device, torch.float32)
        vecs = vecs / vecs.norm(dim=-1, keepdim=True).clamp_min(1e-12)
        metadatas = [dict(m or {}) for m in metadatas]
        with self.lock, side_stream(self.device, wait_caller=vectors.is_cuda):
            self._drain_readers()
            rows = np.empty(n, dtype=np.int64)
            fresh = []
            for i, rid in enumerate(row_ids):
                r = self.rows.lookup(rid)
                if r is None:
                    fresh.append(i)
                    rows[i] = -1
                else:
                    rows[i] = r
                    self.rows.update(r, texts[i], metadatas[i])
            if fresh:
                r0 = self.rows.append([row_ids[i] for i in fresh], [texts[i] for i in fresh],
                                      [metadatas[i] for i in fresh])
                rows[fresh] = np.arange(r0, r0 + len(fresh))
            self._row_slot_grow(self.rows.n)
            old = self.row_slot[rows]
            if self.ivf:
                # overwritten rows: tombstone the old slot; every written row gets a fresh append slot
                dead = old[old >= 0]
                if dead.size:
                    self._set_live(dead, False)
                    self.deleted += int(dead.size)
                slots = np.arange(self.n, self.n + n, dtype=np.int64)
                self._grow(self.n + n)
                self.n += n
            else:  # flat: a row keeps its slot
                slots = np.where(old >= 0, old, 0)
                newmask = old < 0
                k = int(newmask.sum())
                slots[newmask] = np.arange(self.n, self.n + k)
                self._grow(self.n + k)
                self.n += k
            self.row_slot[rows] = slots
            self._write_slots(slots, vecs, metadatas, rows)
            self._version += 1
            if self.device.type == "cuda":  # searches read the table from other (side) streams
                torch.cuda.current_stream(self.device).synchronize()
            if self.ivf and self._needs_compaction():
                self._compact_locked()
        if self.on_write is not None:
            self.on_write("upsert", (list(row_ids), list(texts), vecs.to("cpu", torch.float16), metadatas))
        return len(fresh)

    @guarded
    def delete(self, row_ids: list[str]) -> int:
        with self.lock, side_stream(self.device):
            self._drain_readers()
            rows = [self.rows.lookup(r) for r in row_ids]
            rows = np.asarray([r for r in rows if r is not None], dtype=np.int64)
            if rows.size == 0:
                return 0
            slots = self.row_slot[rows]
            slots = slots[slots >= 0]
            if slots.size:
                self._set_live(slots, False)
                self.row_slot[rows] = -1
                for r in row_ids:
                    self.rows.key_to_row.pop(r, None)
                self.deleted += int(slots.size)
                self._version += 1
            if self.device.type == "cuda":
                torch.cuda.current_stream(self.device).synchronize()
        if self.on_write is not None:
            self.on_write("delete", (list(row_ids),))
        return int(slots.size)

    def count(self) -> int:
        return self.n - self.deleted

    # ------------------------------------------------------------------ bulk / ivf maintenance
    @guarded
    def add_virtual(self, provider, vectors: torch.Tensor, columns: dict[str, torch.Tensor] | None = None) -> int:
        """Bulk-load a synthetic corpus: ``vectors`` [n, d] (device, normalised bf16) and
        pre-encoded int32 ``columns`` (dictionary codes registered by the provider via
        ``provider.register(table)``); host rows are generated on demand.  Returns row0."""
        n = vectors.shape[0]
        with self.lock, side_stream(self.device, wait_caller=vectors.is_cuda):
            self._drain_readers()
            r0 = self.rows.append_virtual(provider, n)
            if columns is None and hasattr(provider, "columns"):
                provider.register(self)
                columns = provider.columns(self.device)
            self._row_slot_grow(self.rows.n)
            s0 = self.n
            self._grow(s0 + n)
            self.vectors[s0:s0 + n] = vectors.to(self.device, self.dtype)
            for f, c in (columns or {}).items():
                self.columns[f][s0:s0 + n] = c.to(self.device, torch.int32)
            if self.ivf:
                self.slot_row[s0:s0 + n] = torch.arange(r0, r0 + n, device=self.device)
                self.slot_list[s0:s0 + n] = -1
            self.row_slot[r0:r0 + n] = np.arange(s0, s0 + n)
            _set_range(self.live, s0, s0 + n)
            self.n += n
            self._version += 1
            if self.device.type == "cuda":
                torch.cuda.current_stream(self.device).synchronize()
            return r0

    def _needs_compaction(self) -> bool:
        app = self.n - self.nc
        return app > max(self.compact_min, self.compact_frac * self.nc)

    @guarded
    def compact(self, train_iters: int = 10, sample: int = 1 << 18, seed: int = 0, group=None) -> None:
        """(ivf) train the quantiser if needed (k-means sums all-reduced over ``group``
        when the table is one shard of a DP index), assign the append
        region, and re-sort every live slot by inverted list (tombstones dropped)."""
        with self.lock, side_stream(self.device):
            self._drain_readers()
            self._compact_locked(train_iters, sample, seed, group)

    def _compact_locked(self, train_iters: int = 10, sample: int = 1 << 18, seed: int = 0, group=None) -> None:
        if not self.ivf or self.n == 0:
            return
        from .ivf import IVFIndex

        dev = self.device
        live = _live_slots(self.live, self.n)
        if live.numel() < 2 * self.nlist:
            return  # too small to cluster: the append region stays a flat scan
        if self.centroids is None:
            g = torch.Generator(device="cpu").manual_seed(seed)
            pick = live[torch.randperm(live.numel(), generator=g)[: min(sample, live.numel())].to(dev)]
            q = IVFIndex(self.dim, self.nlist, dev, self.dtype)
            q.train(self.vectors[pick], iters=train_iters, seed=seed, group=group)
            self.centroids = q.centroids
        lists = self.slot_list[live].clone()
        need = lists < 0
        if bool(need.any()):
            idx = live[need]
            out = []
            for s in range(0, idx.numel(), 1 << 18):
                _, a = score_topk(self.centroids, self.vectors[idx[s:s + (1 << 18)]], 1)
                out.append(a[:, 0].to(torch.int32))
            lists[need] = torch.cat(out)
        order = torch.argsort(lists, stable=True)
        src = live[order]
        m = src.numel()
        self.vectors[:m] = self.vectors[src].clone()
        for f in self.columns:
            self.columns[f][:m] = self.columns[f][src].clone()
        self.slot_row[:m] = self.slot_row[src].clone()
        self.slot_list[:m] = lists[order]
        self.slot_row[m:self.n] = -1
        self.slot_list[m:self.n] = -1
        self.live.zero_()
        _set_range(self.live, 0, m)
        cnt = torch.bincount(lists.long(), minlength=self.nlist)
        self.offsets = torch.zeros(self.nlist + 1, dtype=torch.int64, device=dev)
        self.offsets[1:] = torch.cumsum(cnt, 0)
        rows = self.slot_row[:m].cpu().numpy()
        self.row_slot[:] = -1
        self.row_slot[rows] = np.arange(m)
        self.n = self.nc = m
        self.deleted = 0
        self.stats["compactions"] += 1
        if dev.type == "cuda":
            torch.cuda.current_stream(dev).synchronize()

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

    @staticmethod
    def _host_ok(md: dict, checks) -> bool:
        for k, v in checks:
            if k in MULTI_FIELDS:
                if v not in _split_multi(md.get(k)):
                    return False
            elif str(md.get(k, "")) != v:
                return False
        return True

    # ------------------------------------------------------------------ search
    def selectivity(self, preds) -> float:
        """Estimated fraction of rows passing the fused predicates (independence
        assumption; equality predicates from cached code counts, bloom bits 1/2)."""
        sel = 1.0
        for p in preds or []:
            if p.op != OP_EQ:
                sel *= 0.5
                continue
            key = id(p.column)
            ent = self._counts.get(key)
            if ent is None or ent[0] != self._version:
                c = p.column[: self.n]
                cnt = torch.bincount(c[c >= 0].long()).cpu() if self.n else torch.zeros(1, dtype=torch.long)
                ent = self._counts[key] = (self._version, cnt, max(1, self.n))
            _, cnt, n = ent
            sel *= (float(cnt[p.value]) if 0 <= p.value < cnt.numel() else 0.0) / n
        return max(sel, 1e-9)

    def _scan(self, q: torch.Tensor, kk: int, preds, bitmap, qpred):
        """Device scores/ids (ids = logical rows) of the top-kk per query."""
        nq = q.shape[0]
        row_ids = self.slot_row if self.ivf else None
        if not self.ivf or self.nc == 0 or self.centroids is None:
            return score_topk(self.vectors[: self.n], q, kk, preds=preds, bitmap=bitmap, row_ids=row_ids, qpred=qpred)
        L = num_waves() * kk
        app = self.n > self.nc
        boost = min(self.max_probe_boost, self.selectivity(preds) ** -0.5) if preds else 1.0
        nprobe = min(self.nlist, int(round(self.nprobe * boost)))
        if q.is_cuda:
            nprobe = max(1, min(nprobe, (lib_merge_cap() - (kk if app else 0)) // L))
        _, lists = score_topk(self.centroids, q, nprobe)
        if q.is_cuda and merge_fits(nprobe, L, kk if app else 0, kk):
            step = max(1, min(nq, plan_max_pairs() // nprobe))
            outs = []
            for a in range(0, nq, step):  # the probe plan handles nq * nprobe <= its LDS capacity
                qa, la = q[a:a + step], lists[a:a + step]
                rows, wq, cand = ivf_plan(la, self.offsets, self.nlist)
                ps, pi = score_topk_work(self.vectors, qa, kk, rows, wq, 1, preds=preds, bitmap=bitmap,
                                         row_ids=row_ids, qpred=_qpred_slice(qpred, a, a + step))
                extra = None
                if app:
                    extra = score_topk(self.vectors, qa, kk, preds=preds, bitmap=bitmap, row_ids=row_ids,
                                       row_begin=self.nc, row_end=self.n, qpred=_qpred_slice(qpred, a, a + step))
                outs.append(merge_partials(ps.view(-1, L), pi.view(-1, L), kk, qa.shape[0], cand=cand, cnt=nprobe,
                                           extra=extra))
            if len(outs) == 1:
                return outs[0]
            return torch.cat([o[0] for o in outs]), torch.cat([o[1] for o in outs])
        return self._scan_ref(q, kk, lists, preds, bitmap, qpred)

    def _scan_ref(self, q, kk, lists, preds, bitmap, qpred):
        """Reference / fallback IVF scan (CPU tensors, or shapes past the device plan)."""
        from ..ops.topk import _mask_ref

        nq = q.shape[0]
        offs = self.offsets.cpu().tolist()
        out_s = torch.full((nq, kk), float("-inf"), device=q.device)
        out_i = torch.full((nq, kk), -1, dtype=torch.long, device=q.device)
        for qi in range(nq):
            parts = [torch.arange(offs[l], offs[l + 1]) for l in lists[qi].tolist() if l >= 0]
            parts.append(torch.arange(self.nc, self.n))
            slots = torch.cat(parts).to(self.vectors.device)
            if slots.numel() == 0:
                continue
            ok = _mask_ref(self.n, preds, bitmap, q.device)[slots.to(q.device)]
            if qpred is not None:
                cols, sel, vals = qpred
                c = int(sel[qi])
                if c >= 0:
                    ok &= cols[c][slots] == int(vals[qi])
            slots = slots[ok.to(slots.device)]
            if slots.numel() == 0:
                continue
            sc = self.vectors[slots].float() @ q[qi].float()
            m = min(kk, sc.numel())
            v, j = sc.topk(m)
            out_s[qi, :m] = v
            out_i[qi, :m] = self.slot_row[slots[j]]
        return out_s, out_i

    @guarded
    def search(self, qvecs: torch.Tensor, k: int, flt: dict | None = None, qpred=None) -> list[list[Hit]]:
        """Batched filtered top-k by cosine. qvecs [nq, d].  The table lock covers
        only the snapshot + launches; the device->host copy and hit assembly run
        outside it (concurrent searches and upserts do not serialise on the sync)."""
        nq = qvecs.shape[0]
        with side_stream(self.device, wait_caller=qvecs.is_cuda):
            with self.lock:
                self.stats["searches"] += 1
                if self.n == 0:
                    return [[] for _ in range(nq)]
                pc = self.predicates(flt)
                if pc is None:
                    return [[] for _ in range(nq)]
                preds, checks = pc
                extra = None
                if len(preds) > 4:
                    # AND the overflow predicates into a row bitmap with one torch pass
                    m = torch.ones(self.n, dtype=torch.bool, device=self.device)
                    for p in preds[4:]:
                        c = p.column[: self.n]
                        m &= (c == p.value) if p.op == OP_EQ else ((c & p.value) != 0)
                    extra = m
                    preds = preds[:4]
                bitmap = self.live if extra is None else _and_bitmap(self.live, extra)
                if qpred is not None and qpred[0] and isinstance(qpred[0][0], str):
                    # per-query predicates by column NAME (search_pairs): the column tensors are taken
                    # here, under the lock, so a concurrent upsert's _grow cannot swap them between the
                    # lookup and the scan (a stale, shorter column read up to the new self.n)
                    qpred = ([self.columns[f] for f in qpred[0]], qpred[1], qpred[2])
                q = qvecs.to(self.device, self.dtype)
                kk = min(32, k + (8 if checks else 0))
                scores, ids = self._scan(q, kk, preds, bitmap, qpred)
                self._track_read()
            scores, ids = scores.cpu().tolist(), ids.cpu().tolist()
        out = []
        for qi in range(nq):
            hits = []
            for s, r in zip(scores[qi], ids[qi]):
                if r < 0 or s == float("-inf"):
                    continue
                rid, text, md = self.rows.get(r)
                if checks and not self._host_ok(md, checks):
                    continue
                hits.append(Hit(rid, text, md, float(s), r))
                if len(hits) >= k:
                    break
            out.append(hits)
        return out

    def search_pairs(self, q: torch.Tensor, pairs, k: int, base_filter: dict | None = None) -> list[list[Hit]]:
        """Graph-traversal lookups (retrieval/graph.py): for each ``(field, value)``
        pair, the ``k`` rows most similar to the one query ``q`` [1, d] whose
        ``field`` equals ``value`` (on top of ``base_filter``).  Every indexed pair
        of a call is ONE launch of the fused score+top-k kernel with per-query
        predicates (the query repeated, each copy carrying its own ``column ==
        code`` test); unindexed fields fall back to one filtered search each.
        Pairs whose value this table has never stored return no rows."""
        q = q.reshape(1, -1)
        cols: list[str] = []
        col_idx: dict[str, int] = {}
        sel, vals, slot = [], [], []
        host_pairs = []
        out: list[list[Hit]] = [[] for _ in pairs]
        with self.lock:  # codes are stable once assigned; read them consistently with the columns' state
            for j, (f, v) in enumerate(pairs):
                if f in FILTER_FIELDS:
                    code = self.dicts[f].get(str(v))
                    if code is None:  # value never seen in this table: no row can match
                        continue
                    if f not in col_idx:
                        col_idx[f] = len(cols)
                        cols.append(f)
                    sel.append(col_idx[f])
                    vals.append(code)
                    slot.append(j)
                else:
                    host_pairs.append(j)
        if slot:
            Q = q.expand(len(slot), -1).contiguous()
            dev = self.device
            # columns by name: search() takes the tensors under the table lock (a concurrent upsert may
            # grow and replace them until then)
            qpred = (cols, torch.tensor(sel, dtype=torch.int32, device=dev),
                     torch.tensor(vals, dtype=torch.int32, device=dev))
            for j, hits in zip(slot, self.search(Q, k, base_filter, qpred=qpred)):
                out[j] = hits
        for j in host_pairs:  # unindexed edge field: filtered search per value
            f, v = pairs[j]
            out[j] = self.search(q, k, dict(base_filter or {}, **{f: v}))[0]
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
            if self.ivf:
                tensors["slot_row"] = self.slot_row[: self.n].contiguous().cpu()
                tensors["slot_list"] = self.slot_list[: self.n].contiguous().cpu()
                if self.centroids is not None:
                    tensors["centroids"] = self.centroids.contiguous().cpu()
                    tensors["offsets"] = self.offsets.contiguous().cpu()
            tensors["row_slot"] = torch.from_numpy(self.row_slot[: self.rows.n].copy())
            tmp = path / "table.safetensors.tmp"
            save_file(tensors, str(tmp))
            tmp.replace(path / "table.safetensors")
            self.rows.save(path)
            meta = {"name": self.name, "dim": self.dim, "n": self.n, "nc": self.nc, "deleted": self.deleted,
                    "index_kind": self.index_kind, "nlist": self.nlist, "nprobe": self.nprobe, "dicts": self.dicts}
            tmpj = path / "table.json.tmp"
            tmpj.write_text(json.dumps(meta, ensure_ascii=False))
            tmpj.replace(path / "table.json")

    @classmethod
    def load(cls, path: str | Path, device="cpu", index_kind: str | None = None, nprobe: int | None = None
             ) -> "VectorTable":
        from safetensors.torch import load_file

        path = Path(path)
        meta = json.loads((path / "table.json").read_text())
        t = load_file(str(path / "table.safetensors"))
        kind = meta.get("index_kind", "flat")
        tab = cls(meta["name"], meta["dim"], device=device, capacity=max(16, meta["n"]), index_kind=kind,
                  nlist=meta.get("nlist", 1024), nprobe=nprobe or meta.get("nprobe", 16))
        n = meta["n"]
        tab.n, tab.nc = n, meta.get("nc", 0)
        tab.vectors[:n] = t["vectors"].to(tab.device)
        for f in tab.columns:
            if f"col.{f}" in t:
                tab.columns[f][:n] = t[f"col.{f}"].to(tab.device)
        lv = t["live"].to(tab.device)
        tab.live[: lv.numel()] = lv[: tab.live.numel()]
        if tab.ivf:
            tab.slot_row[:n] = t["slot_row"].to(tab.device)
            tab.slot_list[:n] = t["slot_list"].to(tab.device)
            if "centroids" in t:
                tab.centroids = t["centroids"].to(tab.device)
                tab.offsets = t["offsets"].to(tab.device)
        tab.rows = RowStore.load(path)
        rs = t["row_slot"].numpy()
        tab._row_slot_grow(max(1, rs.shape[0]))
        tab.row_slot[: rs.shape[0]] = rs
        tab.dicts = {f: dict(d) for f, d in meta["dicts"].items()}
        tab.deleted = meta.get("deleted", 0)
        if index_kind is not None and index_kind != kind:
            raise ValueError(f"{path}: table was saved as {kind!r}, requested {index_kind!r}")
        return tab


def lib_merge_cap() -> int:
    from ..ops._lib import lib

    return lib().grag_topk_merge_cap()


def plan_max_pairs() -> int:
    from ..ops._lib import lib

    return lib().grag_ivf_plan_max_pairs()


def _qpred_slice(qpred, a: int, b: int):
    if qpred is None:
        return None
    cols, sel, vals = qpred
    return cols, sel[a:b], vals[a:b]


def _set_range(live: torch.Tensor, a: int, b: int) -> None:
    """Set live bits [a, b) (whole words in one fill, edges by mask)."""
    if b <= a:
        return
    w0, w1 = a >> 5, (b - 1) >> 5

    def word_mask(lo, hi):  # bits lo..hi inclusive within one word, as int32
        m = ((1 << (hi + 1)) - 1) ^ ((1 << lo) - 1)
        return m - (1 << 32) if m >= (1 << 31) else m

    if w0 == w1:
        live[w0] |= word_mask(a & 31, (b - 1) & 31)
        return
    live[w0] |= word_mask(a & 31, 31)
    if w1 > w0 + 1:
        live[w0 + 1:w1] = -1
    live[w1] |= word_mask(0, (b - 1) & 31)


def _live_slots(live: torch.Tensor, n: int) -> torch.Tensor:
    idx = torch.arange(n, device=live.device)
    bits = (live[idx >> 5].long() >> (idx & 31)) & 1
    return idx[bits.bool()]


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

    def __init__(self, dim: int, device="cpu", table_names: dict | None = None, capacity: int = 1024,
                 index_kind: str = "flat", nlist: int = 1024, nprobe: int = 16):
        self.dim = dim
        self.device = torch.device(device)
        self.table_names = dict(DEFAULT_TABLES, **(table_names or {}))
        self.index_kind = index_kind
        self.tables = {s: VectorTable(self.table_names[s], dim, device, capacity, index_kind=index_kind,
                                      nlist=nlist, nprobe=nprobe) for s in SCOPES}
        self.audit: list[dict] = []

    def table(self, scope: str) -> VectorTable:
        return self.tables[scope]

    # ------------------------------------------------------------------ replica mirroring
    def add_listener(self, fn) -> None:
        """fn(scope, (op, args)) after every upsert/delete made through this store (not for writes
        applied with ``apply_remote``), so a front door can mirror one replica's ingest on the others."""
        self._remote = threading.local()

        def hook(scope):
            def on_write(op, args):
                if not getattr(self._remote, "active", False):
                    fn(scope, (op, args))
            return on_write

        for scope, t in self.tables.items():
            t.on_write = hook(scope)

    def apply_remote(self, scope: str, payload) -> None:
        """Apply a write mirrored from another replica (not re-broadcast)."""
        op, args = payload
        remote = getattr(self, "_remote", None)
        if remote is not None:
            remote.active = True
        try:
            t = self.tables[scope]
            if op == "upsert":
                t.upsert(*args)
            elif op == "delete":
                t.delete(*args)
        finally:
            if remote is not None:
                remote.active = False

    def counts(self) -> dict:
        return {self.table_names[s]: t.count() for s, t in self.tables.items()}

    def save(self, path: str | Path) -> None:
        path = Path(path)
        path.mkdir(parents=True, exist_ok=True)
        for s, t in self.tables.items():
            t.save(path / s)
        manifest = {"dim": self.dim, "tables": self.table_names, "counts": self.counts(), "audit": self.audit,
                    "index_kind": self.index_kind}
        tmp = path / "manifest.json.tmp"
        tmp.write_text(json.dumps(manifest, indent=1))
        tmp.replace(path / "manifest.json")

    @classmethod
    def load(cls, path: str | Path, device="cpu", nprobe: int | None = None) -> "VectorStore":
        path = Path(path)
        man = json.loads((path / "manifest.json").read_text())
        st = cls(man["dim"], device, man["tables"], index_kind=man.get("index_kind", "flat"))
        for s in SCOPES:
            if (path / s / "table.json").exists():
                st.tables[s] = VectorTable.load(path / s, device, nprobe=nprobe)
        st.audit = man.get("audit", [])
        return st
