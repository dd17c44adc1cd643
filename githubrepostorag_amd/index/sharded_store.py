"""Row-sharded five-table store for N serving replicas (SURVEY §2.9 "index
sharding (DP)", collectives C3/C4 of §2.8).

The reference answers every worker from ONE Cassandra ANN store
(rag_worker/src/worker/services/graph_rag_retrievers.py:68-134,
helm/templates/cassandra-initdb-configmap.yaml:26-29).  With N per-GPU
replicas behind one front door (service/cluster.py), a full copy per GPU
wastes HBM that the model and KV cache need (100M x 1024-d bf16 = 205 GB), so
each replica keeps 1/N of every scope table and every read fans out:

  search(Q, k, filter)      C4: the query vectors go to every other shard;
                            each shard runs its fused filtered score+top-k
                            locally; C3: the per-shard top-k lists come back
                            and are merged by score into the global top-k.
  search_pairs(q, pairs, k) one graph-traversal depth (retrieval/graph.py):
                            every (field, value) lookup on every shard in one
                            round, merged per pair -> traversal over the union.
  upsert / delete           routed to the owning shard (crc32(row_id) mod N),
                            so ingest on any replica writes each row once.

The local shard's search runs while the remote ones are in flight.  The
transport is pluggable: ``service/mesh.py`` (the serving default) runs every
round replica-to-replica over direct authenticated sockets with coalesced
requests and acknowledged writes; ``service/cluster.py`` HubShardTransport
relays rounds through the front door's hub (``GRAG_SHARD_TRANSPORT=hub``);
``LocalShardTransport`` wires N stores in one process (tests, rehearsals).
Merged results equal a flat store's up to score ties
(tests/test_sharded_store.py).

A round that did not hear from every shard is DEGRADED (its answer lacks the
missing shards' rows): it is counted in the table's stats, the
``rag_index_degraded_rounds_total`` metric and the calling thread's
``round_health()`` record, which the worker reports in the job's
``retrieval`` event (``degraded``, ``missing_shards``)."""
from __future__ import annotations

import concurrent.futures as cf
import contextlib
import logging
import threading
import zlib

import numpy as np
import torch

from .store import SCOPES, Hit, VectorStore, VectorTable

log = logging.getLogger(__name__)


def shard_of(row_id: str, n: int) -> int:
    """Owning shard of a row: stable across processes and restarts."""
    return zlib.crc32(row_id.encode("utf-8")) % n if n > 1 else 0


# ---------------------------------------------------------------------- local execution
def _vec(q) -> torch.Tensor:
    return torch.from_numpy(np.asarray(q, dtype=np.float32))


def execute(store: VectorStore, scope: str, op: str, payload):
    """Run one fanned-out operation on THIS replica's shard (the receiving end of a round)."""
    t = store.tables[scope]
    if op == "search":
        Q, k, flt = payload
        return t.search(_vec(Q).to(t.device), k, flt)
    if op == "pairs":
        q, pairs, k, base = payload
        return t.search_pairs(_vec(q).to(t.device), pairs, k, base)
    if op == "count":
        return t.count()
    if op == "upsert":
        ids, texts, vecs, metas = payload
        return t.upsert(ids, texts, _vec(vecs), metas)
    if op == "delete":
        return t.delete(payload)
    raise ValueError(f"unknown shard op {op!r}")


def merge_hits(parts: list[list[list[Hit]]], k: int) -> list[list[Hit]]:
    """[shard][query][hits] -> [query][top-k hits by score] (C3 merge)."""
    parts = [p for p in parts if p is not None]
    if not parts:
        return []
    out = []
    for qi in range(len(parts[0])):
        best: dict[str, Hit] = {}  # a row is on one shard; a stale copy (re-sharding) must not repeat it
        for p in parts:
            if qi < len(p):
                for h in p[qi]:
                    if h.row_id not in best or h.score > best[h.row_id].score:
                        best[h.row_id] = h
        allh = sorted(best.values(), key=lambda h: (-h.score, h.row_id))
        out.append(allh[:k])
    return out


# ---------------------------------------------------------------------- round health
_TLS = threading.local()


@contextlib.contextmanager
def round_health():
    """Collect the shard rounds the CALLING thread runs inside the block:
    ``{"rounds", "degraded_rounds", "missing_shards"}`` (a job's agent runs on one thread)."""
    rec = {"rounds": 0, "degraded_rounds": 0, "missing_shards": set()}
    prev = getattr(_TLS, "rec", None)
    _TLS.rec = rec
    try:
        yield rec
    finally:
        _TLS.rec = prev


def _note_round(missing) -> None:
    rec = getattr(_TLS, "rec", None)
    if rec is not None:
        rec["rounds"] += 1
        if missing:
            rec["degraded_rounds"] += 1
            rec["missing_shards"].update(missing)


# ---------------------------------------------------------------------- transports
class LocalShardTransport:
    """N shards in one process: a round calls ``execute`` on every other shard's
    store directly (tests; the hub transport behaves the same over sockets)."""

    def __init__(self):
        self.stores: dict[int, VectorStore] = {}

    def register(self, rank: int, store: VectorStore) -> None:
        self.stores[rank] = store

    def fanout(self, origin: int, scope: str, op: str, payload, timeout: float = 60.0) -> list:
        return [execute(st, scope, op, payload) for r, st in sorted(self.stores.items()) if r != origin]

    def write(self, origin: int, owner: int, scope: str, op: str, payload):
        return execute(self.stores[owner], scope, op, payload)


# ---------------------------------------------------------------------- facade
class ShardedTable:
    """One scope table as seen by the agent, retrievers and ingest writer of a
    replica: VectorTable's read/write API over the union of all shards."""

    def __init__(self, local: VectorTable, scope: str, rank: int, nshards: int, transport, owner=shard_of,
                 timeout: float = 60.0):
        self.local, self.scope, self.rank, self.nshards = local, scope, rank, nshards
        self.transport, self.owner, self.timeout = transport, owner, timeout
        self.stats = {"rounds": 0, "remote_parts": 0, "degraded_rounds": 0}
        self._pool = cf.ThreadPoolExecutor(32, thread_name_prefix=f"shard-{scope}")  # rounds wait on replies

    # attributes the retrievers / health read straight from the local shard
    def __getattr__(self, name):
        return getattr(self.local, name)

    def _round(self, op: str, payload, local_fn):
        """Fan ``op`` out to the other shards while this shard runs ``local_fn``."""
        fut = self._pool.submit(self.transport.fanout, self.rank, self.scope, op, payload, self.timeout)
        mine = local_fn()
        try:
            remote = fut.result(self.timeout + 5.0)
            missing = list(getattr(remote, "missing", ()))
        except Exception:
            log.exception("sharded %s round on %s failed; answering from the local shard", op, self.scope)
            remote, missing = [], [r for r in range(self.nshards) if r != self.rank]
        self.stats["rounds"] += 1
        self.stats["remote_parts"] += len(remote)
        if missing:
            # recall dropped by len(missing)/N for this answer: visible, never silent
            self.stats["degraded_rounds"] += 1
            from ..service import metrics as M

            M.INDEX_DEGRADED_ROUNDS.labels(table=self.scope).inc()
            log.warning("sharded %s round on %s: no answer from shard(s) %s (degraded)", op, self.scope, missing)
        _note_round(missing)
        return mine, remote

    def search(self, qvecs: torch.Tensor, k: int, flt: dict | None = None, qpred=None) -> list[list[Hit]]:
        if qpred is not None:
            raise ValueError("per-query predicates are shard-local codes: use search_pairs on a sharded table")
        if self.nshards <= 1:
            return self.local.search(qvecs, k, flt)
        payload = (qvecs.detach().float().cpu().numpy(), k, flt)
        mine, remote = self._round("search", payload, lambda: self.local.search(qvecs, k, flt))
        return merge_hits([mine, *remote], k)

    def search_pairs(self, q: torch.Tensor, pairs, k: int, base_filter: dict | None = None) -> list[list[Hit]]:
        if self.nshards <= 1:
            return self.local.search_pairs(q, pairs, k, base_filter)
        pairs = [(f, str(v)) for f, v in pairs]
        payload = (q.detach().float().reshape(1, -1).cpu().numpy(), pairs, k, base_filter)
        mine, remote = self._round("pairs", payload, lambda: self.local.search_pairs(q, pairs, k, base_filter))
        return merge_hits([mine, *remote], k)

    def count(self) -> int:
        if self.nshards <= 1:
            return self.local.count()
        mine, remote = self._round("count", None, self.local.count)
        return mine + sum(int(r) for r in remote if r is not None)

    def upsert(self, row_ids, texts, vectors: torch.Tensor, metadatas) -> int:
        owners = [self.owner(r, self.nshards) for r in row_ids]
        new = 0
        for o in sorted(set(owners)):
            idx = [i for i, x in enumerate(owners) if x == o]
            ids = [row_ids[i] for i in idx]
            tx = [texts[i] for i in idx]
            md = [metadatas[i] for i in idx]
            sel = torch.as_tensor(idx, device=vectors.device)
            if o == self.rank:
                new += self.local.upsert(ids, tx, vectors.index_select(0, sel), md)
            else:
                v = vectors.index_select(0, sel).detach().float().cpu().numpy()
                # acknowledged transports (mesh, local) return the owner's count or raise
                r = self.transport.write(self.rank, o, self.scope, "upsert", (ids, tx, v, md))
                new += int(r) if isinstance(r, int) else 0
        return new

    def delete(self, row_ids) -> int:
        owners = [self.owner(r, self.nshards) for r in row_ids]
        n = 0
        for o in sorted(set(owners)):
            ids = [r for r, x in zip(row_ids, owners) if x == o]
            if o == self.rank:
                n += self.local.delete(ids)
            else:
                r = self.transport.write(self.rank, o, self.scope, "delete", ids)
                n += int(r) if isinstance(r, int) else 0
        return n

    def close(self) -> None:
        self._pool.shutdown(wait=False)


class ShardedStore:
    """``VectorStore`` facade of a replica holding shard ``rank`` of ``nshards``."""

    def __init__(self, local: VectorStore, rank: int, nshards: int, transport, owner=shard_of):
        self.local, self.rank, self.nshards, self.transport = local, rank, nshards, transport
        self.dim, self.device, self.table_names = local.dim, local.device, local.table_names
        self.index_kind = local.index_kind
        self.tables = {s: ShardedTable(t, s, rank, nshards, transport, owner) for s, t in local.tables.items()}
        self.audit = local.audit

    def table(self, scope: str) -> ShardedTable:
        return self.tables[scope]

    def counts(self) -> dict:
        """This shard's rows per table (health stays local: no fan-out on a probe)."""
        return {f"{self.table_names[s]}@shard{self.rank}/{self.nshards}": t.local.count()
                for s, t in self.tables.items()}

    def save(self, path) -> None:
        from pathlib import Path

        self.local.save(Path(path) / shard_dir(self.rank, self.nshards))

    def close(self) -> None:
        for t in self.tables.values():
            t.close()


def shard_dir(rank: int, n: int) -> str:
    return f"shard-{rank}-of-{n}"


def retain_shard(store: VectorStore, rank: int, n: int, owner=shard_of) -> int:
    """Drop the rows another shard owns (a replica that loaded a full snapshot).
    Returns the rows dropped."""
    dropped = 0
    for s in SCOPES:
        t = store.tables[s]
        foreign = [rid for rid in list(t.rows.key_to_row) if owner(rid, n) != rank]
        if foreign:
            dropped += t.delete(foreign)
            if t.ivf:
                t.compact()
    return dropped


def load_shard(index_dir, rank: int, n: int, device, nprobe: int | None = None) -> VectorStore | None:
    """This replica's shard of INDEX_DIR: its own ``shard-r-of-N`` snapshot when one
    exists, else the full snapshot with the foreign rows dropped; None if neither."""
    from pathlib import Path

    d = Path(index_dir)
    own = d / shard_dir(rank, n)
    if (own / "manifest.json").exists():
        return VectorStore.load(own, device, nprobe=nprobe)
    if (d / "manifest.json").exists():
        st = VectorStore.load(d, device, nprobe=nprobe)
        retain_shard(st, rank, n)
        return st
    return None


# ---------------------------------------------------------------------- data-parallel ingest (C5)
def export_rows(table: VectorTable):
    """Every live real row of a table: (row ids, texts, vectors fp32 [n, d] on the host, metadata)."""
    with table.lock:
        items = [(rid, r) for rid, r in table.rows.key_to_row.items() if 0 <= r < table.row_slot.shape[0]
                 and table.row_slot[r] >= 0]
        if not items:
            return [], [], torch.zeros(0, table.dim), []
        slots = torch.as_tensor(np.asarray([table.row_slot[r] for _, r in items], dtype=np.int64))
        vecs = table.vectors[slots.to(table.device)].float().cpu()
        ids, texts, metas = [], [], []
        for rid, r in items:
            _, text, md = table.rows.get(r)
            ids.append(rid)
            texts.append(text)
            metas.append(md)
    return ids, texts, vecs, metas


def split_store(store: VectorStore, n: int, owner=shard_of) -> list[VectorStore]:
    """Partition a store's rows by owning shard into ``n`` host stores (same tables / index kind)."""
    parts = [VectorStore(store.dim, "cpu", store.table_names, index_kind=store.index_kind) for _ in range(n)]
    for scope, t in store.tables.items():
        ids, texts, vecs, metas = export_rows(t)
        by = {}
        for i, rid in enumerate(ids):
            by.setdefault(owner(rid, n), []).append(i)
        for s, idx in by.items():
            parts[s].table(scope).upsert([ids[i] for i in idx], [texts[i] for i in idx], vecs[idx],
                                          [metas[i] for i in idx])
    for p in parts:
        p.audit = list(store.audit)
    return parts


def merge_into(dst: VectorStore, src: VectorStore) -> int:
    """Upsert every row of ``src`` into ``dst`` (idempotent: content-hash row ids); returns rows merged."""
    n = 0
    for scope, t in src.tables.items():
        ids, texts, vecs, metas = export_rows(t)
        if ids:
            dst.table(scope).upsert(ids, texts, vecs.to(dst.device), metas)
            n += len(ids)
    dst.audit.extend(a for a in src.audit if a not in dst.audit)
    return n
