"""Direct replica-to-replica shard rounds.

The reference answers every worker from ONE Cassandra ANN store
(rag_worker/src/worker/services/graph_rag_retrievers.py:68-80); here each
serving replica holds 1/N of every scope table (index/sharded_store.py) and a
retrieval hop fans out to the other N-1 shards.  Round 3 relayed every hop
through the front door's Python hub (replica -> hub -> N-1 replicas -> hub ->
origin).  This module takes the hub off the data path:

  * every replica runs a ``PeerMesh``: an authenticated listener (the cluster's
    hub authkey) whose address it announces in its ``hello``; the hub only
    distributes the peer table (``("peers", {rank: address})``) when membership
    changes, it never sees a shard round;
  * a round is one request per peer over a direct connection, answered on the
    same connection: 2 socket hops instead of 4, and no serialisation through
    one process;
  * requests COALESCE: each peer connection has one sender thread that drains
    everything queued while its previous send was on the wire into one message
    (concurrent jobs' hops share a pickle + syscall), and the receiving shard
    stacks the coalesced plain searches that share (table, k, filter) into ONE
    fused score+top-k launch;
  * writes are acknowledged: an owner applies routed upserts / deletes in
    arrival order on one writer thread and answers with the applied count; a
    write that cannot reach its owner raises ``ShardWriteError`` (the ingest
    batch fails loudly instead of losing the row);
  * a round that could not hear from some shard (peer unknown, connection lost,
    timeout) returns ``Parts`` carrying ``missing`` ranks, which the sharded
    table turns into ``degraded`` retrieval (index/sharded_store.py
    ``round_health``, surfaced in the job's ``retrieval`` event and the
    ``rag_index_degraded_rounds_total`` metric).

Wire (pickled tuples over multiprocessing.connection, our own processes only):
  client -> server  ("batch", [(req_id, scope, op, payload), ...])
  server -> client  ("res",   [(req_id, ok, result_or_error), ...])
"""
from __future__ import annotations

import collections
import itertools
import logging
import queue
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from multiprocessing.connection import AuthenticationError, Client, Listener, answer_challenge, deliver_challenge

log = logging.getLogger(__name__)

WRITE_OPS = ("upsert", "delete")


class ShardWriteError(RuntimeError):
    """A routed write did not reach (or was not applied by) its owning shard."""


def run_one(store, req_id, scope, op, payload):
    """One shard operation on ``store`` -> (req_id, ok, result or error text)."""
    from ..index.sharded_store import execute

    try:
        return (req_id, True, execute(store, scope, op, payload))
    except Exception as e:  # answer anyway: the origin must not wait for a failed shard
        log.exception("shard %s on %s failed", op, scope)
        return (req_id, False, f"{type(e).__name__}: {e}")


def run_reads(store, reads, stats: dict | None = None):
    """Coalesced reads of one message / round: plain searches sharing (table, k, filter) run as ONE
    stacked search (one fused score+top-k launch for all their queries); the rest one by one."""
    import numpy as np

    out, groups = [], {}
    for item in reads:
        req_id, scope, op, payload = item
        if op == "search":
            Q, k, flt = payload
            key = (scope, int(k), repr(sorted((flt or {}).items())))
            groups.setdefault(key, []).append(item)
        else:
            out.append(run_one(store, *item))
    for (scope, k, _), items in groups.items():
        if len(items) == 1:
            out.append(run_one(store, *items[0]))
            continue
        flt = items[0][3][2]
        qs = [np.asarray(it[3][0], dtype=np.float32).reshape(-1, np.asarray(it[3][0]).shape[-1]) for it in items]
        res = run_one(store, -1, scope, "search", (np.concatenate(qs), k, flt))
        if not res[1]:
            out.extend((it[0], False, res[2]) for it in items)
            continue
        if stats is not None:
            stats["stacked_searches"] = stats.get("stacked_searches", 0) + 1
        hits, a = res[2], 0
        for it, q in zip(items, qs):
            out.append((it[0], True, hits[a:a + q.shape[0]]))
            a += q.shape[0]
    return out


class Parts(list):
    """Results of the shards that answered a round; ``missing`` = ranks that did not."""

    def __init__(self, items=(), missing=()):
        super().__init__(items)
        self.missing = list(missing)


def cut_connection(conn) -> None:
    """Shut a multiprocessing Connection's socket down (wakes a thread blocked reading it), then close it."""
    import socket

    try:
        s = socket.fromfd(conn.fileno(), socket.AF_INET, socket.SOCK_STREAM)
        try:
            s.shutdown(socket.SHUT_RDWR)
        finally:
            s.close()
    except (OSError, ValueError):
        pass
    try:
        conn.close()
    except OSError:
        pass


class _Pending:
    __slots__ = ("ev", "ok", "res")

    def __init__(self):
        self.ev = threading.Event()
        self.ok = False
        self.res = None


class _PeerLink:
    """Client side of one peer: a connection, a coalescing sender and a reply reader."""

    def __init__(self, rank: int, address, authkey: bytes, max_batch: int = 256):
        self.rank = rank
        self.address = tuple(address)
        self.conn = Client(self.address, authkey=authkey)
        self.outbox: queue.SimpleQueue = queue.SimpleQueue()
        self.pending: dict[int, _Pending] = {}
        self.lock = threading.Lock()
        self.alive = True
        self.max_batch = max_batch
        self.sent_msgs = 0
        self.sent_reqs = 0
        threading.Thread(target=self._sender, name=f"mesh-send-{rank}", daemon=True).start()
        threading.Thread(target=self._reader, name=f"mesh-recv-{rank}", daemon=True).start()

    def submit(self, req_id: int, scope: str, op: str, payload) -> _Pending:
        p = _Pending()
        with self.lock:
            if not self.alive:
                p.ev.set()
                return p
            self.pending[req_id] = p
        self.outbox.put((req_id, scope, op, payload))
        return p

    def _sender(self) -> None:
        while self.alive:
            item = self.outbox.get()
            if item is None:
                return
            batch = [item]
            while len(batch) < self.max_batch:  # everything queued meanwhile rides in this message
                try:
                    nxt = self.outbox.get_nowait()
                except queue.Empty:
                    break
                if nxt is None:
                    self.alive = False
                    break
                batch.append(nxt)
            try:
                self.conn.send(("batch", batch))
                self.sent_msgs += 1
                self.sent_reqs += len(batch)
            except (OSError, EOFError, BrokenPipeError, ValueError):
                self._fail()
                return

    def _reader(self) -> None:
        try:
            while True:
                kind, items = self.conn.recv()
                if kind != "res":
                    continue
                for req_id, ok, res in items:
                    with self.lock:
                        p = self.pending.pop(req_id, None)
                    if p is not None:
                        p.ok, p.res = ok, res
                        p.ev.set()
        except (EOFError, OSError, ValueError, TypeError):  # TypeError: the link was closed under recv()
            self._fail()

    def _fail(self) -> None:
        with self.lock:
            self.alive = False
            owed = list(self.pending.values())
            self.pending.clear()
        for p in owed:  # answered "missing", never a hang
            p.ev.set()

    def close(self) -> None:
        self.alive = False
        self.outbox.put(None)
        try:
            self.conn.close()
        except OSError:
            pass
        self._fail()


class PeerMesh:
    """This replica's end of the shard mesh: serves its shard to the peers and
    runs its own rounds against theirs (the ``transport`` of index/sharded_store.py)."""

    def __init__(self, rank: int, nshards: int, authkey: bytes, store=None, host: str = "127.0.0.1",
                 read_workers: int = 4):
        self.rank, self.nshards, self.authkey = rank, nshards, authkey
        self.store = store  # this replica's LOCAL shard (VectorStore); set before serving
        # the authentication handshake runs on the accepted connection's own thread (_serve), never on the
        # accept thread: a slow peer cannot hold up the others, and a deep backlog absorbs connect bursts
        self.listener = Listener((host, 0), backlog=128)
        self.address = self.listener.address
        self._peers: dict[int, tuple] = {}
        self._links: dict[int, _PeerLink] = {}
        self._lock = threading.Lock()
        self._ids = itertools.count(1)
        self._connecting: dict[int, threading.Lock] = collections.defaultdict(threading.Lock)
        self._reads = ThreadPoolExecutor(read_workers, thread_name_prefix="mesh-read")
        self._writes = ThreadPoolExecutor(1, thread_name_prefix="mesh-write")  # routed writes applied in order
        self._closed = False
        self._served: set = set()  # accepted connections (closed with the mesh: peers see EOF, not a hang)
        self.stats = {"rounds": 0, "degraded_rounds": 0, "served_msgs": 0, "served_reqs": 0, "stacked_searches": 0}
        self._lat = collections.deque(maxlen=8192)  # seconds per round (fan-out -> last part)
        self._t_first = None
        threading.Thread(target=self._accept_loop, name="mesh-accept", daemon=True).start()

    # ------------------------------------------------------------------ membership
    def set_peers(self, peers: dict) -> None:
        """The hub's peer table {rank: address}; links to departed / moved peers are dropped."""
        peers = {int(r): tuple(a) for r, a in (peers or {}).items() if a is not None and int(r) != self.rank}
        with self._lock:
            self._peers = peers
            stale = [r for r, ln in self._links.items() if peers.get(r) != ln.address or not ln.alive]
            dropped = [self._links.pop(r) for r in stale]
        for ln in dropped:
            ln.close()

    def _link(self, rank: int) -> _PeerLink | None:
        with self._lock:
            ln = self._links.get(rank)
            if ln is not None and ln.alive:
                return ln
            addr = self._peers.get(rank)
        if addr is None:
            return None
        with self._lock:
            gate = self._connecting[rank]
        with gate:  # one connect per peer at a time; concurrent rounds wait for it and share the link
            with self._lock:
                cur = self._links.get(rank)
                if cur is not None and cur.alive:
                    return cur
            try:
                ln = _PeerLink(rank, addr, self.authkey)
            except (OSError, EOFError, AuthenticationError) as e:
                log.warning("mesh: cannot reach shard %d at %s (%s)", rank, addr, e)
                return None
            with self._lock:
                self._links[rank] = ln
        return ln

    # ------------------------------------------------------------------ client: rounds
    def fanout(self, origin: int, scope: str, op: str, payload, timeout: float = 60.0) -> Parts:
        """Run ``op`` on every other shard; the shards that did not answer are ``missing``."""
        waits, missing = [], []
        for r in range(self.nshards):
            if r == self.rank:
                continue
            ln = self._link(r)
            if ln is None:
                missing.append(r)
                continue
            waits.append((r, ln.submit(next(self._ids), scope, op, payload)))
        t_round = time.monotonic()
        deadline = t_round + timeout
        parts = []
        for r, p in waits:
            if p.ev.wait(max(0.0, deadline - time.monotonic())) and p.ok:
                parts.append(p.res)
            else:
                if p.ev.is_set() and not p.ok and p.res is not None:
                    log.warning("mesh: shard %d failed %s on %s: %s", r, op, scope, p.res)
                missing.append(r)
        self.stats["rounds"] += 1
        now = time.monotonic()
        self._lat.append(now - t_round)
        if self._t_first is None:
            self._t_first = t_round
        if missing:
            self.stats["degraded_rounds"] += 1
        return Parts(parts, missing)

    def round_stats(self) -> dict:
        """Rounds this replica originated: count, degraded count, latency p50 / p99 (ms) over the last 8192,
        rounds/s since the first; plus what it served for its peers (messages, requests, stacked launches)."""
        lat = sorted(self._lat)
        out = dict(self.stats)
        if lat:
            out["p50_ms"] = round(1000 * lat[len(lat) // 2], 3)
            out["p99_ms"] = round(1000 * lat[min(len(lat) - 1, int(0.99 * len(lat)))], 3)
            span = time.monotonic() - self._t_first
            out["rounds_per_s"] = round(self.stats["rounds"] / span, 2) if span > 0 else None
        return out

    def write(self, origin: int, owner: int, scope: str, op: str, payload, timeout: float = 120.0):
        """A routed upsert / delete, acknowledged by the owner (returns its applied count)."""
        ln = self._link(owner)
        if ln is None:
            raise ShardWriteError(f"shard {owner} is not connected: {op} on {scope} not applied")
        p = ln.submit(next(self._ids), scope, op, payload)
        if not p.ev.wait(timeout):
            raise ShardWriteError(f"shard {owner} did not acknowledge {op} on {scope} within {timeout:.0f}s")
        if not p.ok:
            raise ShardWriteError(f"shard {owner} failed {op} on {scope}: {p.res}")
        return p.res

    # ------------------------------------------------------------------ server: this shard
    def _accept_loop(self) -> None:
        while not self._closed:
            try:
                conn = self.listener.accept()
            except (OSError, EOFError):
                if self._closed:
                    return
                continue
            except Exception:  # a stray connection that failed authentication
                log.warning("mesh: rejected a connection", exc_info=True)
                continue
            threading.Thread(target=self._serve, args=(conn,), name="mesh-serve", daemon=True).start()

    def _serve(self, conn) -> None:
        guard = threading.Timer(10.0, cut_connection, (conn,))  # a peer that never finishes the handshake
        guard.start()
        try:
            deliver_challenge(conn, self.authkey)
            answer_challenge(conn, self.authkey)
        except (AuthenticationError, EOFError, OSError, AssertionError, TypeError):
            log.warning("mesh: rejected a connection (authentication)")
            conn.close()
            return
        finally:
            guard.cancel()
        send_lock = threading.Lock()
        with self._lock:
            self._served.add(conn)

        def reply(items):
            try:
                with send_lock:
                    conn.send(("res", items))
            except (OSError, EOFError, BrokenPipeError, ValueError):
                pass

        try:
            while True:
                kind, batch = conn.recv()
                if kind != "batch":
                    continue
                self.stats["served_msgs"] += 1
                self.stats["served_reqs"] += len(batch)
                reads = [b for b in batch if b[2] not in WRITE_OPS]
                for b in batch:
                    if b[2] in WRITE_OPS:
                        self._writes.submit(lambda b=b: reply([self._run_one(*b)]))
                if reads:
                    self._reads.submit(lambda reads=reads: reply(self._run_reads(reads)))
        except (EOFError, OSError, ValueError, RuntimeError, TypeError):
            # RuntimeError: executors shut down; TypeError: the connection was closed under recv() (close())
            pass
        finally:
            with self._lock:
                self._served.discard(conn)
            try:
                conn.close()
            except OSError:
                pass

    def _run_one(self, req_id, scope, op, payload):
        return run_one(self.store, req_id, scope, op, payload)

    def _run_reads(self, reads):
        return run_reads(self.store, reads, self.stats)

    def close(self) -> None:
        self._closed = True
        try:
            self.listener.close()
        except OSError:
            pass
        with self._lock:
            links = list(self._links.values())
            self._links.clear()
            served = list(self._served)
        for ln in links:
            ln.close()
        for c in served:
            try:
                c.close()
            except OSError:
                pass
        self._reads.shutdown(wait=False)
        self._writes.shutdown(wait=False)
