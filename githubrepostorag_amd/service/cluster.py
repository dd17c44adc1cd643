"""One front door for N per-GPU replicas (SURVEY §2.9 "DP replicas").

The reference decouples its API from N ARQ workers through Redis: the API
enqueues ``run_rag_job`` (rest_api/src/app/controllers/jobs_controller.py:15-20),
any worker pod picks it up (rag_worker/src/worker/worker.py:182-187) and
progress flows back over pub/sub (rag_shared/bus.py:8-40).  Here:

  front door (no GPU):  FastAPI (service/api.py) + JobQueue + EventLog +
                        CancelFlags + ReplicaHub (this module)
  replica r (GPU r):    a child process (``python -m githubrepostorag_amd
                        replica``) holding one RAGRuntime (engine, encoder,
                        store) and a RAGWorker, connected to the hub over a
                        local authenticated socket (multiprocessing.connection)

Scheduling: the hub's job function ``run_rag_job`` waits for a live replica
with a free slot (each replica advertises WORKER_MAX_JOBS), sends the job to
the least-loaded one and returns when that replica reports the job's ``final``
event.  Every event a replica's worker emits is forwarded and appended to the
front door's replayable EventLog, so ``GET /rag/jobs/{id}/events`` is one SSE
endpoint for the whole node; cancels are forwarded to the owning replica; a
replica that disconnects fails its in-flight jobs (``error`` + ``final``) and
the hub stops dispatching to it.

The index (INDEX_SHARDING, default ``shard``): each replica holds 1/N of every
scope table (index/sharded_store.py, rows owned by crc32(row_id) mod N).  A
replica's search / traversal round goes straight to every other replica over
the peer mesh (service/mesh.py; C4), their per-shard top-k lists come back on
the same connections (C3) and are merged there with its own shard's; an
ingest write goes to the owning replica only and is acknowledged.  The hub
only distributes the peer table (``("peers", {rank: address})``) when
membership changes.  ``GRAG_SHARD_TRANSPORT=hub`` keeps the round-3 relay
through the hub.  A replica lost mid-round is reported as a missing shard
(``degraded`` retrieval; nothing hangs).
``INDEX_SHARDING=mirror`` keeps the round-2 mode: full copies, every ingest
write broadcast to every replica.

Wire messages (pickled tuples over the authenticated socket, our own processes
only):
  replica -> hub: ("hello", rank, capacity, info{..., mesh: address}) | ("event", job, name, data)
                  | ("health", info) | ("upsert", table, payload)          [mirror]
                  | ("shard_req", req, scope, op, payload)                 [shard round]
                  | ("shard_res", origin, req, result) | ("shard_wreq", req, owner, scope, op, payload)
  hub -> replica: ("run", job, request) | ("cancel", job) | ("upsert", table, payload) | ("stop",)
                  | ("peers", {rank: mesh address})                        [mesh membership]
                  | ("shard_plan", req, n_parts, ranks) | ("shard_part", req, rank, result)
                  | ("shard_exec", origin, req, scope, op, payload) | ("shard_wexec", origin, req, scope, op, payload)
A routed write (shard_wreq) is a one-part round: the owner applies it in arrival order (one writer thread)
and answers with its applied count; an owner that is not connected answers None and the writer raises.
"""
from __future__ import annotations

import asyncio
import logging
import os
import secrets
import subprocess
import sys
import threading
import time
from multiprocessing.connection import AuthenticationError, Client, Listener, answer_challenge, deliver_challenge

from . import metrics as M
from .events import CancelFlags, EventLog

log = logging.getLogger(__name__)


class _Replica:
    __slots__ = ("rank", "conn", "capacity", "inflight", "alive", "info", "lock", "jobs")

    def __init__(self, rank: int, conn, capacity: int, info: dict):
        self.rank = rank
        self.conn = conn
        self.capacity = max(0, int(capacity))  # 0: a shard-only replica (answers index rounds, runs no jobs)
        self.inflight = 0
        self.alive = True
        self.info = info
        self.lock = threading.Lock()
        self.jobs: set[str] = set()

    def send(self, msg) -> bool:
        with self.lock:
            if not self.alive:
                return False
            try:
                self.conn.send(msg)
                return True
            except (OSError, EOFError, BrokenPipeError):
                self.alive = False
                return False


class HubCancelFlags(CancelFlags):
    """Front-door cancel flags: a cancel is also forwarded to the replica that runs the job."""

    def __init__(self, hub: "ReplicaHub", ttl: float = 3600.0):
        super().__init__(ttl)
        self.hub = hub

    def cancel_sync(self, job_id: str) -> None:
        super().cancel_sync(job_id)
        self.hub.forward_cancel(job_id)


class ReplicaHub:
    """Accepts replica connections and dispatches jobs to them."""

    def __init__(self, events: EventLog, host: str = "127.0.0.1", port: int = 0, authkey: bytes | None = None,
                 job_timeout: float = 300.0, keep_result: float = 3600.0):
        from .worker import JobQueue

        self.events = events
        self.authkey = authkey or secrets.token_bytes(16)
        # authentication runs on each connection's reader thread (never the accept thread: one slow or stuck
        # client cannot hold up the other replicas' connects); a deep backlog absorbs connect bursts
        self.listener = Listener((host, port), backlog=128)
        self.address = self.listener.address
        self.replicas: dict[int, _Replica] = {}
        self.owner: dict[str, _Replica] = {}
        self._done: dict[str, tuple[asyncio.AbstractEventLoop, asyncio.Future]] = {}
        self._lock = threading.Lock()
        self._loop: asyncio.AbstractEventLoop | None = None
        self._slot_cond: asyncio.Condition | None = None
        self.flags = HubCancelFlags(self)
        # shard rounds in flight, by the replica that still owes a part: {rank: {(origin, req)}}
        self._shard_pending: dict[int, set] = {}
        # jobs the front door timed out whose replica has not sent its final event yet: {job: replica}
        self._timed_out: dict[str, _Replica] = {}
        self.timeout_grace = 60.0
        # the front door's queue admits as many jobs as the replicas have slots (it grows with every
        # replica that connects: set_max_jobs in _admit_capacity); the rest wait in FIFO order
        self.queue = JobQueue({"run_rag_job": self.run_rag_job}, max_jobs=16, job_timeout=job_timeout,
                              keep_result=keep_result)
        self.queue.ctx["on_timeout"] = self._on_timeout
        self._closed = False
        self._acceptor = threading.Thread(target=self._accept_loop, name="replica-hub-accept", daemon=True)
        self._acceptor.start()

    # ------------------------------------------------------------------ connections
    def _accept_loop(self) -> None:
        while not self._closed:
            try:
                conn = self.listener.accept()
            except (OSError, EOFError):
                if self._closed:
                    return
                continue
            except Exception:  # authentication failure of a stray connection
                log.warning("replica hub: rejected a connection", exc_info=True)
                continue
            threading.Thread(target=self._reader, args=(conn,), name="replica-hub-reader", daemon=True).start()

    def _reader(self, conn) -> None:
        rep = None
        from .mesh import cut_connection

        guard = threading.Timer(10.0, cut_connection, (conn,))  # a peer that never finishes the handshake
        guard.start()
        try:
            deliver_challenge(conn, self.authkey)
            answer_challenge(conn, self.authkey)
        except (AuthenticationError, EOFError, OSError, AssertionError, TypeError):
            log.warning("replica hub: rejected a connection (authentication)")
            conn.close()
            return
        finally:
            guard.cancel()
        try:
            hello = conn.recv()
            if not (isinstance(hello, tuple) and hello and hello[0] == "hello"):
                conn.close()
                return
            _, rank, capacity, info = hello
            rep = _Replica(int(rank), conn, capacity, info or {})
            with self._lock:
                old = self.replicas.get(rep.rank)
                self.replicas[rep.rank] = rep
            if old is not None:
                self._fail_replica(old, "replica re-registered")
            log.info("replica %d connected (capacity %d)", rep.rank, rep.capacity)
            M.CLUSTER_REPLICAS.set(self.live_count())
            self._broadcast_peers()  # before any job reaches the new replica (same connection, in order)
            self._admit_capacity()
            self._notify_slots()
            while True:
                msg = conn.recv()
                kind = msg[0]
                if kind == "event":
                    _, job_id, name, data = msg
                    if job_id in self._timed_out:  # the client already got error + final
                        if name == "final":
                            self._timed_out.pop(job_id, None)
                            self._finish(job_id)
                        continue
                    self.events.emit_sync(job_id, name, data)
                    if name == "final":
                        self._finish(job_id)
                elif kind == "health":
                    rep.info = {**rep.info, **msg[1]}  # hello fields (pid, shard) persist
                elif kind == "upsert":  # mirror mode: an ingest on this replica, applied on every other one
                    for other in self.live_replicas():
                        if other is not rep:
                            other.send(msg)
                elif kind == "shard_req":
                    self._shard_fanout(rep, *msg[1:])
                elif kind == "shard_res":
                    _, origin, req, result = msg
                    with self._lock:
                        self._shard_pending.get(rep.rank, set()).discard((origin, req))
                        o = self.replicas.get(origin)
                    if o is not None:
                        o.send(("shard_part", req, rep.rank, result))
                elif kind == "shard_wreq":  # an acknowledged routed write: a one-part round to the owner
                    _, req, owner, scope, op, payload = msg
                    with self._lock:
                        o = self.replicas.get(owner)
                        if o is not None and o.alive:
                            self._shard_pending.setdefault(owner, set()).add((rep.rank, req))
                    rep.send(("shard_plan", req, 1, [owner]))
                    if o is None or not o.alive or not o.send(("shard_wexec", rep.rank, req, scope, op, payload)):
                        with self._lock:
                            self._shard_pending.get(owner, set()).discard((rep.rank, req))
                        log.warning("shard write for replica %d not applied: replica not connected", owner)
                        rep.send(("shard_part", req, owner, None))
        except (EOFError, OSError, ConnectionResetError):
            pass
        finally:
            if rep is not None:
                self._fail_replica(rep, "replica disconnected")

    def _shard_fanout(self, origin: _Replica, req, scope, op, payload) -> None:
        """C4 of one shard round: every other live replica runs ``op`` on its shard."""
        targets = [r for r in self.live_replicas() if r is not origin]
        with self._lock:
            for t in targets:
                self._shard_pending.setdefault(t.rank, set()).add((origin.rank, req))
        origin.send(("shard_plan", req, len(targets), [t.rank for t in targets]))
        for t in targets:
            if not t.send(("shard_exec", origin.rank, req, scope, op, payload)):
                with self._lock:
                    self._shard_pending.get(t.rank, set()).discard((origin.rank, req))
                origin.send(("shard_part", req, t.rank, None))

    def _fail_replica(self, rep: _Replica, why: str) -> None:
        with rep.lock:
            was_alive = rep.alive
            rep.alive = False
        with self._lock:
            owed = self._shard_pending.pop(rep.rank, set())
        for origin, req in owed:  # rounds still waiting for this replica's part: answer them empty
            with self._lock:
                o = self.replicas.get(origin)
            if o is not None:
                o.send(("shard_part", req, rep.rank, None))
        with self._lock:
            if self.replicas.get(rep.rank) is rep:
                self.replicas.pop(rep.rank, None)
            jobs = [j for j, r in self.owner.items() if r is rep]
        if was_alive:
            log.warning("replica %d: %s (%d jobs in flight)", rep.rank, why, len(jobs))
        for j in jobs:
            if not self.events.is_closed(j):
                self.events.emit_sync(j, "error", {"message": f"replica {rep.rank} lost: {why}"})
                self.events.emit_sync(j, "final", {"answer": "", "sources": None, "error": True})
            self._finish(j)
        M.CLUSTER_REPLICAS.set(self.live_count())
        if was_alive:
            self._broadcast_peers()
        self._notify_slots()

    def _broadcast_peers(self) -> None:
        """Mesh membership: every live replica learns every live replica's mesh address."""
        live = self.live_replicas()
        peers = {r.rank: tuple(r.info["mesh"]) for r in live if r.info.get("mesh")}
        for r in live:
            if r.info.get("mesh"):
                r.send(("peers", peers))

    def _admit_capacity(self) -> None:
        """The front door's queue runs as many jobs at once as the replicas have slots (never fewer
        than it ever had: a reconnecting replica finds its consumers there)."""
        cap = self.capacity()
        if cap > self.queue.max_jobs:
            self.queue.set_max_jobs(cap)

    # ------------------------------------------------------------------ scheduling
    def live_replicas(self) -> list[_Replica]:
        with self._lock:
            return [r for r in self.replicas.values() if r.alive]

    def live_count(self) -> int:
        return len(self.live_replicas())

    def capacity(self) -> int:
        return sum(r.capacity for r in self.live_replicas())

    def _notify_slots(self) -> None:
        loop, cond = self._loop, self._slot_cond
        if loop is None or cond is None:
            return

        async def _n():
            async with cond:
                cond.notify_all()

        coro = _n()
        try:
            asyncio.run_coroutine_threadsafe(coro, loop)
        except RuntimeError:  # loop closed
            coro.close()

    def _pick(self) -> _Replica | None:
        free = [r for r in self.live_replicas() if r.inflight < r.capacity]
        return min(free, key=lambda r: (r.inflight / r.capacity, r.rank)) if free else None

    def _finish(self, job_id: str) -> None:
        with self._lock:
            rep = self.owner.pop(job_id, None)
            fut = self._done.pop(job_id, None)
        if rep is not None:
            with rep.lock:
                rep.inflight = max(0, rep.inflight - 1)
                rep.jobs.discard(job_id)
            M.CLUSTER_INFLIGHT.labels(replica=str(rep.rank)).set(rep.inflight)
        if fut is not None:
            loop, f = fut
            loop.call_soon_threadsafe(lambda: f.done() or f.set_result(True))
        self._notify_slots()

    async def wait_for_replicas(self, n: int, timeout: float = 600.0) -> None:
        self._bind_loop()
        t0 = time.time()
        while self.live_count() < n:
            if time.time() - t0 > timeout:
                raise TimeoutError(f"only {self.live_count()} of {n} replicas connected")
            await asyncio.sleep(0.05)

    def _bind_loop(self) -> None:
        if self._loop is None:
            self._loop = asyncio.get_running_loop()
            self._slot_cond = asyncio.Condition()

    async def run_rag_job(self, ctx, job_id: str, req: dict):
        """JobQueue function: place the job on a replica and wait for its final event."""
        self._bind_loop()
        loop = asyncio.get_running_loop()
        t0 = time.perf_counter()
        async with self._slot_cond:
            while True:
                rep = self._pick()
                if rep is not None:
                    break
                if self.live_count() == 0 and time.perf_counter() - t0 > 30.0:
                    self.events.emit_sync(job_id, "error", {"message": "no replica available"})
                    self.events.emit_sync(job_id, "final", {"answer": "", "sources": None, "error": True})
                    return None
                try:
                    await asyncio.wait_for(self._slot_cond.wait(), timeout=1.0)
                except asyncio.TimeoutError:
                    pass
            fut = loop.create_future()
            with self._lock:
                self.owner[job_id] = rep
                self._done[job_id] = (loop, fut)
            with rep.lock:
                rep.inflight += 1
                rep.jobs.add(job_id)
        M.CLUSTER_INFLIGHT.labels(replica=str(rep.rank)).set(rep.inflight)
        M.CLUSTER_DISPATCH.labels(replica=str(rep.rank)).inc()
        req = dict(req, _enqueued=(self.queue.results.get(job_id) or {}).get("enqueued"))
        if not rep.send(("run", job_id, req)):
            self._fail_replica(rep, "send failed")
        if self.flags.is_cancelled_sync(job_id):
            rep.send(("cancel", job_id))
        await fut
        return {"replica": rep.rank}

    def forward_cancel(self, job_id: str) -> None:
        with self._lock:
            rep = self.owner.get(job_id)
        if rep is not None:
            rep.send(("cancel", job_id))

    async def _on_timeout(self, job_id: str, req: dict) -> None:
        """The client gets error + final now; the replica's slot stays taken until the replica
        reports the (cooperatively) cancelled job's final event, or ``timeout_grace`` passes, so the
        hub never sends a replica more jobs than it advertised capacity for."""
        with self._lock:
            rep = self.owner.get(job_id)
            if rep is not None:
                self._timed_out[job_id] = rep
        self.flags.cancel_sync(job_id)
        if not self.events.is_closed(job_id):
            await self.events.emit(job_id, "error", {"message": f"job timed out after {self.queue.job_timeout}s"})
            await self.events.emit(job_id, "final", {"answer": "", "sources": None, "error": True})
        if rep is None:
            self._finish(job_id)
            return

        def _deadline():
            if self._timed_out.pop(job_id, None) is not None:
                log.warning("replica %d never finished timed-out job %s; freeing its slot", rep.rank, job_id)
                self._finish(job_id)

        asyncio.get_running_loop().call_later(self.timeout_grace, _deadline)

    def health(self) -> dict:
        reps = sorted(self.live_replicas(), key=lambda r: r.rank)
        return {"replicas": [{"rank": r.rank, "capacity": r.capacity, "inflight": r.inflight, **r.info}
                             for r in reps], "live": len(reps)}

    def close(self) -> None:
        self._closed = True
        for r in self.live_replicas():
            r.send(("stop",))
        try:
            self.listener.close()
        except OSError:
            pass


class ClusterRuntimeView:
    """What the API and /health need from a runtime, at a front door that holds no model."""

    def __init__(self, hub: ReplicaHub, settings):
        self.hub = hub
        self.settings = settings
        self.runner = None

    def health(self) -> dict:
        return self.hub.health()


# ---------------------------------------------------------------------- replica side
class _ForwardingEvents(EventLog):
    """A replica's event log: every event is also forwarded to the hub (the replica keeps its own copy so
    its worker's timeout / cancel paths behave exactly as in a single-process server)."""

    def __init__(self, send):
        super().__init__()
        self._send = send

    def emit_sync(self, job_id: str, event: str, data) -> None:
        super().emit_sync(job_id, event, data)
        self._send(("event", job_id, event, data))

    emit_threadsafe = emit_sync


class HubShardTransport:
    """A replica's end of the shard rounds routed by the hub (index/sharded_store.py transport)."""

    def __init__(self, send, rank: int):
        import itertools

        self._send = send
        self.rank = rank
        self._ids = itertools.count()
        self._lock = threading.Lock()
        self._rounds: dict[int, dict] = {}

    def fanout(self, origin: int, scope: str, op: str, payload, timeout: float = 60.0) -> list:
        req = next(self._ids)
        st = {"n": None, "parts": {}, "ev": threading.Event()}
        with self._lock:
            self._rounds[req] = st
        try:
            self._send(("shard_req", req, scope, op, payload))
            if not st["ev"].wait(timeout):
                log.warning("shard %s round %d on %s: %d of %s parts after %.0fs", op, req, scope,
                            len(st["parts"]), st["n"], timeout)
            with self._lock:
                parts = dict(st["parts"])
                expected = st.get("ranks")
                planned = st["n"] is not None
            from .mesh import Parts

            missing = [r for r, p in parts.items() if p is None]
            # a shard that never answered before the timeout is missing too (the round is degraded); with no
            # plan at all (the hub itself did not answer) the expected ranks are unknown: flagged as rank -1
            missing += [r for r in (expected or []) if r not in parts]
            if not planned:
                missing.append(-1)
            return Parts([p for p in parts.values() if p is not None], missing=missing)
        finally:
            with self._lock:
                self._rounds.pop(req, None)

    def write(self, origin: int, owner: int, scope: str, op: str, payload, timeout: float = 120.0):
        """An acknowledged routed write (a one-part round to the owner): its applied count, or
        ShardWriteError when the owner is gone or did not answer."""
        from .mesh import ShardWriteError

        req = next(self._ids)
        st = {"n": None, "parts": {}, "ev": threading.Event()}
        with self._lock:
            self._rounds[req] = st
        try:
            self._send(("shard_wreq", req, owner, scope, op, payload))
            if not st["ev"].wait(timeout):
                raise ShardWriteError(f"shard {owner} did not acknowledge {op} on {scope} within {timeout:.0f}s")
            res = st["parts"].get(owner)
            if res is None:
                raise ShardWriteError(f"shard {owner} did not apply {op} on {scope} (not connected or failed)")
            return res
        finally:
            with self._lock:
                self._rounds.pop(req, None)

    def deliver(self, msg) -> None:
        """Reader thread: a plan or a part of one of this replica's rounds."""
        kind, req = msg[0], msg[1]
        with self._lock:
            st = self._rounds.get(req)
            if st is None:
                return
            if kind == "shard_plan":
                st["n"] = msg[2]
                st["ranks"] = list(msg[3]) if len(msg) > 3 else None
            else:  # keyed by the answering rank: a duplicate (e.g. an empty answer from the hub's
                # failed-send path AND its replica-lost path) cannot complete the round early
                st["parts"].setdefault(int(msg[2]), msg[3])
            if st["n"] is not None and len(st["parts"]) >= st["n"]:
                st["ev"].set()


def attach_sharded_store(runtime, transport, rank: int, nshards: int):
    """Serve ``runtime``'s (already shard-local) store as shard ``rank`` of ``nshards``:
    the agent's retrievers and the ingest writer see the union of all shards."""
    from ..index.sharded_store import ShardedStore
    from ..retrieval.graph import RetrieverFactory

    local = runtime.store
    runtime.local_store = local
    runtime.store = ShardedStore(local, rank, nshards, transport)
    runtime.retrievers = RetrieverFactory(runtime.store, runtime.embedder)
    return local


def run_replica(runtime, address, authkey: bytes, rank: int, capacity: int | None = None,
                health_every: float = 5.0, shards: int = 1, group=None) -> int:
    """Serve jobs from the hub until it says stop or the connection drops (blocking).
    ``shards`` > 1: this replica holds shard ``rank`` of a row-sharded index and answers
    the other replicas' shard rounds (service/cluster.py docstring)."""
    from concurrent.futures import ThreadPoolExecutor

    from ..index.sharded_store import execute
    from .worker import RAGWorker

    s = runtime.settings
    cap = capacity if capacity is not None else s.worker_max_jobs
    conn = Client(tuple(address) if isinstance(address, list) else address, authkey=authkey)
    send_lock = threading.Lock()

    def send(msg):
        with send_lock:
            conn.send(msg)

    transport = None
    mesh = None
    coll = None
    local_store = getattr(runtime, "store", None)
    kind = os.environ.get("GRAG_SHARD_TRANSPORT", "collective" if group is not None else "mesh")
    if shards > 1 and local_store is not None:
        if kind == "hub":
            transport = HubShardTransport(send, rank)
        else:  # replica-to-replica rounds (service/mesh.py); the hub only tells us who the peers are
            from .mesh import PeerMesh

            transport = mesh = PeerMesh(rank, shards, authkey, host=os.environ.get("GRAG_MESH_HOST", "127.0.0.1"))
            if kind == "collective" and group is not None and group.size == shards:
                # reads as lockstep collectives over the replicas' process group (service/collective.py: RCCL
                # over xGMI with one replica per GPU); routed writes stay on the mesh
                from .collective import CollectiveShardTransport

                transport = coll = CollectiveShardTransport(rank, shards, group, getattr(runtime, "device", "cpu"),
                                                            fallback=mesh)
        local_store = attach_sharded_store(runtime, transport, rank, shards)
        if mesh is not None:
            mesh.store = local_store
        if coll is not None:
            coll.store = local_store
    # other replicas' shard rounds and routed writes run here, off the job loop (GPU search + sync)
    shard_pool = ThreadPoolExecutor(4, thread_name_prefix="shard-exec")
    events = _ForwardingEvents(send)
    flags = CancelFlags()
    worker = RAGWorker(runtime, events, flags, max(1, cap), s.job_timeout_s, s.keep_result_s, s.stream_tokens)
    store = getattr(runtime, "store", None)
    if transport is None and store is not None and hasattr(store, "add_listener"):
        store.add_listener(lambda table, payload: send(("upsert", table, payload)))
    send(("hello", rank, cap, {"device": str(getattr(runtime, "device", "cpu")), "pid": os.getpid(),
                               "shard": f"{rank}/{shards}" if transport is not None else "full",
                               **({"mesh": tuple(mesh.address)} if mesh is not None else {})}))

    def shard_exec(origin, req, scope, op, payload):
        try:
            res = execute(local_store, scope, op, payload)
        except Exception:  # answer the round anyway: the origin must not wait for a failed shard
            log.exception("shard %s on %s for replica %d failed", op, scope, origin)
            res = None
        try:
            send(("shard_res", origin, req, res))
        except (OSError, EOFError):
            pass

    write_pool = ThreadPoolExecutor(1, thread_name_prefix="shard-write")  # routed writes: in arrival order

    def shard_wexec(origin, req, scope, op, payload):
        try:
            res = execute(local_store, scope, op, payload)
        except Exception:
            log.exception("routed shard write (%s on %s) from replica %d failed", op, scope, origin)
            res = None
        try:
            send(("shard_res", origin, req, res))
        except (OSError, EOFError):
            pass

    async def main():
        loop = asyncio.get_running_loop()
        inbox: asyncio.Queue = asyncio.Queue()

        def reader():
            try:
                while True:
                    msg = conn.recv()
                    kind = msg[0]
                    if kind == "peers" and mesh is not None:
                        mesh.set_peers(msg[1])
                    elif kind in ("shard_plan", "shard_part") and isinstance(transport, HubShardTransport):
                        transport.deliver(msg)
                    elif kind == "shard_exec":
                        shard_pool.submit(shard_exec, *msg[1:])
                    elif kind == "shard_wexec":
                        write_pool.submit(shard_wexec, *msg[1:])
                    else:
                        loop.call_soon_threadsafe(inbox.put_nowait, msg)
            except (EOFError, OSError):
                try:
                    loop.call_soon_threadsafe(inbox.put_nowait, ("stop",))
                except RuntimeError:  # the replica loop already returned (the hub said stop)
                    pass

        threading.Thread(target=reader, name="replica-reader", daemon=True).start()
        tasks = set()
        last_h = 0.0
        while True:
            try:
                msg = await asyncio.wait_for(inbox.get(), timeout=health_every)
            except asyncio.TimeoutError:
                msg = None
            if time.time() - last_h >= health_every:
                last_h = time.time()
                try:
                    h = runtime.health() if hasattr(runtime, "health") else {}
                    if mesh is not None:
                        h = {**h, "mesh_stats": mesh.round_stats()}
                    if coll is not None:
                        h = {**h, "collective_stats": coll.round_stats()}
                    send(("health", {"device": str(getattr(runtime, "device", "cpu")), **h}))
                except Exception:  # pragma: no cover
                    pass
            if msg is None:
                continue
            kind = msg[0]
            if kind == "run":
                _, job_id, req = msg
                enq = req.pop("_enqueued", None)
                worker.queue.results[job_id] = {"status": "running", "enqueued": enq or time.time()}

                async def _run(job_id=job_id, req=req):
                    try:
                        await asyncio.wait_for(worker.run_rag_job(worker.queue.ctx, job_id, req),
                                               timeout=worker.queue.job_timeout)
                    except asyncio.TimeoutError:
                        await worker._on_timeout(job_id, req)
                    finally:
                        worker.queue.results.pop(job_id, None)

                t = asyncio.create_task(_run())
                tasks.add(t)
                t.add_done_callback(tasks.discard)
            elif kind == "cancel":
                flags.cancel_sync(msg[1])
            elif kind == "upsert" and store is not None and hasattr(store, "apply_remote"):
                # mirror mode: a write (maybe triggering a compaction) must not stall job dispatch / health
                loop.run_in_executor(shard_pool, store.apply_remote, msg[1], msg[2])
            elif kind == "stop":
                for t in list(tasks):
                    t.cancel()
                return

    try:
        asyncio.run(main())
    finally:
        shard_pool.shutdown(wait=False)
        write_pool.shutdown(wait=False)
        if coll is not None:
            coll.close()  # collective: the rounds stop once every replica has asked to
        if mesh is not None:
            mesh.close()
        try:
            conn.close()
        except OSError:
            pass
    return 0


def spawn_replicas(n: int, address, authkey: bytes, extra_args=(), gpus: list[int] | None = None,
                   env: dict | None = None, shards: int = 1) -> list[subprocess.Popen]:
    """Start one replica child process per GPU (HIP_VISIBLE_DEVICES pins it; never an exec of this
    process).  The authkey travels in the environment, not on the command line.  With
    sharded replicas (the default transport, GRAG_SHARD_TRANSPORT=collective; =mesh / =hub keep the socket
    transports) the replicas also form a torch.distributed group (rank = replica) for their shard rounds
    (service/collective.py)."""
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        pg_port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        e = dict(os.environ, **(env or {}))
        e["GRAG_HUB_AUTHKEY"] = authkey.hex()
        if gpus is not None:
            e["HIP_VISIBLE_DEVICES"] = str(gpus[r])
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if shards > 1 and e.setdefault("GRAG_SHARD_TRANSPORT", "collective") == "collective":
            # the replicas' process group (service/collective.py): RCCL when each has its own GPU
            e.update(RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                     MASTER_PORT=str(pg_port))
            if gpus is None or len(set(gpus[:n])) < n:
                e.setdefault("GRAG_DIST_BACKEND", "gloo")
        cmd = [sys.executable, "-m", "githubrepostorag_amd", "replica", "--hub", f"{address[0]}:{address[1]}",
               "--rank", str(r), "--shards", str(shards), *extra_args]
        procs.append(subprocess.Popen(cmd, env=e))
    return procs


def gpu_demo_runtime(settings):
    """A GPU replica runtime on the product path: the real in-process engine (QWEN_MODEL, e.g. the
    qwen2-small config with random weights: hipGraph decode, paged KV, fused sampler), a tiny encoder and
    the GPU vector store over the demo chunks.  For the front door's GPU test (tests/test_cluster_gpu.py)
    and GPU rehearsals of ``serve --replicas`` without checkpoints."""
    from ..embed.service import Embedder
    from ..index.store import VectorStore
    from .runtime import RAGRuntime

    dev = "cuda"
    emb = Embedder.from_name("encoder-tiny", device=dev, seed=3)
    store = VectorStore(emb.dim, dev)
    texts = ["widgets code", "gadget service", "billing module"]
    store.table("chunk").upsert(["widgets", "gadget", "billing"], texts, emb.embed_documents(texts),
                                [{"namespace": "default", "repo": "r", "module": "m", "file_path": f"{x}.py"}
                                 for x in "abc"])
    return RAGRuntime(settings, device=dev, embedder=emb, store=store)


def demo_runtime(settings):
    """A CPU replica runtime with a scripted LLM and a tiny encoder over three chunks (tests, and a
    GPU-less rehearsal of ``serve --replicas``: ``replica --factory
    githubrepostorag_amd.service.cluster:demo_runtime``).  GRAG_DEMO_LLM_DELAY (s) slows each LLM call;
    GRAG_DEMO_DEVICE=cuda keeps the tables (and the shard rounds' searches) on the GPU."""
    from ..agent.llm import ScriptedLLM
    from ..embed.service import Embedder
    from ..index.store import VectorStore
    from .runtime import RAGRuntime

    delay = float(os.environ.get("GRAG_DEMO_LLM_DELAY", "0"))

    def router(p):
        if delay:
            time.sleep(delay)
        if p.startswith("Choose the best search scope"):
            return '{"scope": "code"}'
        if "Judge if the retrieved" in p:
            return '{"coverage": 0.9, "needs_more": false}'
        if p.startswith("Generate 3-4"):
            return '["alt query"]'
        return f"Widgets are handled in [1] (replica pid {os.getpid()})."

    dev = os.environ.get("GRAG_DEMO_DEVICE", "cpu")
    emb = Embedder.from_name("encoder-tiny", device="cpu", seed=3)
    store = VectorStore(emb.dim, dev)
    texts = ["widgets code", "gadget service", "billing module"]
    # row ids split over two shards (crc32 mod 2: widgets -> 1, gadget / billing -> 0)
    store.table("chunk").upsert(["widgets", "gadget", "billing"], texts, emb.embed_documents(texts),
                                [{"namespace": "default", "repo": "r", "module": "m", "file_path": f"{x}.py"}
                                 for x in "abc"])
    extra = int(os.environ.get("GRAG_DEMO_ROWS", "0"))  # load tests: a larger synthetic table per scope
    if extra:
        import torch

        g = torch.Generator().manual_seed(11)
        for scope in ("chunk", "file", "module", "repo"):
            v = torch.nn.functional.normalize(torch.randn(extra, emb.dim, generator=g), dim=1)
            store.table(scope).upsert([f"{scope}-{i}" for i in range(extra)], [f"{scope} text {i}" for i in range(extra)],
                                      v, [{"namespace": "default", "repo": f"r{i % 7}", "module": f"m{i % 23}",
                                           "file_path": f"m{i % 23}/f{i % 97}.py"} for i in range(extra)])
    settings.worker_max_jobs = int(os.environ.get("GRAG_DEMO_SLOTS", settings.worker_max_jobs))
    return RAGRuntime(settings, device=dev, llm=ScriptedLLM(router), embedder=emb, store=store,
                      build_engine=False)
