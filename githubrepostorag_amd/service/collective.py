"""Shard rounds as lockstep device collectives among the replicas.

``service/mesh.py`` answers a replica's retrieval hop over direct sockets: pickled numpy
payloads, one request per peer.  When the replicas share a process group (one process per
GPU: RCCL over xGMI; on one shared card: gloo), this transport carries the same hops as
collectives instead:

  * every replica runs ONE round thread; a round starts every ``tick`` seconds on all of them
    (lockstep: the group's collectives are issued in the same order on every rank);
  * C4 -- the reads each replica queued since the last round (its jobs' searches, graph-edge
    lookups, counts) are pickled into a uint8 tensor and ALL-GATHERED (sizes first, then the
    padded payloads): every shard sees every replica's requests of the round;
  * each shard runs all the other replicas' reads against its own rows, the plain searches that
    share (table, k, filter) stacked into ONE fused score+top-k launch (as the mesh does);
  * C3 -- the answers go back in ONE all-to-all (slice j = the answers to replica j's requests,
    padded to the round's largest slice); every origin then holds each shard's part of each of
    its requests and the sharded table merges them (index/sharded_store.merge_hits);
  * a round nobody queued anything for costs one 2-int all-gather and a sleep.

Writes (routed upserts / deletes, acknowledged in order by the owner) stay on the ``fallback``
transport (the mesh): they are rare, ordered and need an owner acknowledgement, not a round.
On one card with several replica processes (the test box) the group is gloo and the payloads
cross the host; on a node with one replica per GPU the group is RCCL and every hop is a device
collective over xGMI.
"""
from __future__ import annotations

import logging
import pickle
import threading
import time

import torch

log = logging.getLogger(__name__)


class _Req:
    __slots__ = ("rid", "scope", "op", "payload", "ev", "parts")

    def __init__(self, rid, scope, op, payload):
        self.rid, self.scope, self.op, self.payload = rid, scope, op, payload
        self.ev = threading.Event()
        self.parts: dict[int, object] = {}


class CollectiveShardTransport:
    def __init__(self, rank: int, nshards: int, group, device, store=None, fallback=None, tick: float = 0.0005):
        self.rank, self.nshards = rank, nshards
        self.group = _own_group(group)
        self.device = torch.device(device)
        self.store = store  # this replica's shard (set by the caller once the sharded store is attached)
        self.fallback = fallback
        self.tick = tick
        self._q: list[_Req] = []
        self._lock = threading.Lock()
        self._cv = threading.Condition(self._lock)
        self._ids = 0
        self._stop = False
        self._closed = threading.Event()
        # rounds / degraded_rounds: this replica's fan-outs (as the mesh counts them); ticks: lockstep rounds
        self.stats = {"rounds": 0, "degraded_rounds": 0, "ticks": 0, "busy_rounds": 0, "requests": 0, "served": 0, "stacked_searches": 0,
                      "bytes_out": 0, "device_exchanges": 0}
        # plain-search answers pruned to each query's global winners through a score all-gather (C3 as a
        # tensor exchange, _prune_searches); GRAG_SHARD_PRUNE=0 sends every shard's top-k
        import os

        self.prune = os.environ.get("GRAG_SHARD_PRUNE", "1") != "0"
        self.prune_min = int(os.environ.get("GRAG_SHARD_PRUNE_MIN", "128"))  # candidate hits in the round
        self._broken = False  # the group failed: rounds go to the fallback transport (fanout)
        self._ipc_bad = False  # this rank's device exchange timed out (reported in the next round's header)
        self._ipc_off = False  # every rank left the device exchange at the same round
        self._lat: list[float] = []
        self._th = threading.Thread(target=self._loop, name="shard-collective", daemon=True)
        self._th.start()

    # ------------------------------------------------------------------ client side (the sharded table)
    def fanout(self, origin: int, scope: str, op: str, payload, timeout: float = 60.0):
        from .mesh import Parts

        r = None
        with self._cv:
            if not (self._broken and self.fallback is not None):
                self._ids += 1
                r = _Req(self._ids, scope, op, payload)
                self._q.append(r)
                self._cv.notify()
        if r is None:
            # the replicas' process group broke (a replica died: a collective cannot leave one rank out):
            # the socket mesh carries the rounds from here on and reports the lost shard as missing
            self.stats["fallback_rounds"] = self.stats.get("fallback_rounds", 0) + 1
            return self.fallback.fanout(origin, scope, op, payload, timeout)
        t0 = time.monotonic()
        ok = r.ev.wait(timeout)
        self._lat.append(time.monotonic() - t0)
        if len(self._lat) > 8192:
            del self._lat[:4096]
        missing = [s for s in range(self.nshards) if s != self.rank and s not in r.parts]
        self.stats["rounds"] += 1
        if missing or any(v is None for v in r.parts.values()):
            self.stats["degraded_rounds"] += 1
        if not ok:
            log.warning("collective %s round on %s timed out after %.0fs", op, scope, timeout)
        return Parts([v for s, v in sorted(r.parts.items()) if v is not None],
                     missing=missing + [s for s, v in r.parts.items() if v is None])

    def write(self, origin: int, owner: int, scope: str, op: str, payload, timeout: float = 120.0):
        if self.fallback is None:
            from .mesh import ShardWriteError

            raise ShardWriteError("collective shard transport has no write path (fallback transport missing)")
        return self.fallback.write(origin, owner, scope, op, payload, timeout)

    def round_stats(self) -> dict:
        lat = sorted(self._lat)
        out = dict(self.stats)
        if lat:
            out["p50_ms"] = round(1000 * lat[len(lat) // 2], 3)
            out["p99_ms"] = round(1000 * lat[min(len(lat) - 1, int(0.99 * len(lat)))], 3)
        return out

    def close(self, timeout: float = 30.0) -> None:
        """Stop after the round in which EVERY replica asked to stop (collective: call on all ranks)."""
        with self._cv:
            self._stop = True
            self._cv.notify()
        self._closed.wait(timeout)

    # ------------------------------------------------------------------ the round thread
    def _device_path(self):
        """The group's one-shot IPC exchange (parallel/custom_ar.py) when attached: payloads move
        through GPU memory of the replicas' card(s); None -> the process group's own collectives."""
        return None if self._ipc_off else getattr(self.group, "custom_ar", None)

    def _gather_bytes(self, blob: bytes, sizes: list[int]) -> list[bytes]:
        """Every rank's ``blob`` (their sizes already agreed in the round header)."""
        mx = -(-max(sizes) // 16) * 16
        if mx == 0:
            return [b""] * len(sizes)
        buf = torch.zeros(mx, dtype=torch.uint8)
        if blob:
            buf[: len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
        allb = self._gather_payload(buf)
        return [allb[r, : sizes[r]].numpy().tobytes() for r in range(len(sizes))]

    def _gather_payload(self, buf: torch.Tensor) -> torch.Tensor:
        """[nbytes] host uint8 (a multiple of 16) -> [size, nbytes] host: the device exchange when it
        fits, else the process group (RCCL on the GPU, gloo on the host)."""
        ar = self._device_path()
        if ar is not None and buf.numel() <= ar.slot_bytes:
            d = buf.to(self.device, non_blocking=False)
            out = ar.all_gather(d).cpu()  # the D2H copy is the round's sync point
            if ar.failed():
                self._ipc_bad = True
            self.stats["device_exchanges"] += 1
            return out
        if self._cdev.type == "cuda":
            return self.group.all_gather(buf.to(self._cdev)).cpu()
        return _host_gather(self.group, buf)

    def _exchange(self, slices: list[bytes]) -> list[bytes]:
        """slices[j] -> rank j; returns what every rank sent to this one.  One all-to-all on the process
        group; on the device exchange one all-gather of the [size, max] slab (each rank keeps its column:
        the IPC one-shot gather has no all-to-all, and these slabs are KBs)."""
        g = self.group
        lens = torch.tensor([len(b) for b in slices], dtype=torch.int64, device=self._cdev)
        all_lens = (g.all_gather(lens).cpu() if self._cdev.type == "cuda" else _host_gather(g, lens))
        all_lens = all_lens.view(g.size, g.size)  # [src, dst]
        mx = -(-int(all_lens.max()) // 16) * 16
        if mx == 0:
            return [b""] * g.size
        buf = torch.zeros(g.size, mx, dtype=torch.uint8)
        for j, b in enumerate(slices):
            if b:
                buf[j, : len(b)] = torch.frombuffer(bytearray(b), dtype=torch.uint8)
        self.stats["bytes_out"] += sum(len(b) for b in slices)
        ar = self._device_path()
        if ar is not None and buf.numel() <= ar.slot_bytes:
            got = self._gather_payload(buf.view(-1)).view(g.size, g.size, mx)[:, self.rank]
        elif self._cdev.type == "cuda":
            got = g.all_to_all(buf.to(self._cdev)).cpu()
        else:
            got = _host_all_to_all(g, buf)
        return [got[s, : int(all_lens[s, self.rank])].numpy().tobytes() for s in range(g.size)]

    def _loop(self) -> None:
        from ..utils.gpu_guard import gpu_shared, set_device_of, side_stream

        g = self.group
        # the round header (and the fallback payload path) on the group's control device: RCCL -> the GPU,
        # gloo -> the host.  The header is what keeps the ranks in step: it is a host-synchronising
        # collective under gloo, so the device exchange that follows never spins long on a late peer.
        self._cdev = g.ctrl_device(self.device) if hasattr(g, "ctrl_device") else torch.device("cpu")
        if self.device.type == "cuda":
            set_device_of(self.device)
        idle = 0
        try:
            while True:
                with self._cv:
                    if not self._q:  # (a closing rank keeps the tick until every rank has closed)
                        # lockstep rounds: a busy system turns every tick; an idle one backs off (x4 after
                        # 64 empty rounds, x20 after 1024) -- a new request then waits at most that long
                        self._cv.wait(self.tick if idle < 64 else 4 * self.tick if idle < 1024 else 20 * self.tick)
                    mine, self._q = self._q, []
                    stop = self._stop
                # the round's host syncs (.cpu() of its collectives) never run inside another thread's hipGraph
                # capture: the round holds the capture guard shared -- "urgent", i.e. not queued behind a
                # capture that is only waiting, since job threads holding the guard wait on this round
                with (gpu_shared(urgent=True) if self.device.type == "cuda" else _null()), \
                        (side_stream(self.device) if self.device.type == "cuda" else _null()):
                    blob = pickle.dumps([(r.rid, r.scope, r.op, r.payload) for r in mine],
                                        protocol=pickle.HIGHEST_PROTOCOL) if mine else b""
                    hdr = torch.tensor([len(mine), int(stop), int(not self._ipc_bad), len(blob)], dtype=torch.int64)
                    head = (g.all_gather(hdr.to(self._cdev)).cpu() if self._cdev.type == "cuda"
                            else _host_gather(g, hdr)).view(-1, 4)
                    self.stats["ticks"] += 1
                    if int(head[:, 2].min()) == 0 and not self._ipc_off:
                        # some rank's device exchange timed out last round: every rank leaves it at this
                        # same round (that round's requests on the failing rank were reported missing)
                        log.warning("collective shard transport: device exchange failed on a replica; "
                                    "rounds continue on the process group")
                        self._ipc_off = True
                        self.stats["device_detached"] = 1
                    if int(head[:, 1].min()) == 1:  # every replica is closing: the last round
                        for r in mine:
                            r.ev.set()
                        return
                    if int(head[:, 0].sum()) == 0:
                        idle += 1
                        continue
                    idle = 0
                    self.stats["busy_rounds"] += 1
                    self.stats["requests"] += len(mine)
                    failed_before = self._ipc_bad
                    allreq = [_loads(b) for b in self._gather_bytes(blob, head[:, 3].tolist())]
                    # answer every other replica's reads on this shard (stacked plain searches)
                    results = {}
                    for src, items in enumerate(allreq):
                        if src == self.rank or not items:
                            continue
                        self.stats["served"] += len(items)
                        results[src] = self._run_reads(items)
                    if self.prune:  # C3 as a tensor exchange: only each query's global winners travel back
                        _t = time.perf_counter()
                        results = self._prune_searches(allreq, results)
                        self.stats["prune_s"] = self.stats.get("prune_s", 0.0) + time.perf_counter() - _t
                    answers = [pickle.dumps(results[src], protocol=pickle.HIGHEST_PROTOCOL) if src in results
                               else b"" for src in range(g.size)]
                    back = self._exchange(answers)
                    round_bad = self._ipc_bad and not failed_before
                by_id = {r.rid: r for r in mine}
                for src, b in enumerate(back):
                    if src == self.rank or round_bad:  # a timed-out exchange: this round's parts are missing
                        continue
                    res = _loads(b)
                    for rid, ok, val in (res if isinstance(res, list) else []):
                        r = by_id.get(rid)
                        if r is not None:
                            r.parts[src] = val if ok else None
                for r in mine:
                    r.ev.set()
        except Exception:  # a broken group: every waiter learns it at once (missing shards -> degraded)
            log.exception("collective shard transport: round failed; later rounds go to the fallback transport")
            with self._cv:
                self._broken = True
                pending, self._q = self._q, []
            for r in pending:
                r.ev.set()
        finally:
            self._closed.set()

    def _run_reads(self, items):
        from .mesh import run_reads

        return run_reads(self.store, items, self.stats)

    def _prune_searches(self, allreq, results: dict) -> dict:
        """C3 of the round's plain searches as one tensor collective: every shard's per-query top-k SCORES
        ([rows, K] fp32, -inf padded; rows = every plain-search query row of the round in request order,
        the same layout on every rank since every rank holds every request) are all-gathered; each rank
        then computes, for every row, the global top-k over the shards other than the row's origin (the
        origin merges its own shard locally) -- identically on every rank (stable sort by score, ties by
        shard, then position) -- and sends back only ITS winning hits.  Without this every shard returned k
        hits per query, (W - 1) k per query to merge at the origin; now at most k travel in total.  The
        score exchange is a device all-gather on RCCL (host gloo on one shared card)."""
        import numpy as np

        g = self.group
        layout = []
        for o, items in enumerate(allreq):
            for rid, scope, op, payload in items or ():
                if op == "search":
                    Q, k, _ = payload
                    q = np.asarray(Q)
                    layout.append((o, rid, 1 if q.ndim == 1 else int(q.shape[0]), int(k)))
        if not layout:
            return results
        R = sum(x[2] for x in layout)
        K = max(1, max(x[3] for x in layout))
        # the score exchange is one more collective in the round: it pays when the candidates it keeps off
        # the answer exchange are many (decided from the gathered requests, so identically on every rank)
        if R * K * (g.size - 1) < self.prune_min:
            return results
        row0, r = {}, 0
        for o, rid, nq, _ in layout:
            row0[(o, rid)] = r
            r += nq
        S = torch.full((R, K), float("-inf"), dtype=torch.float32)
        for src, res in results.items():
            for rid, ok, val in res:
                base = row0.get((src, rid))
                if base is None or not ok or not isinstance(val, list):
                    continue
                for qi, hits in enumerate(val):
                    for j, h in enumerate(hits[:K]):
                        sc = getattr(h, "score", None)
                        S[base + qi, j] = float(sc) if sc is not None else float("inf")  # unscored: always kept
        allS = (g.all_gather(S.to(self._cdev)).cpu() if self._cdev.type == "cuda"
                else _host_gather(g, S)).view(g.size, R, K)
        self.stats["score_exchanges"] = self.stats.get("score_exchanges", 0) + 1
        keep = {}  # (origin, rid) -> [per row: set of this shard's winning positions]
        shard_of = torch.arange(g.size).view(-1, 1).expand(g.size, K).reshape(-1)
        pos_of = torch.arange(K).view(1, -1).expand(g.size, K).reshape(-1)
        for o, rid, nq, k in layout:
            base = row0[(o, rid)]
            cand = allS[:, base:base + nq, :].clone()  # [W, nq, K]
            cand[o] = float("-inf")  # the origin's own shard is merged at the origin
            flat = cand.permute(1, 0, 2).reshape(nq, g.size * K)
            order = torch.sort(-flat, dim=1, stable=True).indices[:, :k]
            rows = []
            for qi in range(nq):
                idx = order[qi]
                ok = flat[qi, idx] > float("-inf")
                sel = idx[ok & (shard_of[idx] == self.rank)]
                rows.append(set(pos_of[sel].tolist()))
            keep[(o, rid)] = rows
        sent = pruned = 0
        out = {}
        for src, res in results.items():
            new = []
            for rid, ok, val in res:
                rows = keep.get((src, rid))
                if rows is not None and ok and isinstance(val, list):
                    kept = [[h for j, h in enumerate(hits) if qi < len(rows) and j in rows[qi]]
                            for qi, hits in enumerate(val)]
                    n_all = sum(len(h) for h in val)
                    n_kept = sum(len(h) for h in kept)
                    sent += n_kept
                    pruned += n_all - n_kept
                    val = kept
                new.append((rid, ok, val))
            out[src] = new
        self.stats["hits_sent"] = self.stats.get("hits_sent", 0) + sent
        self.stats["hits_pruned"] = self.stats.get("hits_pruned", 0) + pruned
        return out


def _own_group(group):
    """A private communicator over the same ranks (collective: every replica constructs its transport):
    the round thread's collectives must never interleave with other threads' on a shared group.  The
    one-shot IPC exchange attached to ``group`` (if any) comes along: its buffers are this transport's."""
    import torch.distributed as dist

    from ..parallel.comm import Group

    if getattr(group, "pg", None) is None or not dist.is_initialized():
        return group
    own = Group(list(group.ranks), pg=dist.new_group(list(group.ranks)))
    own.custom_ar = getattr(group, "custom_ar", None)
    return own


def _loads(b: bytes):
    """A peer's pickled batch (the replicas' own process group); garbage from a timed-out device
    exchange reads as an empty batch -- that round is reported missing on the failing rank."""
    if not b:
        return []
    try:
        return pickle.loads(b)
    except Exception:
        return []


def _host_gather(g, t: torch.Tensor) -> torch.Tensor:
    """[...] host tensor -> [size, ...] over the group's (gloo) process group."""
    import torch.distributed as dist

    src = t.contiguous().view(-1)
    out = torch.empty(g.size * src.numel(), dtype=t.dtype)
    dist.all_gather_into_tensor(out, src, group=g.pg)
    return out.view(g.size, *t.shape)


def _host_all_to_all(g, t: torch.Tensor) -> torch.Tensor:
    import torch.distributed as dist

    out = torch.empty_like(t)
    dist.all_to_all_single(out.view(-1), t.contiguous().view(-1), group=g.pg)
    return out


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
