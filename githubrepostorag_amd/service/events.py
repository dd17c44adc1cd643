"""Per-job progress events and cancel flags.

Reference: ``ProgressBus`` / ``CancelFlags`` over Redis pub/sub
(rag_shared/bus.py:8-40).  Its pub/sub transport loses events published
before the SSE client subscribes and the stream loop delivers at most ~1
event per second (bus.py:21-27).  Here every job has an
append-only, replayable event log: a subscriber first replays everything the
job already emitted, then waits on a condition for new events (no polling
sleep), keep-alive pings go out only when idle, and the stream ends after the
``final`` event.  Producers may be asyncio code or agent threads
(``emit_threadsafe``).  The wire format is unchanged:
``data: {"event": E, "data": D}\\n\\n`` frames and ``: ping\\n\\n`` comments.
Across processes (one front door, N per-GPU replicas) the replicas forward
their events to the front door's log over the replica hub (service/cluster.py)
instead of Redis.
"""
from __future__ import annotations

import asyncio
import json
import threading
import time
from collections import defaultdict
from typing import AsyncIterator

from ..utils.wakeups import wake


class _JobLog:
    __slots__ = ("events", "cond", "created", "closed")

    def __init__(self):
        self.events: list[str] = []
        self.cond = threading.Condition()
        self.created = time.time()
        self.closed = False


class EventLog:
    TERMINAL = ("final",)

    def __init__(self, keep_seconds: float = 3600.0):
        self.keep = keep_seconds
        self._jobs: dict[str, _JobLog] = defaultdict(_JobLog)
        self._lock = threading.Lock()
        self._waiters: dict[str, list[tuple[asyncio.AbstractEventLoop, asyncio.Event]]] = defaultdict(list)

    def _log(self, job_id: str) -> _JobLog:
        with self._lock:
            return self._jobs[job_id]

    def emit_sync(self, job_id: str, event: str, data) -> None:
        payload = json.dumps({"event": event, "data": data}, ensure_ascii=False, default=str)
        lg = self._log(job_id)
        with lg.cond:
            lg.events.append(payload)
            if event in self.TERMINAL:
                lg.closed = True
            lg.cond.notify_all()
        with self._lock:
            waiters = list(self._waiters.get(job_id, []))
        for loop, ev in waiters:  # coalesced when the caller batches (utils/wakeups.deferred)
            wake(loop, ev)

    async def emit(self, job_id: str, event: str, data) -> None:
        self.emit_sync(job_id, event, data)

    # thread-safe alias used by agent threads
    emit_threadsafe = emit_sync

    def events(self, job_id: str) -> list[dict]:
        lg = self._log(job_id)
        with lg.cond:
            return [json.loads(e) for e in lg.events]

    def is_closed(self, job_id: str) -> bool:
        return self._log(job_id).closed

    async def stream(self, job_id: str, ping_seconds: float = 15.0) -> AsyncIterator[str]:
        loop = asyncio.get_running_loop()
        ev = asyncio.Event()
        with self._lock:
            self._waiters[job_id].append((loop, ev))
        lg = self._log(job_id)
        sent = 0
        try:
            while True:
                with lg.cond:
                    pending = lg.events[sent:]
                    closed = lg.closed
                    ev.clear()
                for p in pending:
                    yield f"data: {p}\n\n"
                sent += len(pending)
                if closed and sent >= len(lg.events):
                    return
                try:
                    await asyncio.wait_for(ev.wait(), timeout=ping_seconds)
                except asyncio.TimeoutError:
                    yield ": ping\n\n"
        finally:
            with self._lock:
                ws = self._waiters.get(job_id, [])
                if (loop, ev) in ws:
                    ws.remove((loop, ev))

    def gc(self) -> int:
        now = time.time()
        with self._lock:
            old = [j for j, lg in self._jobs.items() if lg.closed and now - lg.created > self.keep]
            for j in old:
                self._jobs.pop(j, None)
        return len(old)


class CancelFlags:
    """Cooperative cancel (bus.py:32-40: SET job:{id}:cancel EX 3600)."""

    def __init__(self, ttl: float = 3600.0):
        self.ttl = ttl
        self._flags: dict[str, float] = {}
        self._lock = threading.Lock()
        self._listeners: dict[str, list] = defaultdict(list)

    async def cancel(self, job_id: str) -> None:
        self.cancel_sync(job_id)

    def cancel_sync(self, job_id: str) -> None:
        with self._lock:
            self._flags[job_id] = time.time() + self.ttl
            ls = list(self._listeners.pop(job_id, []))
        for fn in ls:
            try:
                fn()
            except Exception:
                pass

    def is_cancelled_sync(self, job_id: str) -> bool:
        with self._lock:
            exp = self._flags.get(job_id)
            if exp is None:
                return False
            if exp < time.time():
                self._flags.pop(job_id, None)
                return False
            return True

    async def is_cancelled(self, job_id: str) -> bool:
        return self.is_cancelled_sync(job_id)

    def on_cancel(self, job_id: str, fn) -> None:
        """Register a callback fired when the job is cancelled (e.g. abort the
        job's in-flight LLM requests so cancel takes effect mid-decode)."""
        with self._lock:
            self._listeners[job_id].append(fn)
