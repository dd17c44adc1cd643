"""Process-wide guard that serialises hipGraph capture with GPU work issued
from other threads.

The engine thread captures decode graphs lazily (a new batch bucket / split
plan / window size).  On HIP a synchronising call made by ANY thread while a
capture is open — a pageable copy, ``.cpu()``, a device sync, a fresh
``hipMalloc`` — invalidates that capture (hipErrorStreamCaptureInvalidated),
and the service runs retrieval / embedding / ingest on other threads against
the same device.  Captures are rare (warm-up, first use of a shape), so the
cost is one uncontended RLock acquire per retrieval / embedding call.

Captures hold the guard exclusively (``with gpu_guard():``); a thread's GPU
section that synchronises holds it shared (``with gpu_shared():`` or the
``@guarded`` decorator), so retrieval / embedding / ingest sections run
concurrently with each other and only wait while a capture is open.  ``side_stream`` keeps such
latency-bound sections off the engine's stream (its closing sync is a shared section too).  The
engine holds the guard shared for every step (its host reads sync while the embedder may capture a
query-bucket graph on a retrieval thread) and upgrades to exclusive for its own lazy captures.
"""
from __future__ import annotations

import contextlib
import os
import functools
import threading

import torch

class _CaptureGuard:
    """Shared/exclusive guard.  Capture holds it EXCLUSIVE; any thread section
    that may synchronise (a search's ``.cpu()``, an embedding batch, an upsert)
    holds it SHARED, so those sections run concurrently with each other and
    only wait while a capture is open.  Re-entrant per thread (a shared
    section inside the capturing thread's exclusive one is a no-op); a thread
    never upgrades shared -> exclusive (it would deadlock against itself)."""

    def __init__(self):
        self._cond = threading.Condition()
        self._readers = 0
        self._writer = None
        self._waiting = 0
        self._tls = threading.local()

    def _depth(self, kind):
        return getattr(self._tls, kind, 0)

    @contextlib.contextmanager
    def shared(self, urgent: bool = False):
        """``urgent``: enter while a capture is only WAITING (not running).  For a thread other shared
        holders depend on -- the shard-round thread: a job thread holds the guard while it waits for a round's
        answer, and that round must not queue behind a capture that waits for the job thread."""
        if self._depth("ex") or self._depth("sh"):
            self._tls.sh = self._depth("sh") + 1
            try:
                yield
            finally:
                self._tls.sh -= 1
            return
        with self._cond:
            while self._writer is not None or (self._waiting and not urgent):
                self._cond.wait()
            self._readers += 1
        self._tls.sh = 1
        try:
            yield
        finally:
            self._tls.sh = 0
            with self._cond:
                self._readers -= 1
                if self._readers == 0:
                    self._cond.notify_all()

    @contextlib.contextmanager
    def exclusive(self):
        if self._depth("ex"):
            self._tls.ex += 1
            try:
                yield
            finally:
                self._tls.ex -= 1
            return
        # a thread inside a shared section (the engine thread holds one for its whole step and captures
        # lazily inside it) gives its read hold up while it waits and captures, and takes it back after:
        # two upgrading threads then wait as plain writers instead of each holding the other's read count
        sh = self._depth("sh")
        me = threading.get_ident()
        with self._cond:
            if sh:
                self._readers -= 1
                if self._readers == 0:
                    self._cond.notify_all()
            self._waiting += 1
            while self._writer is not None or self._readers:
                self._cond.wait()
            self._waiting -= 1
            self._writer = me
        self._tls.ex, self._tls.sh = 1, 0
        try:
            yield
        finally:
            self._tls.ex = 0
            with self._cond:
                self._writer = None
                self._cond.notify_all()
                if sh:
                    while self._writer is not None or self._waiting:
                        self._cond.wait()
                    self._readers += 1
            self._tls.sh = sh


_GUARD = _CaptureGuard()


def gpu_guard():
    """Exclusive section (hipGraph capture): ``with gpu_guard(): ...``"""
    return _GUARD.exclusive()


def gpu_shared(urgent: bool = False):
    """Shared section (may synchronise; must not overlap a capture).  ``urgent``: see _CaptureGuard.shared."""
    return _GUARD.shared(urgent)


def guarded(fn):
    @functools.wraps(fn)
    def wrapper(*a, **k):
        with _GUARD.shared():
            return fn(*a, **k)

    return wrapper


_TLS = threading.local()


def _thread_stream(device: torch.device) -> torch.cuda.Stream:
    streams = getattr(_TLS, "streams", None)
    if streams is None:
        streams = _TLS.streams = {}
    s = streams.get(device.index)
    if s is None:  # high priority: latency-bound retrieval preempts bulk engine work
        lo, hi = torch.cuda.Stream.priority_range()
        prio = min(lo, hi) if os.environ.get("GRAG_SIDE_PRIORITY", "high") == "high" else 0
        s = streams[device.index] = torch.cuda.Stream(device=device, priority=prio)
    return s


@contextlib.contextmanager
def side_stream(device, wait_caller: bool = False, join: str = "sync"):
    """Run a thread's latency-bound GPU work (query embedding, index search,
    graph traversal) on a per-thread, high-priority, non-blocking stream.

    The engine replays its decode graphs on the default stream; a retrieval
    issued there queues behind a whole multi-step decode window and its
    ``.cpu()`` waits for it.  On a side stream the search's sync only waits
    for the search.  Re-entrant: nested blocks on the same thread stay on the
    same stream.  ``wait_caller``: the block consumes device tensors made on
    the caller's stream, so the side stream first waits for that stream.

    ``join`` (on exit): "sync" (default) waits on the host for the side
    stream alone (the wait releases the GIL), so results are complete for any
    stream or thread; "event" makes the caller's stream wait for the side work
    without a host sync.  "event" enqueues into the caller's stream, which for
    a retrieval thread is the default stream the engine keeps full: measured
    on ROCm, that enqueue blocked the retrieval thread ~12 ms per block with
    the GIL held, and the engine thread (needing the GIL to launch) left the
    GPU idle for the whole time (profiles/timeline_r2_*.txt)."""
    dev = torch.device(device)
    if dev.type != "cuda":
        yield None
        return
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    s = _thread_stream(dev)
    prev = torch.cuda.current_stream(dev)
    if prev == s:
        yield s
        return
    if wait_caller:
        s.wait_stream(prev)
    with torch.cuda.stream(s):
        yield s
    if join == "event":
        prev.wait_stream(s)
    else:
        with _GUARD.shared():  # a host sync: never while another thread's capture is open
            s.synchronize()


def set_device_of(dev) -> None:
    """torch.cuda.set_device for a device that may carry no index ("cuda" means the current device)."""
    d = torch.device(dev)
    if d.type == "cuda":
        torch.cuda.set_device(d.index if d.index is not None else torch.cuda.current_device())


@contextlib.contextmanager
def no_gc():
    """Cyclic GC off for the block (a hipGraph capture): a collection that runs in the capturing thread
    can free an OLD graph (e.g. a dropped engine's), and destroying a graph while a stream captures is
    an illegal call that aborts the process from the graph's destructor.  Collection resumes after."""
    import gc

    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()
