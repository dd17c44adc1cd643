"""Process-wide guard that serialises hipGraph capture with GPU work issued
from other threads.

The engine thread captures decode graphs lazily (a new batch bucket / split
plan / window size).  On HIP a synchronising call made by ANY thread while a
capture is open — a pageable copy, ``.cpu()``, a device sync, a fresh
``hipMalloc`` — invalidates that capture (hipErrorStreamCaptureInvalidated),
and the service runs retrieval / embedding / ingest on other threads against
the same device.  Captures are rare (warm-up, first use of a shape), so the
cost is one uncontended RLock acquire per retrieval / embedding call.

Use ``with gpu_guard():`` around a thread's GPU section that synchronises, or
decorate an entry point with ``@guarded``.  ``side_stream`` keeps such
latency-bound sections off the engine's stream.
"""
from __future__ import annotations

import contextlib
import functools
import threading

import torch

_LOCK = threading.RLock()
_TLS = threading.local()


def gpu_guard() -> threading.RLock:
    return _LOCK


def guarded(fn):
    @functools.wraps(fn)
    def wrapper(*a, **k):
        with _LOCK:
            return fn(*a, **k)

    return wrapper


def _thread_stream(device: torch.device) -> torch.cuda.Stream:
    streams = getattr(_TLS, "streams", None)
    if streams is None:
        streams = _TLS.streams = {}
    s = streams.get(device.index)
    if s is None:  # high priority: latency-bound retrieval preempts bulk engine work
        lo, hi = torch.cuda.Stream.priority_range()
        s = streams[device.index] = torch.cuda.Stream(device=device, priority=min(lo, hi))
    return s


@contextlib.contextmanager
def side_stream(device, wait_caller: bool = False):
    """Run a thread's latency-bound GPU work (query embedding, index search,
    graph traversal) on a per-thread, high-priority, non-blocking stream.

    The engine replays its decode graphs on the default stream; a retrieval
    issued there queues behind a whole multi-step decode window and its
    ``.cpu()`` waits for it.  On a side stream the search's sync only waits
    for the search.  Re-entrant: nested blocks on the same thread stay on the
    same stream.  ``wait_caller``: the block consumes device tensors made on
    the caller's stream, so the side stream first waits for that stream.  On
    exit the caller's stream is made to wait for the side work (no host
    sync), so results are safe to consume there."""
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
    prev.wait_stream(s)
