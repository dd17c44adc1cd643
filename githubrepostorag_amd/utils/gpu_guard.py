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
decorate an entry point with ``@guarded``.
"""
from __future__ import annotations

import functools
import threading

_LOCK = threading.RLock()


def gpu_guard() -> threading.RLock:
    return _LOCK


def guarded(fn):
    @functools.wraps(fn)
    def wrapper(*a, **k):
        with _LOCK:
            return fn(*a, **k)

    return wrapper
