"""Coalesced cross-thread wake-ups of asyncio waiters.

A producer thread that wakes an event loop once per event (``loop.call_soon_threadsafe``) writes to the
loop's self-pipe every time -- a syscall that releases the GIL, after which the producer waits up to a
switch interval to get it back.  The engine's token stream did that once per streamed token: at 1024
concurrent agent jobs the engine thread spent 232 of 647 s in decode post-processing
(profiles/agent_saturation_r4b.json).  Inside ``deferred()`` the wake-ups a thread requests are
collected and issued at exit as ONE ``call_soon_threadsafe`` per loop.
"""
from __future__ import annotations

import contextlib
import threading

_tls = threading.local()


def _set_all(events) -> None:
    for ev in events:
        ev.set()


def wake(loop, ev) -> None:
    """Set asyncio event ``ev`` on ``loop`` from any thread (deferred inside ``deferred()``)."""
    pend = getattr(_tls, "pending", None)
    if pend is not None:
        pend.setdefault(loop, set()).add(ev)
        return
    try:
        loop.call_soon_threadsafe(ev.set)
    except RuntimeError:  # loop closed
        pass


@contextlib.contextmanager
def deferred():
    """Collect this thread's wake-ups; issue them, one call per event loop, when the block ends."""
    if getattr(_tls, "pending", None) is not None:  # nested: the outer block flushes
        yield
        return
    _tls.pending = {}
    try:
        yield
    finally:
        pend, _tls.pending = _tls.pending, None
        for loop, evs in pend.items():
            try:
                loop.call_soon_threadsafe(_set_all, list(evs))
            except RuntimeError:
                pass
