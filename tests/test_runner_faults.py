"""Fault injection for the engine loop: a step that raises fails
the in-flight requests and the loop keeps serving; a step that hangs past the
watchdog marks the engine unhealthy and releases every waiter at once; the
engine is healthy again once a step completes."""
import threading
import time

import pytest

from githubrepostorag_amd.engine.runner import EngineRunner
from githubrepostorag_amd.engine.sequence import Completion


class _Sched:
    def __init__(self):
        self.running, self.waiting = [], []

    def reap_cancelled(self):
        return []


class FakeEngine:
    """Minimal engine: each request finishes after one step with a fixed text;
    ``mode`` injects faults into the next step."""

    on_gpu = False

    def __init__(self):
        self.sched = _Sched()
        self.reqs = {}
        self.mode = "ok"
        self.release = threading.Event()
        self.stats = {}
        self.popped = []

    def add_request(self, prompt, params, req_id, on_token):
        self.reqs[req_id] = on_token

    def has_unfinished(self):
        return bool(self.reqs)

    def abort(self, rid):
        pass

    def pop(self, rid):
        self.popped.append(rid)
        return None

    def completion(self, seq):
        return Completion(seq.req_id, "done", [1], "length", 1, 0.0, 0.0)

    def step(self, max_window=None, prefill_budget=None, bulk_budget=None):
        if self.mode == "raise":
            self.mode = "ok"
            self.reqs.clear()
            raise RuntimeError("injected kernel fault")
        if self.mode == "hang":
            self.release.wait(10)
            self.mode = "ok"
        reqs, self.reqs = self.reqs, {}
        finished = []
        for rid, cb in reqs.items():  # streamed requests finish through their callback, the rest are returned
            seq = type("S", (), {"req_id": rid, "on_token": cb})()
            if cb is not None:
                cb(seq, "done", True)
            else:
                finished.append(seq)
        return finished


def test_step_exception_fails_requests_then_recovers():
    eng = FakeEngine()
    eng.mode = "raise"
    r = EngineRunner(eng, watchdog_s=0)
    try:
        with pytest.raises(RuntimeError, match="injected"):
            r.generate("p", timeout=5)
        assert not r.healthy and r.num_faults == 1
        assert r.generate("p", timeout=5).text == "done"
        assert r.healthy
    finally:
        r.shutdown()


def test_watchdog_releases_waiters_on_hung_step():
    eng = FakeEngine()
    eng.mode = "hang"
    health = []
    r = EngineRunner(eng, watchdog_s=0.4, on_health=health.append)
    try:
        t0 = time.monotonic()
        with pytest.raises(TimeoutError, match="watchdog"):
            r.generate("p", timeout=8)
        assert time.monotonic() - t0 < 4  # released by the watchdog, not the client timeout
        assert r.hung and not r.healthy and health == [False]
        eng.release.set()  # the stuck step finally returns
        assert r.generate("p", timeout=5).text == "done"
        assert r.healthy and not r.hung and health == [False, True]
    finally:
        eng.release.set()
        r.shutdown()


def test_watchdog_reaped_request_is_popped_when_the_step_returns():
    """A callback-free request the watchdog failed (its handle dropped) finishes in the stuck step once it
    returns: the runner still pops it from the engine (else its Sequence would stay in engine._seqs)."""
    eng = FakeEngine()
    eng.mode = "hang"
    r = EngineRunner(eng, watchdog_s=0.4)
    try:
        h = r.submit("p")
        with pytest.raises(TimeoutError, match="watchdog"):
            h.wait(8)
        eng.release.set()
        t0 = time.monotonic()
        while h.req_id not in eng.popped and time.monotonic() - t0 < 5:
            time.sleep(0.01)
        assert h.req_id in eng.popped
    finally:
        eng.release.set()
        r.shutdown()


def test_arrival_paced_window():
    """GRAG_ARRIVAL_WINDOW=auto (engine/runner.py _window): while interactive arrivals keep coming, a decode
    replay lasts at most half the mean gap between arrival events; batch submits (ingest) do not pace it;
    no recent arrival -> full windows; an open arrival() hint -> one step."""
    eng = FakeEngine()
    r = EngineRunner(eng, watchdog_s=0, start=False)
    assert r.ARRIVAL_WINDOW == -1  # auto is the default
    assert r._window() is None  # nothing measured yet
    r._step_s = 0.010  # 10 ms decode steps
    for _ in range(6):  # arrival events every 60 ms (each a burst of 4 submits)
        for _ in range(4):
            r.submit("q")
        time.sleep(0.06)
    assert r._gap is not None and 0.05 < r._gap < 0.2, r._gap
    w = r._window()
    assert w == max(1, min(8, int(0.5 * r._gap / 0.010))), (w, r._gap)
    assert 2 <= w <= 8
    with r.arrival():
        assert r._window() == 1
    r._last_event -= 10.0  # long quiet: full windows again
    assert r._window() is None
    g = r._gap
    for _ in range(3):
        r.submit("ingest prompt", interactive=False)
        time.sleep(0.01)
    assert r._gap == g and r._window() is None  # batch work does not pace the window


def test_streamed_tokens_batched_off_the_engine_thread():
    """Streamed requests: the engine thread only notes (callback, delta) per token; the streamer thread runs
    the callbacks in order, one engine step's batch at a time, and their event-loop wake-ups are coalesced
    to one call per loop per batch (utils/wakeups.py)."""
    import asyncio

    from githubrepostorag_amd.service.events import EventLog

    log = EventLog()
    loop = asyncio.new_event_loop()
    calls = []
    real = loop.call_soon_threadsafe

    def counting(cb, *a):
        calls.append(cb)
        return real(cb, *a)

    loop.call_soon_threadsafe = counting
    ev = asyncio.Event()
    log._waiters["job"].append((loop, ev))
    from githubrepostorag_amd.utils.wakeups import deferred

    with deferred():
        for i in range(50):
            log.emit_sync("job", "token", {"i": i})
    assert len(calls) == 1  # one wake-up for the whole batch
    log.emit_sync("job", "token", {"i": 50})
    assert len(calls) == 2  # outside a batch: one per event
    assert [e["data"]["i"] for e in log.events("job")] == list(range(51))
    loop.close()

    seen = []
    eng = FakeEngine()
    r = EngineRunner(eng, watchdog_s=0)
    try:
        h = r.submit("q", on_token=lambda d: seen.append((threading.current_thread().name, d)))
        # the fake engine streams one delta then finishes through the callback
        assert h.wait(5).text == "done"
    finally:
        r.shutdown()
    assert seen and all(name == "grag-stream" for name, _ in seen)
