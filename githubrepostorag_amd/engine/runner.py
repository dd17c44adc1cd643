"""Background engine loop.

Many agent jobs (the reference worker runs ``max_jobs=10`` concurrently,
worker.py:182-187) and ingest extractor waves submit generations from their
own threads; one loop thread owns the GPU engine and steps it whenever work
is queued, so all of them share continuous batches.  ``generate`` blocks the
caller (agent threads), ``submit`` returns a handle with a per-token
callback (SSE token streaming) and supports cancellation.

Tensor parallelism (replicated scheduling): every rank of a TP group runs the
same engine.  The leader (TP rank 0) owns the request queue; at the top of
every loop iteration it broadcasts the iteration's new requests (token ids +
sampling params), aborts and the stop flag over the TP group, and every rank
applies them and steps.  The scheduler is deterministic given the same
request stream, so all ranks form the same batches and meet in the same
collectives; followers only drop their outputs.  ``follow()`` is the
followers' loop (no API server on those ranks).

Failure handling (SURVEY §5.3 "engine watchdog"): an exception inside a step
fails every in-flight request and the loop keeps serving; a step that runs
longer than ``watchdog_s`` (a hung kernel, a wedged collective) is detected by
a separate watchdog thread, which marks the engine unhealthy (/health -> 503,
``grag_engine_healthy`` 0) and fails the waiting requests at once instead of
letting every client hang until its own timeout.  If the step eventually
returns, the engine is marked healthy again.
"""
from __future__ import annotations

import logging
import os
import threading
import time

import torch

from .llm_engine import LLMEngine
from .sequence import Completion, SamplingParams

log = logging.getLogger(__name__)


class GenerationHandle:
    def __init__(self, runner: "EngineRunner", req_id: str):
        self.runner = runner
        self.req_id = req_id
        self.done = threading.Event()
        self.result: Completion | None = None
        self.error: BaseException | None = None

    def wait(self, timeout: float | None = None) -> Completion:
        if not self.done.wait(timeout):
            self.runner.abort(self.req_id)
            self.done.wait(5.0)
            raise TimeoutError(f"generation {self.req_id} timed out after {timeout}s")
        if self.error is not None:
            raise self.error
        return self.result

    def cancel(self) -> None:
        self.runner.abort(self.req_id)


class EngineRunner:
    # arrival-aware decode window (GRAG_ARRIVAL_WINDOW=N): while requests keep arriving (one submitted
    # within the last ARRIVAL_RECENT_S) a decode replay runs at most N steps, so a new prompt waits ~N
    # decode steps before its prefill instead of a whole 8-step window.  Off by default: on the bench's
    # agent e2e phase (64 concurrent 3-round jobs of short calls) N = 2 measured 11.1-11.9 vs 11.8-12.4
    # jobs/s and p50 first-answer-token 4.26-4.59 vs 4.01-4.28 s (same box, profiles/ab_arrival_window_r2.txt):
    # a chain of short calls pays for the extra replays more than it gains on admission
    ARRIVAL_RECENT_S = 0.05
    ARRIVAL_WINDOW = int(os.environ.get("GRAG_ARRIVAL_WINDOW", "0"))

    def __init__(self, engine: LLMEngine, idle_sleep: float = 0.0005, watchdog_s: float = 120.0,
                 on_health=None, tp=None, start: bool = True):
        self.engine = engine
        self._last_submit = -1e9
        self.tp = tp if tp is not None and not tp.trivial else None
        self.leader = self.tp is None or self.tp.rank == 0
        self._aborts: list[str] = []
        self.idle_sleep = idle_sleep
        self.watchdog_s = watchdog_s
        self._on_health = on_health  # callable(bool), e.g. a Prometheus gauge setter
        self._cv = threading.Condition()
        self._stop = False
        self._handles: dict[str, GenerationHandle] = {}
        self._pending: list[tuple] = []
        self.last_error: BaseException | None = None
        self.healthy = True
        self.hung = False
        self.num_faults = 0
        self._step_t0: float | None = None
        self._thread = threading.Thread(target=self._loop if self.leader else self.follow, name="grag-engine",
                                        daemon=True)
        if start:
            self._thread.start()
        self._wd = None
        if watchdog_s and watchdog_s > 0 and self.leader:
            self._wd = threading.Thread(target=self._watchdog, name="grag-engine-watchdog", daemon=True)
            self._wd.start()

    # ------------------------------------------------------------------ API
    def submit(self, prompt, params: SamplingParams | None = None, on_token=None) -> GenerationHandle:
        import uuid

        rid = uuid.uuid4().hex
        h = GenerationHandle(self, rid)
        with self._cv:
            self._handles[rid] = h
            self._pending.append((rid, prompt, params, on_token))
            self._last_submit = time.monotonic()
            self._cv.notify()
        return h

    def _window(self) -> int | None:
        if self.ARRIVAL_WINDOW <= 0:
            return None
        return self.ARRIVAL_WINDOW if time.monotonic() - self._last_submit < self.ARRIVAL_RECENT_S else None

    def generate(self, prompt, params: SamplingParams | None = None, on_token=None,
                 timeout: float | None = None) -> Completion:
        return self.submit(prompt, params, on_token).wait(timeout)

    def abort(self, req_id: str) -> None:
        with self._cv:
            if self.tp is not None:  # applied on every rank at the same iteration
                self._aborts.append(req_id)
            else:
                self.engine.abort(req_id)
            self._cv.notify()

    def shutdown(self) -> None:
        with self._cv:
            self._stop = True
            self._cv.notify()
        self._thread.join(timeout=10)
        if self._wd is not None:
            self._wd.join(timeout=2)

    def stats(self) -> dict:
        sch = self.engine.sched
        return {"running": len(sch.running), "waiting": len(sch.waiting), "kv_usage": self.engine.kv.usage(),
                **self.engine.stats, **self.engine.kv.stats()}

    # ------------------------------------------------------------------ loop
    def _on_token_wrapper(self, user_cb):
        def cb(seq, delta, finished):
            if user_cb is not None and delta:
                user_cb(delta)
            if finished:
                h = self._handles.pop(seq.req_id, None)
                self.engine.pop(seq.req_id)
                if h is not None:
                    h.result = self.engine.completion(seq)
                    h.done.set()
        return cb

    # ------------------------------------------------------------------ TP
    def _bcast(self, msg):
        import torch.distributed as dist

        obj = [msg]
        dist.broadcast_object_list(obj, src=self.tp.ranks[0], group=self.tp.pg)
        return obj[0]

    def follow(self) -> None:
        """Follower loop of a TP rank: mirror the leader's request stream and
        step in lockstep until the leader stops."""
        if self.engine.on_gpu:
            torch.cuda.set_device(self.engine.device)

        def drop(seq, delta, finished):
            if finished:
                self.engine.pop(seq.req_id)

        while True:
            msg = self._bcast(None)
            for rid, ids, params in msg["add"]:
                try:
                    self.engine.add_request(ids, params, req_id=rid, on_token=drop)
                except Exception:  # the leader failed the same request
                    pass
            for rid in msg["abort"]:
                self.engine.abort(rid)
            if msg["stop"]:
                break
            if not msg.get("step", True):
                continue
            ok = True
            try:
                self.engine.step(max_window=msg.get("window"))
            except Exception as e:
                log.exception("TP follower step failed")
                self.last_error = e
                self.num_faults += 1
                ok = False
            # every rank learns whether the step succeeded everywhere, so all
            # ranks fail the same requests and stay in lockstep
            if not self.tp.agree(ok, self.engine.device):
                self._drop_all()

    def _drop_all(self) -> None:
        """Follower side of a failed step: cancel every in-flight sequence
        (the leader fails the same requests in _fail_all)."""
        for rid in list(self.engine._seqs):
            self.engine.abort(rid)
        try:
            for s in self.engine.sched.reap_cancelled():
                self.engine.pop(s.req_id)
        except Exception:
            pass

    def join(self, timeout: float | None = None) -> None:
        self._thread.join(timeout)

    def _loop(self):
        if self.engine.on_gpu:
            torch.cuda.set_device(self.engine.device)
        while True:
            with self._cv:
                while not self._stop and not self._pending and not self._aborts and not self.engine.has_unfinished():
                    self._cv.wait(timeout=1.0)
                    if self.tp is not None:
                        break  # idle heartbeat: followers block in the broadcast meanwhile
                stop = self._stop
                pending, self._pending = self._pending, []
                aborts, self._aborts = self._aborts, []
            will_step = bool(pending) or self.engine.has_unfinished()
            win = self._window()  # decided before the TP broadcast: every rank replays the same graph
            if self.tp is not None:
                adds = []
                for rid, prompt, params, cb in pending:
                    ids = self.engine.tok.encode(prompt) if isinstance(prompt, str) else list(prompt)
                    adds.append((rid, ids, params or SamplingParams()))
                self._bcast({"add": adds, "abort": aborts, "stop": stop, "step": will_step and not stop,
                             "window": win})
                pending = [(rid, ids, p, cb) for (rid, ids, p), (_, _, _, cb) in zip(adds, pending)]
            if stop:
                break
            if self.tp is not None and not will_step:
                continue
            for rid, prompt, params, cb in pending:
                try:
                    self.engine.add_request(prompt, params, req_id=rid, on_token=self._on_token_wrapper(cb))
                except Exception as e:  # bad request: fail just this handle
                    h = self._handles.pop(rid, None)
                    if h is not None:
                        h.error = e
                        h.done.set()
            if self.tp is not None:  # after the adds, as the followers do
                for rid in aborts:
                    self.engine.abort(rid)
            self._step_t0 = time.monotonic()
            err = None
            try:
                self.engine.step(max_window=win)
            except Exception as e:  # engine fault: fail every in-flight request, keep serving
                log.exception("engine step failed")
                err = e
            self._step_t0 = None
            if self.tp is not None and not self.tp.agree(err is None, self.engine.device) and err is None:
                err = RuntimeError("a TP follower rank failed this engine step")
            if err is None:
                if self.hung:
                    log.warning("engine step returned after the watchdog fired; marking healthy again")
                    self.hung = False
                    self.engine.sched.reap_cancelled()
                self._set_health(True)
            else:
                self.last_error = err
                self.num_faults += 1
                self._set_health(False)
                self._fail_all(err)
                time.sleep(0.05)

    def _set_health(self, ok: bool) -> None:
        if ok != self.healthy and self._on_health is not None:
            try:
                self._on_health(ok)
            except Exception:
                pass
        self.healthy = ok

    def _watchdog(self) -> None:
        period = min(1.0, self.watchdog_s / 4)
        while not self._stop:
            time.sleep(period)
            t0 = self._step_t0
            if t0 is None or self.hung or time.monotonic() - t0 < self.watchdog_s:
                continue
            err = TimeoutError(f"engine step exceeded the {self.watchdog_s:.0f}s watchdog")
            log.error("%s; failing in-flight requests", err)
            self.hung = True
            self.last_error = err
            self.num_faults += 1
            self._set_health(False)
            # only flag + release waiters here: the stuck loop thread still owns the engine
            with self._cv:
                handles, self._handles = self._handles, {}
            for rid, h in handles.items():
                self._abort_mirrored(rid)
                h.error = err
                h.done.set()

    def _abort_mirrored(self, rid: str) -> None:
        """Abort that every TP rank applies at the same iteration (queued for the
        next broadcast); a plain abort without TP."""
        if self.tp is not None:
            with self._cv:
                self._aborts.append(rid)
        else:
            self.engine.abort(rid)

    def _fail_all(self, err: BaseException) -> None:
        with self._cv:
            handles, self._handles = self._handles, {}
        for rid, h in handles.items():
            self._abort_mirrored(rid)
            h.error = err
            h.done.set()
        try:  # drop the aborted sequences from the scheduler
            self.engine.sched.reap_cancelled()
        except Exception:
            pass
