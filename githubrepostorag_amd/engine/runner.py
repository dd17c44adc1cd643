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

import contextlib
import dataclasses
import logging
import os
import queue
import threading
import time

import torch

from ..utils.gpu_guard import set_device_of
from .llm_engine import LLMEngine
from .scheduler import INTERACTIVE_PRIORITY
from .sequence import Completion, SamplingParams

log = logging.getLogger(__name__)


class GenerationHandle:
    def __init__(self, runner: "EngineRunner", req_id: str):
        self.runner = runner
        self.req_id = req_id
        self.done = threading.Event()
        self.result: Completion | None = None
        self.error: BaseException | None = None
        self._callbacks: list = []
        self._cb_lock = threading.Lock()
        self.bulk = False  # submitted as bulk (non-interactive) work: counted in the runner's _bulk_live

    def add_done_callback(self, fn) -> None:
        """fn(handle) once the request completes or fails (at once if it already has), on the thread
        that completes it: keep it short (an enqueue), it runs on the engine / streamer thread."""
        with self._cb_lock:
            if not self.done.is_set():
                self._callbacks.append(fn)
                return
        fn(self)

    def _finish(self) -> None:
        with self._cb_lock:
            first = not self.done.is_set()
            self.done.set()
            cbs, self._callbacks = self._callbacks, []
        if first and self.bulk:
            self.runner._bulk_finished()
        for fn in cbs:
            try:
                fn(self)
            except Exception:
                log.exception("generation done-callback failed")

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
    # arrival-aware decode window.  A hipGraph replay of K decode steps cannot be cut short, so a prompt
    # submitted during one waits for the rest of it (up to 8 steps: ~220 ms at 1024 live rows) before its
    # prefill.  GRAG_ARRIVAL_WINDOW:
    #   "auto" (default): paced by the arrival rate -- while arrivals keep coming (one within the last two
    #          mean gaps or PACE_HOLD_S, whichever is longer), a replay lasts at most half the mean gap between
    #          arrival events (EWMA; submits within 2 ms are one event), at least one step: an arrival waits
    #          ~1/4 gap on average instead of half a window.  No arrivals -> full windows.  (The hold: Poisson
    #          arrivals leave a two-gap quiet spell about one time in seven, and a full 8-step window of a
    #          ~340-row ingest batch then ran ~97 ms with the next queries waiting behind it -- the concurrent
    #          ingest trace, bench.py GRAG_DUMP_TRACE.)
    #   N > 0: fixed cap of N steps while requests keep arriving (one within ARRIVAL_RECENT_S);
    #   0:     off (full windows).  profiles/ab_arrival_window_r2.txt: fixed N = 2 on the agent phase
    #          cost 4-6 % jobs/s; the paced form is measured in docs/STATUS.md (round 4).
    ARRIVAL_RECENT_S = 0.05
    PACE_HOLD_S = float(os.environ.get("GRAG_PACE_HOLD_S", "0.5"))
    BULK_RECENT_S = 5.0
    # a paced replay lasts at most this fraction of the mean gap between arrival events
    PACE_FRAC = float(os.environ.get("GRAG_PACE_FRAC", "0.5"))
    _AW = os.environ.get("GRAG_ARRIVAL_WINDOW", "auto")
    ARRIVAL_WINDOW = -1 if _AW == "auto" else int(_AW)
    MAX_WINDOW = 8
    # prefill token budget per step while interactive arrivals keep coming (0: the engine's own
    # max_num_batched_tokens): a burst of prompts is prefilled over a few steps, first come first, so the
    # first of them do not wait for the whole burst's prefill (a decode replay of K steps is the other
    # wait an arrival sees: paced by _window)
    INTERACTIVE_PREFILL = int(os.environ.get("GRAG_INTERACTIVE_PREFILL", "0"))
    # of that budget, the tokens bulk work (ingest: submitted with interactive=False) may take per step while
    # interactive arrivals keep coming: the step an arrival waits for and the step carrying its prompt stay
    # short; 0 = no separate cap
    BULK_PREFILL = int(os.environ.get("GRAG_BULK_PREFILL", "512"))

    def __init__(self, engine: LLMEngine, idle_sleep: float = 0.0005, watchdog_s: float = 120.0,
                 on_health=None, tp=None, start: bool = True, interactive_prefill: int | None = None,
                 bulk_prefill: int | None = None):
        self.engine = engine
        self.interactive_prefill = self.INTERACTIVE_PREFILL if interactive_prefill is None else interactive_prefill
        self.bulk_prefill = self.BULK_PREFILL if bulk_prefill is None else bulk_prefill
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
        self._step_failed: BaseException | None = None  # TP: reported in the next control all-reduce
        self._ar_failed = False
        self._expecting = 0  # admission hints in flight (arrival())
        self._gap = None      # EWMA of the gap between arrival events (s)
        self._last_bulk = -1e9  # last submit of bulk (non-interactive) work: the pacing hold applies beside it
        self._bulk_live = 0     # bulk requests submitted and not finished (the hold also applies while > 0)
        self._last_event = -1e9
        self._step_s = None   # EWMA of one decode step's time (s), from the replays
        self.ctrl_stats = {"iterations": 0, "bytes": 0, "payloads": 0}
        self._notes: list = []  # streamed tokens / completions of the current step (engine thread)
        self._stream_q: queue.SimpleQueue = queue.SimpleQueue()
        self._streamer = threading.Thread(target=self._stream_loop, name="grag-stream", daemon=True)
        if start:
            self._streamer.start()
        self._thread = threading.Thread(target=self._loop if self.leader else self.follow, name="grag-engine",
                                        daemon=True)
        if start:
            self._thread.start()
        self._wd = None
        if watchdog_s and watchdog_s > 0 and self.leader:
            self._wd = threading.Thread(target=self._watchdog, name="grag-engine-watchdog", daemon=True)
            self._wd.start()

    # ------------------------------------------------------------------ API
    def submit(self, prompt, params: SamplingParams | None = None, on_token=None,
               interactive: bool = True) -> GenerationHandle:
        """``interactive``: someone waits for this request's first token (an agent call, an API request);
        batch work (ingest) passes False and does not pace the arrival-aware decode window."""
        import uuid

        rid = uuid.uuid4().hex
        h = GenerationHandle(self, rid)
        if interactive:  # someone waits for it: ahead of bulk work in admission and in each step's budget
            p = params if params is not None else SamplingParams()
            if p.priority < INTERACTIVE_PRIORITY:
                params = dataclasses.replace(p, priority=INTERACTIVE_PRIORITY)
        with self._cv:
            self._handles[rid] = h
            self._pending.append((rid, prompt, params, on_token))
            if not interactive:
                self._last_bulk = time.monotonic()
                self._bulk_live += 1
                h.bulk = True
            if interactive:
                now = time.monotonic()
                self._last_submit = now
                if now - self._last_event > 0.002:  # a new arrival event (a burst of submits is one)
                    if self._last_event > 0:
                        g = min(now - self._last_event, 5.0)
                        self._gap = g if self._gap is None else 0.8 * self._gap + 0.2 * g
                    self._last_event = now
            self._cv.notify()
        return h

    @contextlib.contextmanager
    def arrival(self):
        """Admission hint: the caller will submit a prompt at the end of this block (a RAG query between
        its retrieval and its generation).  While any hint is open, decode replays run ONE step each, so
        the prompt's prefill starts about one decode step after it is submitted instead of after a whole
        multi-step window — the serving-loop form of the headline bench's admission policy (bench.py
        ``--arrival-cap``).  Under TP the leader's window is broadcast, so followers replay alike."""
        with self._cv:
            self._expecting += 1
        try:
            yield self
        finally:
            with self._cv:
                self._expecting -= 1
                self._cv.notify()

    def _window(self) -> int | None:
        if self._expecting > 0:
            return 1
        if self.ARRIVAL_WINDOW == 0:
            return None
        now = time.monotonic()
        if self.ARRIVAL_WINDOW > 0:
            return self.ARRIVAL_WINDOW if now - self._last_submit < self.ARRIVAL_RECENT_S else None
        g, d = self._gap, self._step_s
        if g is None or d is None or now - self._last_event > max(2 * g, self._hold(now)):
            return None
        return max(1, min(self.MAX_WINDOW, int(self.PACE_FRAC * g / d)))

    def _prefill_budget(self) -> tuple[int | None, int | None]:
        """This step's (prefill token cap, bulk share of it): the interactive budget while arrivals are
        pending or paced (within two mean gaps of the last), and at most BULK_PREFILL tokens of bulk work
        for PACE_HOLD_S beyond that too -- the bulk cap (and the scheduler's interactive reserve) only holds
        back ingest, while the interactive cap also splits a saturating closed loop's prefill into smaller
        steps (measured: -10 % queries/s when it was held as long, profiles/pace_hold_ab_r6.json).  The hold applies
        only beside bulk work (_hold)."""
        if not self.interactive_prefill or self.tp is not None:
            return None, None
        g = self._gap
        if self._expecting > 0:
            return self.interactive_prefill, (self.bulk_prefill or None)
        if g is None:
            return None, None
        now = time.monotonic()
        quiet = now - self._last_event
        if quiet <= 2 * g:
            return self.interactive_prefill, (self.bulk_prefill or None)
        if quiet <= self._hold(now) and self.bulk_prefill:
            return None, self.bulk_prefill
        return None, None

    def _hold(self, now: float) -> float:
        """PACE_HOLD_S while bulk work shares the engine (a bulk request in flight, or a bulk submit within
        BULK_RECENT_S), else 0: with only interactive traffic (a saturating closed loop, whose arrivals come
        in bursts at window ends) the hold would shorten decode windows for nothing -- measured -7 %
        queries/s (profiles/pace_hold_ab_r6.json).  (Counting only recent SUBMITS dropped the hold in the
        middle of an ingest wave's long decode: concurrent-ingest TTFT p90 329 ms in the driver-form bench
        against 112 ms with the hold always on.)"""
        return self.PACE_HOLD_S if self._bulk_live > 0 or now - self._last_bulk < self.BULK_RECENT_S else 0.0

    def _bulk_finished(self) -> None:
        with self._cv:
            self._bulk_live = max(0, self._bulk_live - 1)

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
        self._stream_q.put(None)
        if self._streamer.is_alive():
            self._streamer.join(timeout=10)
        if self._wd is not None:
            self._wd.join(timeout=2)

    def stats(self) -> dict:
        sch = self.engine.sched
        return {"running": len(sch.running), "waiting": len(sch.waiting), "kv_usage": self.engine.kv.usage(),
                **self.engine.stats, **self.engine.kv.stats()}

    # ------------------------------------------------------------------ loop
    def _complete(self, finished) -> None:
        """Hand the results of the requests that finished in a step to their handles (the callback-free
        ones; streamed requests complete through their token callback)."""
        for seq in finished or ():
            if seq.on_token is not None:
                continue
            # popped whether or not a handle still waits: the watchdog / _fail_all clear the handles of
            # requests they abort, and those are reaped in a later step (their Sequence must not stay in
            # engine._seqs)
            self.engine.pop(seq.req_id)
            h = self._handles.pop(seq.req_id, None)
            if h is None:
                continue
            h.result = self.engine.completion(seq)
            h._finish()

    def _on_token_wrapper(self, user_cb):
        """Engine-thread side of a streamed request: the step's token deltas and the completion are noted
        and handed to the streamer thread in one batch after the step (``_flush_notes``), so the engine
        thread never runs consumer code (event-log appends, SSE wake-ups) per token."""
        def cb(seq, delta, finished):
            h = comp = None
            if finished:
                h = self._handles.pop(seq.req_id, None)
                self.engine.pop(seq.req_id)
                if h is not None:
                    comp = self.engine.completion(seq)
            if (user_cb is not None and delta) or h is not None:
                self._notes.append((user_cb if delta else None, delta, h, comp))
        return cb

    def _flush_notes(self) -> None:
        if self._notes:
            batch, self._notes = self._notes, []
            self._stream_q.put(batch)

    def _stream_loop(self) -> None:
        """Runs the streamed requests' token callbacks and completions, one engine step's batch at a time,
        in order; their asyncio wake-ups go out once per event loop per batch (utils/wakeups.py)."""
        from ..utils.wakeups import deferred

        while True:
            batch = self._stream_q.get()
            if batch is None:
                return
            with deferred():
                for cb, delta, h, comp in batch:
                    if cb is not None:
                        try:
                            cb(delta)
                        except Exception:  # a broken consumer never stops the stream of the others
                            log.exception("token callback failed")
                    if h is not None:
                        h.result = comp
                        h._finish()

    # ------------------------------------------------------------------ TP control plane
    # One iteration of a TP group = ONE int64 SUM all-reduce of a small header over the TP group (the
    # leader writes the control words, every rank adds its own status words; a SUM is a broadcast for
    # the leader's words and a count for the status words), plus, only when the leader has new requests
    # or aborts, one uint8 broadcast of their pickled payload.  A steady decode iteration therefore moves
    # 48 bytes and syncs the host once (round 2: a pickled broadcast_object_list AND an agree() MIN
    # all-reduce per iteration: two collectives, two host syncs).  Step status is reported in the NEXT
    # header, so every rank applies a failure (fail / drop every in-flight request, detach the one-shot
    # all-reduce, drop the decode graphs that captured it) at the same iteration.
    HDR_FLAGS, HDR_WINDOW, HDR_PAYLOAD, HDR_FAILED, HDR_AR_ERR, HDR_ITER = range(6)
    HDR_WORDS = 6
    FLAG_STOP, FLAG_STEP = 1, 2

    def _control(self, msg: dict | None) -> tuple[dict, int, int]:
        """Collective over the TP group.  ``msg`` (leader only): {"add", "abort", "stop", "step", "window"}.
        Returns (message, ranks whose previous step failed, ranks whose one-shot all-reduce timed out)."""
        import pickle

        import torch.distributed as dist

        dev = self.tp.ctrl_device(self.engine.device)
        h = torch.zeros(self.HDR_WORDS, dtype=torch.int64)
        payload = b""
        if self.leader:
            if msg["add"] or msg["abort"]:
                payload = pickle.dumps((msg["add"], msg["abort"]), protocol=pickle.HIGHEST_PROTOCOL)
            h[self.HDR_FLAGS] = (self.FLAG_STOP if msg["stop"] else 0) | (self.FLAG_STEP if msg["step"] else 0)
            h[self.HDR_WINDOW] = msg["window"] or 0
            h[self.HDR_PAYLOAD] = len(payload)
            h[self.HDR_ITER] = self.ctrl_stats["iterations"]
        h[self.HDR_FAILED] = 1 if self._step_failed is not None else 0
        h[self.HDR_AR_ERR] = 1 if self._ar_failed else 0
        t = h.to(dev)
        dist.all_reduce(t, group=self.tp.pg)
        h = t.tolist()
        self.ctrl_stats["iterations"] += 1
        self.ctrl_stats["bytes"] += 8 * self.HDR_WORDS
        adds, aborts = [], []
        n = h[self.HDR_PAYLOAD]
        if n:
            if self.leader:
                buf = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(dev)
            else:
                buf = torch.empty(n, dtype=torch.uint8, device=dev)
            dist.broadcast(buf, src=self.tp.ranks[0], group=self.tp.pg)
            self.ctrl_stats["bytes"] += n
            self.ctrl_stats["payloads"] += 1
            if not self.leader:
                adds, aborts = pickle.loads(buf.cpu().numpy().tobytes())
        flags = h[self.HDR_FLAGS]
        out = {"add": adds, "abort": aborts, "stop": bool(flags & self.FLAG_STOP),
               "step": bool(flags & self.FLAG_STEP), "window": h[self.HDR_WINDOW] or None}
        return out, h[self.HDR_FAILED], h[self.HDR_AR_ERR]

    def _apply_group_status(self, failed: int, ar_err: int) -> None:
        """Every rank, same iteration: a step failed somewhere in the group last iteration."""
        local = self._step_failed
        self._step_failed, self._ar_failed = None, False
        if not failed and not ar_err:
            return
        if ar_err and self.tp.detach_custom_ar():
            # the decode graphs captured the IPC kernel: recapture them on RCCL
            self.engine._graphs.clear()
            log.warning("one-shot all-reduce reported a peer timeout on %d rank(s): the TP group is back on RCCL",
                        ar_err)
        err = local or RuntimeError(f"{failed} TP rank(s) failed the previous engine step")
        if self.leader:
            self.last_error = err
            if local is None:
                self.num_faults += 1
            self._set_health(False)
            self._fail_inflight(err)
        else:
            self._drop_all()

    def follow(self) -> None:
        """Follower loop of a TP rank: mirror the leader's request stream and
        step in lockstep until the leader stops."""
        if self.engine.on_gpu:
            set_device_of(self.engine.device)

        def drop(seq, delta, finished):
            if finished:
                self.engine.pop(seq.req_id)

        while True:
            msg, failed, ar_err = self._control(None)
            self._apply_group_status(failed, ar_err)
            for rid, ids, params in msg["add"]:
                try:
                    self.engine.add_request(ids, params, req_id=rid, on_token=drop)
                except Exception:  # the leader failed the same request
                    pass
            for rid in msg["abort"]:
                self.engine.abort(rid)
            if msg["stop"]:
                break
            if not msg["step"]:
                continue
            try:
                self.engine.step(max_window=msg["window"])
            except Exception as e:
                log.exception("TP follower step failed")
                self.last_error = e
                self.num_faults += 1
                self._note_failure(e)

    def _note_failure(self, e: BaseException) -> None:
        from ..parallel.custom_ar import CommError

        self._step_failed = e
        self._ar_failed = self._ar_failed or isinstance(e, CommError)

    def _drop_all(self) -> None:
        """Follower side of a failed step: cancel every in-flight sequence
        (the leader fails the same requests in _fail_inflight)."""
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
            set_device_of(self.engine.device)
        while True:
            with self._cv:
                while (not self._stop and not self._pending and not self._aborts
                       and not self.engine.has_unfinished() and self._step_failed is None):
                    self._cv.wait(timeout=1.0)
                    if self.tp is not None:
                        break  # idle heartbeat: followers block in the control all-reduce meanwhile
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
                _, failed, ar_err = self._control({"add": adds, "abort": aborts, "stop": stop,
                                                   "step": will_step and not stop, "window": win})
                self._apply_group_status(failed, ar_err)
                pending = [(rid, ids, p, cb) for (rid, ids, p), (_, _, _, cb) in zip(adds, pending)]
            if stop:
                break
            if self.tp is not None and not will_step:
                continue
            for rid, prompt, params, cb in pending:
                try:
                    # a request nobody streams gets no per-token callback: the engine keeps it on its decode
                    # fast path (tokens appended per window, detokenised once at the end) and the handle is
                    # completed from the step's finished list below
                    self.engine.add_request(prompt, params, req_id=rid,
                                            on_token=None if cb is None else self._on_token_wrapper(cb))
                except Exception as e:  # bad request: fail just this handle
                    h = self._handles.pop(rid, None)
                    if h is not None:
                        h.error = e
                        h._finish()
            if self.tp is not None:  # after the adds, as the followers do
                for rid in aborts:
                    self.engine.abort(rid)
            self._step_t0 = time.monotonic()
            err = None
            try:
                st = self.engine.stats
                ds0, dt0 = st.get("decode_steps", 0), st.get("decode_s", 0.0)
                try:
                    pb, bb = self._prefill_budget()
                    self._complete(self.engine.step(max_window=win, prefill_budget=pb, bulk_budget=bb))
                finally:
                    self._flush_notes()
                n = st.get("decode_steps", 0) - ds0
                if n > 0:  # decode step time for the paced arrival window
                    per = (st.get("decode_s", 0.0) - dt0) / n
                    self._step_s = per if self._step_s is None else 0.7 * self._step_s + 0.3 * per
            except Exception as e:  # engine fault: fail every in-flight request, keep serving
                log.exception("engine step failed")
                err = e
            self._step_t0 = None
            if self.tp is not None:
                # under TP the outcome is applied by every rank at the next control all-reduce
                if err is not None:
                    self.last_error = err
                    self.num_faults += 1
                    self._note_failure(err)
                elif self.hung:
                    self.hung = False
                elif self._step_failed is None:
                    self._set_health(True)
                continue
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
                h._finish()

    def _abort_mirrored(self, rid: str) -> None:
        """Abort that every TP rank applies at the same iteration (queued for the
        next broadcast); a plain abort without TP."""
        if self.tp is not None:
            with self._cv:
                self._aborts.append(rid)
        else:
            self.engine.abort(rid)

    def _fail_inflight(self, err: BaseException) -> None:
        """Fail the requests already inside the engine (not the ones still queued for admission)."""
        with self._cv:
            rids = [r for r in list(self.engine._seqs) if r in self._handles]
            handles = [(r, self._handles.pop(r)) for r in rids]
        for rid in list(self.engine._seqs):
            self.engine.abort(rid)
        for rid, h in handles:
            h.error = err
            h._finish()
        try:
            for s in self.engine.sched.reap_cancelled():
                self.engine.pop(s.req_id)
        except Exception:
            pass

    def _fail_all(self, err: BaseException) -> None:
        with self._cv:
            handles, self._handles = self._handles, {}
        for rid, h in handles.items():
            self._abort_mirrored(rid)
            h.error = err
            h._finish()
        try:  # drop the aborted sequences from the scheduler
            self.engine.sched.reap_cancelled()
        except Exception:
            pass
