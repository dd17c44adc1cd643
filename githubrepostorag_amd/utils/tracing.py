"""Per-request tracing: nested timed spans with attributes.

The reference has no tracing (only Prometheus histograms and the
agent's ``debug.turns`` breadcrumbs).  A ``Trace`` travels with one RAG job
(agent RunContext) and records every stage — plan / retrieve / search /
judge / rewrite / synthesize and each LLM call with its queue-to-first-token
and token count — so the worker can ship the span list in the job's
``timing`` event and feed per-span Prometheus histograms.

Spans are plain dicts: ``{"name", "start_ms" (from trace start), "dur_ms",
"depth", **attrs}``.  Thread-safe (ingest extractor waves record from worker
threads); nesting depth is tracked per thread.
"""
from __future__ import annotations

import threading
import time
import uuid
from contextlib import contextmanager


class Trace:
    def __init__(self, trace_id: str | None = None, observer=None):
        self.trace_id = trace_id or uuid.uuid4().hex[:16]
        self.t0 = time.perf_counter()
        self.spans: list[dict] = []
        self._lock = threading.Lock()
        self._tls = threading.local()
        self._observer = observer  # callable(name, seconds) -> None, e.g. a histogram

    @contextmanager
    def span(self, name: str, **attrs):
        depth = getattr(self._tls, "depth", 0)
        self._tls.depth = depth + 1
        start = time.perf_counter()
        rec = {"name": name, "start_ms": round((start - self.t0) * 1e3, 3), "depth": depth, **attrs}
        try:
            yield rec
        except BaseException as e:
            rec["error"] = type(e).__name__
            raise
        finally:
            dur = time.perf_counter() - start
            rec["dur_ms"] = round(dur * 1e3, 3)
            self._tls.depth = depth
            with self._lock:
                self.spans.append(rec)
            if self._observer is not None:
                try:
                    self._observer(name, dur)
                except Exception:
                    pass

    def add(self, name: str, seconds: float, **attrs) -> None:
        """Record an already-measured interval ending now."""
        end = time.perf_counter()
        rec = {"name": name, "start_ms": round((end - seconds - self.t0) * 1e3, 3),
               "dur_ms": round(seconds * 1e3, 3), "depth": getattr(self._tls, "depth", 0), **attrs}
        with self._lock:
            self.spans.append(rec)
        if self._observer is not None:
            try:
                self._observer(name, seconds)
            except Exception:
                pass

    def to_list(self) -> list[dict]:
        with self._lock:
            return sorted((dict(s) for s in self.spans), key=lambda s: s["start_ms"])

    def totals(self) -> dict:
        """Sum of span durations per name (ms)."""
        out: dict[str, float] = {}
        with self._lock:
            for s in self.spans:
                out[s["name"]] = round(out.get(s["name"], 0.0) + s["dur_ms"], 3)
        return out


class _NullTrace:
    trace_id = ""

    @contextmanager
    def span(self, name, **attrs):
        yield {}

    def add(self, *a, **k):
        pass

    def to_list(self):
        return []

    def totals(self):
        return {}


NULL_TRACE = _NullTrace()
