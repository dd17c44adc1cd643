"""Wall-clock stack sampler for one thread (diagnostics: where does the engine thread spend a step?).

A daemon thread wakes every ``interval`` seconds, reads the target thread's current frame from
``sys._current_frames()`` and counts its innermost ``depth`` frames (file:line function).  Time the
target spends blocked in C code (a GPU sync, a GIL wait) is attributed to the Python line that called
into it.  Overhead: one GIL acquisition per sample.
"""
from __future__ import annotations

import collections
import os
import sys
import threading
import time


class StackSampler:
    def __init__(self, thread_id: int | None = None, interval: float = 0.001, depth: int = 3,
                 all_threads: bool = False):
        self.tid = thread_id if thread_id is not None else threading.get_ident()
        self.all_threads = all_threads
        self.other: collections.Counter = collections.Counter()  # (thread name, frames...) of the other threads
        self.interval = interval
        self.depth = depth
        self.counts: collections.Counter = collections.Counter()
        self.samples = 0
        self._stop = threading.Event()
        self._th: threading.Thread | None = None

    def _key(self, frame) -> tuple:
        out = []
        while frame is not None and len(out) < self.depth:
            co = frame.f_code
            out.append(f"{os.path.basename(co.co_filename)}:{frame.f_lineno} {co.co_name}")
            frame = frame.f_back
        return tuple(out)

    def _run(self):
        me = threading.get_ident()
        names = {}
        while not self._stop.is_set():
            frames = sys._current_frames()
            f = frames.get(self.tid)
            if f is not None:
                self.counts[self._key(f)] += 1
                self.samples += 1
            if self.all_threads:
                for tid, fr in frames.items():
                    if tid in (me, self.tid):
                        continue
                    if tid not in names:
                        names[tid] = next((t.name for t in threading.enumerate() if t.ident == tid), str(tid))
                    self.other[(names[tid],) + self._key(fr)] += 1
            time.sleep(self.interval)

    def start(self) -> "StackSampler":
        self._th = threading.Thread(target=self._run, name="stack-sampler", daemon=True)
        self._th.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._th is not None:
            self._th.join()

    def top(self, n: int = 25) -> list[tuple[float, str]]:
        """(share of samples, 'innermost <- caller <- ...') for the n most frequent stacks."""
        tot = max(1, self.samples)
        return [(round(c / tot, 4), " <- ".join(k)) for k, c in self.counts.most_common(n)]

    def top_other(self, n: int = 25) -> list[tuple[float, str]]:
        """The other threads' most frequent stacks, as shares of the target thread's sample count."""
        tot = max(1, self.samples)
        return [(round(c / tot, 4), f"[{k[0]}] " + " <- ".join(k[1:])) for k, c in self.other.most_common(n)]
