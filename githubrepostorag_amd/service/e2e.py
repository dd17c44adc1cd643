"""End-to-end serving measurement over real HTTP (SURVEY §6 metric
definitions): a uvicorn server on 127.0.0.1 in a
background thread serves ``service/api.py`` over a runtime, and an async
httpx client drives N concurrent jobs exactly as the UI does
(rest_api/src/app/static/index.html:215-224): ``POST /rag/jobs`` ->
``GET /rag/jobs/{id}/events`` (SSE) until the ``final`` event.

  TTFT    = POST issued -> first ``token`` SSE frame received by the client
            (reference: the first visible output is the final event,
            rag_worker/src/worker/worker.py:170, qwen_llm.py:149-151)
  jobs/s  = completed jobs / wall time of the run

The client runs in a child process by default (``client_process``): like the
reference's browser it is not part of the server, and hundreds of SSE streams
parsed in the server's interpreter would compete with the engine thread for
its GIL.  ``python -m githubrepostorag_amd.service.e2e --url U --questions F
--concurrency C --out O`` is that child.
"""
from __future__ import annotations

import asyncio
import json
import socket
import statistics
import sys
import threading
import time


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class ServerThread:
    """uvicorn in a daemon thread (its own event loop); ``url`` once started."""

    def __init__(self, app, port: int | None = None):
        import uvicorn

        self.port = port or _free_port()
        cfg = uvicorn.Config(app, host="127.0.0.1", port=self.port, log_level="warning", lifespan="on",
                             timeout_keep_alive=600)
        self.server = uvicorn.Server(cfg)
        self.thread = threading.Thread(target=self.server.run, name="e2e-uvicorn", daemon=True)

    @property
    def url(self) -> str:
        return f"http://127.0.0.1:{self.port}"

    def __enter__(self):
        self.thread.start()
        t0 = time.time()
        while not self.server.started:
            if not self.thread.is_alive() or time.time() - t0 > 120:
                raise RuntimeError("e2e: uvicorn did not start")
            time.sleep(0.01)
        return self

    def __exit__(self, *exc):
        self.server.should_exit = True
        self.thread.join(timeout=30)


async def _drive(url: str, questions: list[str], concurrency: int, timeout_s: float) -> list[dict]:
    import httpx

    sem = asyncio.Semaphore(concurrency)
    limits = httpx.Limits(max_connections=2 * concurrency + 8, max_keepalive_connections=2 * concurrency + 8)
    async with httpx.AsyncClient(base_url=url, timeout=timeout_s, limits=limits) as client:
        async def one(q: str) -> dict:
            async with sem:
                t0 = time.perf_counter()
                r = await client.post("/rag/jobs", json={"query": q})
                r.raise_for_status()
                jid = r.json()["job_id"]
                first = final = None
                err = degraded = False
                ntok = 0
                async with client.stream("GET", f"/rag/jobs/{jid}/events") as resp:
                    async for line in resp.aiter_lines():
                        if not line.startswith("data:"):
                            continue
                        ev = json.loads(line[5:])
                        now = time.perf_counter()
                        if ev.get("event") == "token":
                            ntok += 1
                            if first is None:
                                first = now
                        elif ev.get("event") == "retrieval":  # sharded index: a round missed a shard
                            degraded = bool((ev.get("data") or {}).get("degraded"))
                        elif ev.get("event") == "final":
                            final = now
                            err = bool((ev.get("data") or {}).get("error"))
                            break
                return {"t0": t0, "first_token": first, "final": final, "error": err, "tokens": ntok,
                        "degraded": degraded}

        done = [0]

        async def counted(q):
            try:
                return await one(q)
            finally:
                done[0] += 1

        async def progress():  # a line every 20 s: long sweeps stay visibly alive
            t_start = time.perf_counter()
            while True:
                await asyncio.sleep(20)
                print(f"[e2e] {done[0]}/{len(questions)} jobs at concurrency {concurrency}, "
                      f"{time.perf_counter() - t_start:.0f} s", file=sys.stderr, flush=True)

        tick = asyncio.ensure_future(progress())
        try:
            return await asyncio.gather(*[counted(q) for q in questions])
        finally:
            tick.cancel()


def _pct(xs: list[float], p: float) -> float | None:
    if not xs:
        return None
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(round(p * (len(xs) - 1))))]


def _drive_child(url: str, questions: list[str], concurrency: int, timeout_s: float) -> tuple[list[dict], float]:
    """_drive in a child process (no torch, no GPU): (per-job records with times relative to its start,
    wall seconds)."""
    import os
    import subprocess
    import sys
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        qf, of = os.path.join(d, "q.json"), os.path.join(d, "out.json")
        with open(qf, "w") as f:
            json.dump(questions, f)
        env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
        r = subprocess.run([sys.executable, "-m", "githubrepostorag_amd.service.e2e", "--url", url, "--questions", qf,
                            "--concurrency", str(concurrency), "--timeout", str(timeout_s), "--out", of],
                           env=env, timeout=timeout_s + 60)
        if r.returncode != 0:
            raise RuntimeError(f"e2e client exited with {r.returncode}")
        with open(of) as f:
            out = json.load(f)
    return out["records"], out["wall_s"]


def run_e2e(app, questions: list[str], concurrency: int, warmup: list[str] | None = None,
            timeout_s: float = 1800.0, sweep: list[tuple[list[str], int]] | None = None,
            client_process: bool = True, stats_fn=None) -> dict:
    """Serve ``app`` on localhost and push ``questions`` through the HTTP API at ``concurrency``.
    ``sweep``: further (questions, concurrency) runs on the same server, one after the other (a
    saturation curve); their summaries go to ``agent_saturation``."""
    with ServerThread(app) as srv:
        loop = None if client_process else asyncio.new_event_loop()

        def drive(qs, conc):
            if client_process:
                return _drive_child(srv.url, qs, conc, timeout_s)
            t0 = time.perf_counter()
            r = loop.run_until_complete(_drive(srv.url, qs, conc, timeout_s))
            return r, time.perf_counter() - t0

        def delta(a, b):  # numeric engine counters accumulated over one run (stats_fn: a dict snapshot)
            return {k: round(b[k] - a[k], 4) for k in b if isinstance(b.get(k), (int, float)) and k in a}

        try:
            if warmup:
                drive(warmup, concurrency)
            s0 = stats_fn() if stats_fn else None
            res, wall = drive(questions, concurrency)
            eng_main = delta(s0, stats_fn()) if stats_fn else None
            curve = []
            for qs, conc in sweep or []:
                s0 = stats_fn() if stats_fn else None
                r, w = drive(qs, conc)
                curve.append(dict(concurrency=conc, **_summary(r, w)))
                if stats_fn:
                    curve[-1]["engine"] = delta(s0, stats_fn())
        finally:
            if loop is not None:
                loop.close()
    out = _summary(res, wall)
    if eng_main is not None:
        out["engine"] = eng_main
    if sweep:
        out["agent_saturation"] = curve
    return out


def _summary(res: list[dict], wall: float) -> dict:
    ttft = [(r["first_token"] - r["t0"]) * 1e3 for r in res if r["first_token"] is not None]
    lat = [(r["final"] - r["t0"]) * 1e3 for r in res if r["final"] is not None]
    # saturation throughput (jobs/s at saturation): completions per second over the middle
    # half of the finish times, past the ramp-up and before the drain (meaningful with jobs >= 4 x concurrency)
    fin = sorted(r["final"] for r in res if r["final"] is not None)
    steady = None
    if len(fin) >= 8:
        a, b = len(fin) // 4, (3 * len(fin)) // 4
        if fin[b] > fin[a]:
            steady = round((b - a) / (fin[b] - fin[a]), 3)
    return {"jobs": len(res), "wall_s": round(wall, 3), "jobs_per_s": round(len(res) / wall, 3),
            "steady_jobs_per_s": steady,
            "e2e_ttft_p50_ms": round(statistics.median(ttft), 1) if ttft else None,
            "e2e_ttft_p90_ms": round(_pct(ttft, 0.9), 1) if ttft else None,
            "job_latency_p50_ms": round(statistics.median(lat), 1) if lat else None,
            "errors": sum(r["error"] for r in res), "degraded_jobs": sum(r.get("degraded", False) for r in res),
            "mean_tokens_streamed": round(
                statistics.mean(r["tokens"] for r in res), 1) if res else 0}


def _main() -> int:
    import argparse

    ap = argparse.ArgumentParser(description="e2e client: drive POST /rag/jobs + SSE at a concurrency")
    ap.add_argument("--url", required=True)
    ap.add_argument("--questions", required=True, help="JSON list of questions")
    ap.add_argument("--concurrency", type=int, required=True)
    ap.add_argument("--timeout", type=float, default=1800.0)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    with open(a.questions) as f:
        qs = json.load(f)
    t0 = time.perf_counter()
    res = asyncio.run(_drive(a.url, qs, a.concurrency, a.timeout))
    wall = time.perf_counter() - t0
    with open(a.out, "w") as f:
        json.dump({"records": res, "wall_s": wall}, f)
    return 0


if __name__ == "__main__":
    raise SystemExit(_main())
