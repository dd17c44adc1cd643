"""Front door + N sharded CPU replicas under load (VERDICT r3 item 7's done-criterion).

N replica processes (service/cluster.py ``demo_runtime`` with GRAG_DEMO_ROWS rows per scope table, a
scripted LLM that sleeps GRAG_DEMO_LLM_DELAY per call) hold 1/N of every table each; the front door
serves ``POST /rag/jobs`` + SSE over real HTTP (service/e2e.py) and every retrieval round of every job
fans out replica-to-replica over the shard mesh (service/mesh.py), or with --transport collective as
lockstep rounds over the replicas' process group (service/collective.py; --device cuda: tables on the
GPU and the rounds' payloads through the one-shot IPC gather).  Reports jobs/s, and per replica the
mesh's rounds, rounds/s, round latency p50 / p99 and degraded rounds.

  python scripts/mesh_load.py --replicas 8 --jobs 512 --concurrency 256 [--out profiles/mesh_load_r4.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(replicas: int = 8, jobs: int = 512, concurrency: int = 256, rows: int = 2000, delay: float = 0.002,
        slots: int = 64, transport: str = "mesh", device: str = "cpu") -> dict:
    from githubrepostorag_amd.config import Settings
    from githubrepostorag_amd.service.api import APIState, create_app
    from githubrepostorag_amd.service.cluster import ClusterRuntimeView, ReplicaHub, spawn_replicas
    from githubrepostorag_amd.service.e2e import run_e2e
    from githubrepostorag_amd.service.events import EventLog

    events = EventLog()
    hub = ReplicaHub(events, job_timeout=600.0)
    env = {"GRAG_DEMO_LLM_DELAY": str(delay), "GRAG_DEMO_SLOTS": str(slots), "GRAG_DEMO_ROWS": str(rows),
           "CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": "", "OMP_NUM_THREADS": "1",
           "GRAG_SHARD_TRANSPORT": transport, "GRAG_HEALTH_EVERY": "0.5", "GRAG_DEMO_DEVICE": device}
    gpus = None
    if device.startswith("cuda"):  # every replica on the one visible card (the 1-GPU box)
        env.pop("CUDA_VISIBLE_DEVICES")
        env.pop("HIP_VISIBLE_DEVICES")
        gpus = [0] * replicas
    procs = spawn_replicas(replicas, hub.address, hub.authkey,
                           ["--factory", "githubrepostorag_amd.service.cluster:demo_runtime", "--device", device],
                           env=env, shards=replicas, gpus=gpus)
    try:
        t0 = time.time()
        while hub.live_count() < replicas:
            if time.time() - t0 > 180 or any(p.poll() is not None for p in procs):
                raise RuntimeError(f"only {hub.live_count()} of {replicas} replicas came up")
            time.sleep(0.1)
        s = Settings(index_dir=None, data_dir=None)
        state = APIState(runtime=ClusterRuntimeView(hub, s), queue=hub.queue, events=events, flags=hub.flags)
        qs = [f"where are the widgets of module m{i % 23} handled {i}" for i in range(jobs)]
        res = run_e2e(create_app(state), qs, concurrency, warmup=qs[:min(16, jobs)])
        time.sleep(1.5)  # replicas report mesh stats every 0.5 s
        reps = hub.health()["replicas"]
        mesh = [dict(rank=r["rank"], **(r.get("collective_stats") or r.get("mesh_stats") or {})) for r in reps]
        rounds = sum(m.get("rounds", 0) for m in mesh)
        return {"replicas": replicas, "transport": transport, "device": device, "rows_per_table": rows, "jobs": res["jobs"],
                "concurrency": concurrency, "jobs_per_s": res["jobs_per_s"], "errors": res["errors"],
                "degraded_jobs": res["degraded_jobs"], "job_latency_p50_ms": res["job_latency_p50_ms"],
                "shard_rounds": rounds,
                "round_p50_ms_max": max((m.get("p50_ms", 0) for m in mesh), default=None),
                "round_p99_ms_max": max((m.get("p99_ms", 0) for m in mesh), default=None),
                "rounds_per_s_total": round(rounds / max(1e-9, res["wall_s"]), 1),
                "stacked_searches": sum(m.get("stacked_searches", 0) for m in mesh),
                "served_msgs": sum(m.get("served_msgs", 0) for m in mesh),
                "served_reqs": sum(m.get("served_reqs", 0) for m in mesh), "per_replica": mesh}
    finally:
        hub.close()
        for p in procs:
            try:
                p.wait(timeout=30)
            except Exception:
                p.kill()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replicas", type=int, default=8)
    ap.add_argument("--jobs", type=int, default=512)
    ap.add_argument("--concurrency", type=int, default=256)
    ap.add_argument("--rows", type=int, default=2000)
    ap.add_argument("--delay", type=float, default=0.002)
    ap.add_argument("--transport", default="mesh", choices=["mesh", "hub", "collective"])
    ap.add_argument("--device", default="cpu", help="cuda: every replica's tables on the visible GPU")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    res = run(a.replicas, a.jobs, a.concurrency, a.rows, a.delay, transport=a.transport, device=a.device)
    print(json.dumps({k: v for k, v in res.items() if k != "per_replica"}))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
