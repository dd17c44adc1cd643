"""The front door over 2 replica processes that both serve from the GPU (service/cluster.py): each replica
runs the product runtime (in-process engine on cuda:0 with hipGraph decode, GPU encoder and vector store;
``gpu_demo_runtime``), jobs go through POST /rag/jobs + SSE, the hub places them on both replicas, and every
job's retrieval fans out over the row-sharded index through the hub (INDEX_SHARDING=shard, 2 shards)."""
import json
import time

import pytest

pytestmark = pytest.mark.gpu


def _sse(client, job_id):
    events = []
    with client.stream("GET", f"/rag/jobs/{job_id}/events") as r:
        for line in r.iter_lines():
            if line.startswith("data:"):
                msg = json.loads(line.split(":", 1)[1])
                events.append((msg["event"], msg["data"]))
                if msg["event"] == "final":
                    break
    return events


def test_front_door_over_gpu_replicas():
    from fastapi.testclient import TestClient

    from githubrepostorag_amd.config import Settings
    from githubrepostorag_amd.service.api import APIState, create_app
    from githubrepostorag_amd.service.cluster import ClusterRuntimeView, ReplicaHub, spawn_replicas
    from githubrepostorag_amd.service.events import EventLog

    events = EventLog()
    hub = ReplicaHub(events, job_timeout=120.0)
    env = {"QWEN_MODEL": "qwen2-small", "QWEN_MAX_OUTPUT": "16", "MAX_MODEL_LEN": "2048", "MAX_NUM_SEQS": "16",
           "KV_CACHE_GB": "0.5", "WORKER_MAX_JOBS": "3", "OMP_NUM_THREADS": "1"}
    procs = spawn_replicas(2, hub.address, hub.authkey,
                           ["--factory", "githubrepostorag_amd.service.cluster:gpu_demo_runtime", "--device", "cuda"],
                           env=env, shards=2)
    state = APIState(runtime=ClusterRuntimeView(hub, Settings(index_dir=None, data_dir=None)), queue=hub.queue,
                     events=events, flags=hub.flags, ping_seconds=0.5)
    client = TestClient(create_app(state))
    client.__enter__()
    try:
        t0 = time.time()
        while hub.live_count() < 2:
            assert time.time() - t0 < 100, "GPU replicas did not connect"
            assert all(p.poll() is None for p in procs), "a GPU replica exited during startup"
            time.sleep(0.2)
        ids = [client.post("/rag/jobs", json={"query": f"where are widgets handled {i}"}).json()["job_id"]
               for i in range(6)]
        replicas = set()
        for jid in ids:
            ev = _sse(client, jid)
            names = [e for e, _ in ev]
            assert names[0] == "started" and names[-1] == "final", names
            final = ev[-1][1]
            assert not final.get("error"), final
            assert isinstance(final.get("answer"), str)
            deadline = time.time() + 10  # the hub records the result just after the forwarded "final" event
            while time.time() < deadline and "result" not in hub.queue.results.get(jid, {}):
                time.sleep(0.05)
            replicas.add(hub.queue.results[jid]["result"]["replica"])
        assert replicas == {0, 1}, "both GPU replicas must have served jobs"
        h = client.get("/health").json()
        assert h["status"] == "UP", h
        assert len(h["components"]["vector_index"]["details"]["replicas"]) == 2
    finally:
        client.__exit__(None, None, None)
        hub.close()
        for p in procs:
            try:
                p.wait(timeout=30)
            except Exception:
                p.kill()
