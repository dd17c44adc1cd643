"""The bench.py driver contract on CPU: single process, and two ranks under
torch.distributed.run (gloo) with tiny models — one JSON line from rank 0
with the whole-job aggregate, weak scaling and the BASELINE metric name."""
import json
import os
import subprocess
import sys

from dist_utils import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = ["--model", "qwen2-tiny", "--encoder", "encoder-tiny", "--index-size", "4000", "--index-kind", "ivf",
        "--nlist", "16", "--nprobe", "4", "--batch", "3", "--prompt-len", "48", "--gen-len", "5",
        "--ingest-files", "4", "--steps", "2", "--warmup", "1", "--agent-jobs", "8", "--agent-concurrency", "4", "--agent-synth-len", "16",
        "--ingest-ref-cap-files", "0"]


def _run(cmd, env, timeout=600):
    # a stuck rank dumps every thread's stack (bench.py GRAG_DUMP_STACKS_AFTER, repeated) well before the
    # test's own limit, and a timed-out run fails with those stacks instead of a bare TimeoutExpired
    env = dict(env, GRAG_DUMP_STACKS_AFTER=str(int(timeout * 0.6)), GRAG_DUMP_STACKS_REPEAT="1")
    p = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, 9)
        out, err = p.communicate()
        raise AssertionError(f"bench run hung (> {timeout} s); stacks:\n{err[-12000:]}") from None

    class R:
        returncode, stdout, stderr = p.returncode, out, err

    r = R
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_single_process_cpu():
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    res = _run([sys.executable, "bench.py", "--gpus", "1", *TINY, "--ingest-ref-cap-files", "3", "--ingest-ref-cap",
                "48"], env)
    assert res["n_gpus"] == 1 and res["steps"] == 2 and res["warmup"] == 1
    assert res["metric"].startswith("RAG queries/sec") and res["value"] > 0 and res["higher_is_better"]
    assert res["scaling"] == "weak" and res["config"]["global_batch"] == 3
    assert res["ingest_docs_per_s"] > 0 and res["p50_ttft_ms"] > 0 and res["p90_ttft_ms"] >= res["p50_ttft_ms"]
    assert res["headline_loop"].startswith("serving loop") and res["harness_loop"]["value"] > 0
    ci = res["concurrent_ingest"]  # ingest + open-loop queries on one engine, with the wait anatomy
    assert ci["queries"] > 0 and "decode" in ci["engine_steps"] or "prefill" in ci["engine_steps"]
    assert "inflight_step_rest_p50_ms" in ci["submit_to_first_token_anatomy"]
    ref = res["ingest_ref_cap"]  # the one-cap-for-every-call ingest pass (2048 by default)
    assert res["ingest_docs_per_s_ref_cap"] > 0 and ref["token_cap"] == 48 and ref["files"] == 3


def test_bench_two_ranks_gloo():
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    res = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "2", *TINY],
               env)
    assert res["n_gpus"] == 2 and res["config"]["global_batch"] == 6 and res["config"]["parallelism"] == "dp2"
    assert res["value"] > 0
    # agent phase through one front door over two sharded replicas (every retrieval fans out over the hub)
    ae = res["agent_e2e"]
    assert ae["front_door"] == "front door + 2 sharded replicas" and ae["errors"] == 0 and ae["jobs"] == 16
    assert sorted(r["shard"] for r in ae["replicas"]) == ["0/2", "1/2"]


def test_bench_tensor_parallel_two_ranks_gloo():
    """--tp 2 on two ranks: one TP group serving one DP replica's queries in
    lockstep (a desync would hang or fail the run), index sharded over both,
    retrieval prefetched on a helper thread (arrivals admitted at an agreed step)."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    res = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "2",
                "--tp", "2", *TINY], env)
    assert res["config"]["parallelism"] == "tp2dp1" and res["config"]["global_batch"] == 3
    assert res["value"] > 0 and "TP=2" in res["config"]["model"]
    # the serving loop under TP: the leader's runner takes the arrivals, the peer's mirrors its steps
    assert res["headline_loop"].startswith("serving loop") and res["serving_runner"]["value"] == res["value"]
    assert all(o["p50_ttft_ms"] > 0 for o in res["serving_runner"]["open_loop"])
    # ingest on the TP group (leader runs the pipeline, the peer mirrors its engine) and the agent
    # phase (TP leader runs jobs, the peer answers index rounds for its shard as a shard-only replica)
    assert res["ingest_docs_per_s"] > 0 and res["retrieval_prefetch"] is True
    ae = res["agent_e2e"]
    assert ae["errors"] == 0 and ae["jobs"] == 8 and "1 shard-only replicas, 2 shards" in ae["front_door"]


def test_bench_self_launch_two_ranks():
    """``python bench.py --gpus 2`` with no launcher spawns two rank processes
    itself (the driver's BENCH command form): the JSON reports n_gpus 2."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2",
               GRAG_DIST_BACKEND="gloo")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    res = _run([sys.executable, "bench.py", "--gpus", "2", *TINY], env)
    assert res["n_gpus"] == 2 and res["config"]["global_batch"] == 6 and res["config"]["parallelism"] == "dp2"
    assert res["value"] > 0 and "ttft_admission_policy" in res["harness_loop"]
    # the headline comes from the serving loop (per-query arrivals, lockstep retrieval rounds over 2 ranks)
    assert res["headline_loop"].startswith("serving loop") and res["serving_runner"]["value"] == res["value"]


def test_bench_self_launch_eight_ranks():
    """The driver's 8-GPU command form, rehearsed on the host: ``python bench.py --gpus 8`` spawns 8 rank
    processes (gloo), shards the index 8 ways, runs the agent phase through ONE front door over 8 sharded
    replicas (every retrieval round fans out replica-to-replica over the shard mesh) and reports the
    whole-job aggregate with no job errors and no degraded (shard-missing) retrieval."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1",
               GRAG_DIST_BACKEND="gloo")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    args = list(TINY)
    args[args.index("--agent-jobs") + 1] = "4"  # per GPU: 32 jobs over the 8 replicas
    args[args.index("--ingest-files") + 1] = "2"
    res = _run([sys.executable, "bench.py", "--gpus", "8", *args], env)  # exactly the driver's form
    assert res["n_gpus"] == 8 and res["config"]["parallelism"] == "dp8" and res["config"]["global_batch"] == 24
    assert res["value"] > 0 and res["ingest_docs_per_s"] > 0
    # serving loop over 8 ranks: per-query arrivals, lockstep retrieval rounds, open loops at 50 / 90 %
    srv = res["serving_runner"]
    assert res["headline_loop"].startswith("serving loop") and srv["value"] == res["value"]
    assert [o["load"] for o in srv["open_loop"]] == [0.5, 0.9] and res["p50_ttft_ms"] > 0
    ae = res["agent_e2e"]
    assert ae["front_door"] == "front door + 8 sharded replicas" and ae["errors"] == 0 and ae["jobs"] == 32
    assert ae["degraded_jobs"] == 0
    assert sorted(r["shard"] for r in ae["replicas"]) == [f"{r}/8" for r in range(8)]


def test_bench_self_launch_tp8_config4_form():
    """BASELINE config 4's exact command form on the host: ``python bench.py --gpus 8 --tp 8`` (one TP group
    of 8 ranks over gloo, a tiny decoder with Qwen2-72B's 8:1 GQA head layout): the TP leader's runner takes
    the serving loop's arrivals while 7 peers mirror its steps, ingest runs on the TP group, and the agent
    phase runs on the leader with 7 shard-only replicas answering index rounds for their shards."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1",
               GRAG_DIST_BACKEND="gloo")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    args = list(TINY)
    args[args.index("--model") + 1] = "qwen2-tiny-tp8"
    args[args.index("--agent-jobs") + 1] = "6"
    args[args.index("--ingest-files") + 1] = "2"
    res = _run([sys.executable, "bench.py", "--gpus", "8", "--tp", "8", *args], env, timeout=900)
    assert res["n_gpus"] == 8 and res["config"]["parallelism"] == "tp8dp1"
    assert res["value"] > 0 and "TP=8" in res["config"]["model"] and res["ingest_docs_per_s"] > 0
    assert res["headline_loop"].startswith("serving loop") and res["serving_runner"]["value"] == res["value"]
    ae = res["agent_e2e"]
    assert ae["errors"] == 0 and ae["jobs"] == 6 and "7 shard-only replicas, 8 shards" in ae["front_door"]
    assert ae["degraded_jobs"] == 0

