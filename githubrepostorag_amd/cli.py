"""Command line entry points (``python -m githubrepostorag_amd <command>``).

Replaces the reference's three process entry points — the API
(rest_api/src/app/__main__.py:5-7, uvicorn on :8000), the ARQ worker
(helm/templates/rag-worker-deployment.yaml:64) and the ingest batch job
(ingest/src/app/__main__.py:7-18) — with one process per GPU that hosts the
engine, encoder, index, job workers and API together:

  serve    FastAPI app (jobs + SSE, /health, /metrics, /static UI, OpenAI /v1)
           with the in-process job workers; the runtime (models, index) is
           built once at startup on this process's GPU.  With TP=N under
           torchrun the engine is sharded over N GPUs and TP rank 0 serves.
           With --replicas N (or DP=N) this process is a GPU-less front door:
           one /rag/jobs + SSE endpoint, one job queue and event log, and N
           replica child processes (one per GPU) that run the jobs
           (service/cluster.py).
  replica  one per-GPU replica of a front door (started by serve --replicas).
  ingest   ingest repositories (github | local dir | synthetic) into the
           index and optionally snapshot it to INDEX_DIR.
  ask      one RAG query through the agent, printing events as they arrive.
  build    compile the gfx950 kernel library and the host runtime in-tree.
  config   print the resolved settings (env-compatible with the reference).
  bench    forward to bench.py (driver contract).
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import subprocess
import sys


def _settings(args):
    from .config import settings

    s = settings(reload=True)
    for k in ("qwen_model", "embed_model", "device", "index_dir", "model_dir", "encoder_dir"):
        v = getattr(args, k, None)
        if v:
            setattr(s, k, v)
    return s


def _runtime(args, build_engine=True, shard=None, device=None):
    from .service.runtime import RAGRuntime

    return RAGRuntime(_settings(args), build_engine=build_engine, shard=shard, device=device)


def cmd_serve(args) -> int:
    import uvicorn

    from .service.api import create_app

    s = _settings(args)
    logging.basicConfig(level=s.log_level, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    replicas = args.replicas if args.replicas is not None else s.dp
    if replicas > 1:
        return _serve_front_door(args, s, replicas)
    def factory():
        rt = _runtime(args)
        n = rt.warmup()  # decode graphs captured before the first request, not inside one
        logging.getLogger(__name__).info("captured %d decode graphs", n)
        return rt

    if s.tp > 1:
        # TP serving under torchrun: every rank builds its shard of the engine
        # now (collective), followers mirror the leader's engine loop, only
        # TP rank 0 of each group runs the API (port + DP index).
        from .service.api import APIState

        rt = factory()
        if not rt.tp_leader:
            rt.runner.join()
            return 0
        port = args.port + (rt.dp_group.rank if rt.dp_group is not None else 0)
        app = create_app(APIState(runtime=rt))
        uvicorn.run(app, host=args.host, port=port, log_level=s.log_level.lower())
        rt.close()
        return 0
    from .service.api import APIState

    app = create_app(APIState(ping_seconds=s.sse_ping_seconds), runtime_factory=factory)
    uvicorn.run(app, host=args.host, port=args.port, log_level=s.log_level.lower())
    return 0


def _serve_front_door(args, s, replicas: int) -> int:
    """One API + queue + event log for N per-GPU replica processes (service/cluster.py)."""
    import uvicorn

    from .service.api import APIState, create_app
    from .service.cluster import ClusterRuntimeView, ReplicaHub, spawn_replicas
    from .service.events import EventLog

    events = EventLog(keep_seconds=s.keep_result_s)
    hub = ReplicaHub(events, job_timeout=s.job_timeout_s, keep_result=s.keep_result_s)
    gpus = [int(g) for g in os.environ.get("GPUS", "").split(",") if g.strip()] or list(range(replicas))
    fwd = []
    for k in ("qwen_model", "embed_model", "index_dir", "model_dir", "encoder_dir"):
        v = getattr(args, k, None)
        if v:
            fwd += [f"--{k.replace('_', '-')}", v]
    shards = replicas if s.index_sharding == "shard" else 1
    procs = spawn_replicas(replicas, hub.address, hub.authkey, fwd, gpus=gpus[:replicas], shards=shards)
    state = APIState(runtime=ClusterRuntimeView(hub, s), queue=hub.queue, events=events, flags=hub.flags,
                     ping_seconds=s.sse_ping_seconds)
    app = create_app(state)
    try:
        uvicorn.run(app, host=args.host, port=args.port, log_level=s.log_level.lower())
    finally:
        hub.close()
        for p in procs:
            try:
                p.wait(timeout=30)
            except Exception:
                p.terminate()
    return 0


def cmd_replica(args) -> int:
    from .service.cluster import run_replica

    s = _settings(args)
    logging.basicConfig(level=s.log_level, format=f"%(asctime)s %(levelname)s replica{args.rank} %(name)s: %(message)s")
    if args.factory:
        import importlib

        mod, fn = args.factory.split(":")
        rt = getattr(importlib.import_module(mod), fn)(s)
        if args.shards > 1 and getattr(rt, "store", None) is not None:
            from .index.sharded_store import retain_shard

            retain_shard(rt.store, args.rank, args.shards)  # a factory builds full tables: keep this shard
    else:
        rt = _runtime(args, shard=(args.rank, args.shards) if args.shards > 1 else None)
        rt.warmup()
    host, port = args.hub.rsplit(":", 1)
    key = bytes.fromhex(os.environ["GRAG_HUB_AUTHKEY"])
    group = None
    if args.shards > 1 and os.environ.get("GRAG_SHARD_TRANSPORT") == "collective" and "WORLD_SIZE" in os.environ:
        from .parallel import comm  # the replicas' process group (spawn_replicas): shard rounds as collectives

        comm.init_distributed()
        group = comm.world_group()
        dev = str(getattr(rt, "device", "cpu"))
        if dev.startswith("cuda") and os.environ.get("GRAG_SHARD_IPC", "1") != "0":
            from .parallel.custom_ar import enable_for_group

            # payloads through the one-shot IPC gather: replicas on one card, or xGMI peers on a node
            enable_for_group(group, dev)
    try:
        return run_replica(rt, (host, int(port)), key, args.rank, shards=args.shards,
                           health_every=float(os.environ.get("GRAG_HEALTH_EVERY", "5")), group=group)
    finally:
        if hasattr(rt, "close"):
            rt.close()


def _spawn_ingest_ranks(n: int) -> int:
    """``ingest --dp N`` without a launcher: N rank processes of this command (one per GPU), no exec."""
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=os.environ.get("MASTER_PORT", str(port)))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, "-m", "githubrepostorag_amd", *sys.argv[1:]], env=env))
    rc = 0
    for p in procs:
        rc = rc or p.wait()
    return rc


def cmd_ingest_dp(args, s) -> int:
    """Data-parallel ingest: rank r of N ingests repositories r, r + N, ... on its own GPU,
    then the rows are re-partitioned by owning shard (crc32(row id) mod S) into S shard snapshots
    ``INDEX_DIR/shard-s-of-S`` that ``serve --replicas S`` loads (index/sharded_store.py).  Ids are content
    hashes (ingest/writer.py), so no id ranges are exchanged; the only collectives are a count all-gather
    (for the run manifest) and the barriers between the phases (gloo: nothing here needs the GPU fabric)."""
    import torch.distributed as dist

    from .index.sharded_store import merge_into, shard_dir, split_store
    from .index.store import VectorStore
    from .ingest.controller import IngestController
    from .parallel import comm

    info = comm.init_distributed(backend="gloo")
    rank, world = info.rank, info.world_size
    out = args.save or s.index_dir
    if not out:
        raise SystemExit("ingest --dp needs --save or INDEX_DIR (the shard snapshots go there)")
    shards = args.shards or world
    standalone = args.dev_force_standalone or s.dev_force_standalone
    if args.repos:
        comps = [{"repo": r, "namespace": args.namespace} for r in args.repos]
    elif args.source == "synthetic":
        comps = [{"repo": f"synthetic-repo-{i}", "namespace": args.namespace} for i in range(max(world, args.n_repos))]
    elif args.source == "github" and standalone:
        # the reference's dev mode (ingest_controller.py:490-542): every repository of the account, each a
        # standalone component; rank 0 lists them once and the list is broadcast so every rank splits the
        # same order
        from .ingest.readers import fetch_repositories

        box = [sorted(fetch_repositories(s.github_user, s.github_token)) if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        comps = [{"repo": r, "namespace": "default", "dev_force_standalone": True} for r in box[0]]
    else:
        raise SystemExit("ingest --dp splits a list of repositories: pass --repos, --source synthetic, or "
                         "--source github --dev-force-standalone")
    mine = comps[rank::world]
    import torch

    dev = f"cuda:{info.local_rank}" if torch.cuda.is_available() and s.device != "cpu" else "cpu"
    rt = _runtime(args, device=dev)
    ctl = IngestController(rt, extract=not args.no_extract)
    res = ctl.ingest_many(mine, branch=args.branch, source=args.source, path=args.path)  # components carry the flag
    counts = [None] * world
    dist.all_gather_object(counts, {"rank": rank, "repos": [r.get("repo") for r in res],
                                    "nodes": sum(r.get("nodes_written") or 0 for r in res),
                                    "documents": sum(r.get("documents") or 0 for r in res)})
    for s_, part in enumerate(split_store(rt.store, shards)):
        part.save(os.path.join(out, "parts", str(rank), shard_dir(s_, shards)))
    rt.close()
    dist.barrier()
    for s_ in range(rank, shards, world):  # each shard merged by one rank
        st = VectorStore(rt.store.dim, dev, rt.store.table_names, index_kind=s.index_kind, nlist=s.nlist,
                         nprobe=s.nprobe)
        for r in range(world):
            merge_into(st, VectorStore.load(os.path.join(out, "parts", str(r), shard_dir(s_, shards)), dev))
        for t in st.tables.values():
            if t.ivf:
                t.compact()
        st.save(os.path.join(out, shard_dir(s_, shards)))
        print(json.dumps({"shard": s_, "of": shards, "counts": st.counts()}))
    dist.barrier()
    if rank == 0:
        print(json.dumps({"ingest_dp": world, "shards": shards, "ranks": counts}))
        import shutil

        shutil.rmtree(os.path.join(out, "parts"), ignore_errors=True)
    dist.destroy_process_group()
    return 0 if all(r.get("ok") for r in res) else 1


def cmd_ingest(args) -> int:
    from .ingest.controller import IngestController

    s = _settings(args)
    if args.dp > 1 and "WORLD_SIZE" not in os.environ:
        return _spawn_ingest_ranks(args.dp)
    if args.dp > 1:
        logging.basicConfig(level=s.log_level, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
        return cmd_ingest_dp(args, s)
    logging.basicConfig(level=s.log_level, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    rt = _runtime(args)
    ctl = IngestController(rt, extract=not args.no_extract)
    if args.repos:
        comps = [{"repo": r, "namespace": args.namespace} for r in args.repos]
    else:
        comps = [{"repo": "synthetic-repo", "namespace": args.namespace}] if args.source == "synthetic" else []
    if args.source == "local" and not args.repos:
        comps = [{"repo": os.path.basename(os.path.abspath(args.path)), "namespace": args.namespace}]
    res = ctl.ingest_many(comps, branch=args.branch, dev_force_standalone=args.dev_force_standalone or s.dev_force_standalone,
                          source=args.source, path=args.path)
    for r in res:
        print(json.dumps({k: r.get(k) for k in ("ok", "repo", "namespace", "nodes_written", "documents",
                                                "nodes_per_scope", "run_seconds")}))
    out = args.save or s.index_dir
    if out:
        rt.store.save(out)
        print(json.dumps({"index_saved": out, "counts": rt.store.counts()}))
    rt.close()
    return 0 if all(r.get("ok") for r in res) else 1


def cmd_ask(args) -> int:
    rt = _runtime(args)
    agent = rt.agent()

    def progress(p):
        print(json.dumps({"event": "turn", "data": p})[:400], file=sys.stderr)

    res = agent.run(args.query, namespace=args.namespace, progress_cb=progress)
    print(json.dumps({"answer": res.get("answer"), "scope": res.get("scope"),
                      "sources": [s.get("metadata", {}) for s in res.get("sources") or []]}, indent=1))
    rt.close()
    return 0


def cmd_build(args) -> int:
    from .utils.native_build import build_all

    build_all(force=args.force, verbose=args.verbose)
    return 0


def cmd_config(args) -> int:
    print(json.dumps(_settings(args).to_dict(), indent=1, default=str))
    return 0


def cmd_bench(args, rest) -> int:
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return subprocess.call([sys.executable, os.path.join(root, "bench.py"), *rest])


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="githubrepostorag_amd", description=__doc__.split("\n\n")[0])
    sub = ap.add_subparsers(dest="cmd", required=True)

    def common(p):
        p.add_argument("--qwen-model", dest="qwen_model")
        p.add_argument("--embed-model", dest="embed_model")
        p.add_argument("--device")
        p.add_argument("--index-dir", dest="index_dir")
        p.add_argument("--model-dir", dest="model_dir")
        p.add_argument("--encoder-dir", dest="encoder_dir")

    p = sub.add_parser("serve", help="API + workers + engine in one process")
    common(p)
    p.add_argument("--host", default="0.0.0.0")
    p.add_argument("--port", type=int, default=8000)
    p.add_argument("--replicas", type=int, default=None,
                   help="front door over N per-GPU replica processes (default DP; GPUS=0,1,.. picks devices)")
    p = sub.add_parser("replica", help="one per-GPU replica of a front door (internal)")
    common(p)
    p.add_argument("--hub", required=True, help="host:port of the front door's replica hub")
    p.add_argument("--rank", type=int, default=0)
    p.add_argument("--shards", type=int, default=1, help="this replica holds shard RANK of SHARDS (index sharding)")
    p.add_argument("--factory", default=None, help="module:function(settings) -> runtime (tests)")
    p = sub.add_parser("ingest", help="ingest repositories into the index")
    common(p)
    p.add_argument("--source", choices=["github", "local", "synthetic"], default="synthetic")
    p.add_argument("--path", help="local directory (source=local)")
    p.add_argument("--repos", nargs="*", default=[])
    p.add_argument("--namespace", default="default")
    p.add_argument("--branch", default=None)
    p.add_argument("--dev-force-standalone", action="store_true")
    p.add_argument("--no-extract", action="store_true", help="skip the LLM summary/title/keyword extractors")
    p.add_argument("--save", help="snapshot directory (default INDEX_DIR)")
    p.add_argument("--dp", type=int, default=1, help="data-parallel ingest over N GPUs (one rank per GPU)")
    p.add_argument("--shards", type=int, default=0, help="--dp: shard snapshots to write (default N)")
    p.add_argument("--n-repos", dest="n_repos", type=int, default=2, help="--dp --source synthetic: repositories")
    p = sub.add_parser("ask", help="one RAG query through the agent")
    common(p)
    p.add_argument("query")
    p.add_argument("--namespace", default="default")
    p = sub.add_parser("build", help="compile the native libraries in-tree")
    p.add_argument("--force", action="store_true")
    p.add_argument("-v", "--verbose", action="store_true")
    p = sub.add_parser("config", help="print resolved settings")
    common(p)
    sub.add_parser("bench", help="run bench.py (remaining args are forwarded)", add_help=False)
    return ap


def main(argv=None) -> int:
    ap = build_parser()
    argv = list(sys.argv[1:] if argv is None else argv)
    if argv and argv[0] == "bench":
        return cmd_bench(None, argv[1:])
    args = ap.parse_args(argv)
    return {"serve": cmd_serve, "replica": cmd_replica, "ingest": cmd_ingest, "ask": cmd_ask, "build": cmd_build,
            "config": cmd_config}[args.cmd](args)


if __name__ == "__main__":
    sys.exit(main())
