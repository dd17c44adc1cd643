"""Shard rounds as lockstep collectives among the replicas (service/collective.py), against the
socket mesh (service/mesh.py) and a flat store: every replica's sharded searches, traversal lookups
and counts equal the flat store's whichever transport carries them; concurrent fan-outs share
rounds; a closing replica keeps ticking until every replica has closed.

CPU: 3 gloo ranks.  GPU (``-m gpu``): 2 replicas on cuda:0, payloads through the one-shot IPC
gather (parallel/custom_ar.py) -- the device exchange VERDICT r4 item 7 asks for -- with identical
results to the mesh.  Reference: one shared ANN store per worker
(rag_worker/src/worker/services/graph_rag_retrievers.py:68-134); SURVEY §2.8 C3/C4, §5.8."""
import pytest
import torch

from tests.dist_utils import run_ranks

D = 32


def _rows(n, seed=0):
    g = torch.Generator().manual_seed(seed)
    ids = [f"row{i}" for i in range(n)]
    texts = [f"text {i}" for i in range(n)]
    vecs = torch.nn.functional.normalize(torch.randn(n, D, generator=g), dim=1)
    metas = [{"namespace": "default", "repo": f"r{i % 5}", "module": f"m{i % 7}", "file_path": f"m{i % 7}/f{i % 11}.py"}
             for i in range(n)]
    return ids, texts, vecs, metas


def _replicas(rank, world, device, ipc):
    """Per rank: the mesh (routed writes, and the A side of the comparison), the collective transport
    over the world group, and one ShardedStore on each."""
    import secrets

    import torch.distributed as dist

    from githubrepostorag_amd.index.sharded_store import ShardedStore
    from githubrepostorag_amd.index.store import VectorStore
    from githubrepostorag_amd.parallel import comm
    from githubrepostorag_amd.service.collective import CollectiveShardTransport
    from githubrepostorag_amd.service.mesh import PeerMesh

    key = [secrets.token_bytes(16) if rank == 0 else None]
    dist.broadcast_object_list(key, src=0)
    group = comm.world_group()
    if ipc:
        from githubrepostorag_amd.parallel.custom_ar import enable_for_group

        assert enable_for_group(group, device) is not None, "one-shot IPC exchange unavailable"
    loc = VectorStore(D, device)
    mesh = PeerMesh(rank, world, key[0], store=loc)
    addrs = [None] * world
    dist.all_gather_object(addrs, tuple(mesh.address))
    mesh.set_peers({r: a for r, a in enumerate(addrs)})
    coll = CollectiveShardTransport(rank, world, group, device, store=loc, fallback=mesh)
    return loc, mesh, coll, ShardedStore(loc, rank, world, mesh), ShardedStore(loc, rank, world, coll)


def _check(rank, world, device="cpu", ipc=False, n_rows=300):
    import threading
    import time

    import torch.distributed as dist

    from githubrepostorag_amd.index.sharded_store import round_health
    from githubrepostorag_amd.index.store import VectorStore

    loc, mesh, coll, via_mesh, via_coll = _replicas(rank, world, device, ipc)
    ids, texts, vecs, metas = _rows(n_rows)
    if rank == 1:  # ingest on one replica: rows routed to their owners (writes ride the mesh)
        assert via_coll.table("chunk").upsert(ids, texts, vecs, metas) == n_rows
    dist.barrier()
    flat = VectorStore(D, device)
    flat.table("chunk").upsert(ids, texts, vecs, metas)
    g = torch.Generator().manual_seed(9)
    Q = torch.nn.functional.normalize(torch.randn(5, D, generator=g), dim=1)
    out = {"mismatch": []}
    for flt in (None, {"repo": "r2"}, {"module": "m3", "namespace": "default"}, {"repo": "missing"}):
        ref = [[h.row_id for h in hs] for hs in flat.table("chunk").search(Q, 7, flt)]
        with round_health() as h:
            got_c = [[h_.row_id for h_ in hs] for hs in via_coll.table("chunk").search(Q, 7, flt)]
        got_m = [[h_.row_id for h_ in hs] for hs in via_mesh.table("chunk").search(Q, 7, flt)]
        if got_c != ref or got_m != ref or h["degraded_rounds"]:
            out["mismatch"].append(str(flt))
    pairs = [("repo", "r1"), ("module", "m4"), ("file_path", "m2/f3.py")]
    ref = [[x.row_id for x in hs] for hs in flat.table("chunk").search_pairs(Q[0], pairs, 4)]
    if [[x.row_id for x in hs] for hs in via_coll.table("chunk").search_pairs(Q[0], pairs, 4)] != ref:
        out["mismatch"].append("pairs")
    out["count"] = via_coll.table("chunk").count()
    # concurrent fan-outs from 32 threads share lockstep rounds (and stacked launches on the shards); the
    # mesh runs the same load for comparison
    Qc = torch.nn.functional.normalize(torch.randn(32, D, generator=torch.Generator().manual_seed(rank)), dim=1)
    ref = [[h.row_id for h in hs] for hs in flat.table("chunk").search(Qc, 5, {"namespace": "default"})]
    for name, st in (("mesh", via_mesh), ("collective", via_coll)):
        res, errs = [None] * 32, []

        def job(i, st=st, res=res, errs=errs):
            try:
                res[i] = [h.row_id for h in st.table("chunk").search(Qc[i:i + 1], 5, {"namespace": "default"})[0]]
            except Exception as e:  # pragma: no cover
                errs.append(repr(e))

        b0 = coll.stats["busy_rounds"]
        dist.barrier()
        ths = [threading.Thread(target=job, args=(i,)) for i in range(32)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        bad = [(i, res[i], ref[i]) for i in range(32) if res[i] != ref[i]]
        out[f"concurrent_{name}"] = {"errors": errs[:3], "mismatches": len(bad), "first": bad[:2]}
        if name == "collective":
            out["concurrent_ok"] = not errs and not bad
            out["busy_rounds"] = coll.stats["busy_rounds"] - b0
            # the 32 fan-outs' rounds are big enough for the score exchange (C3 as a tensor all-gather): each
            # query got back at most k = 5 hits in total from the other shards, not 5 per shard
            out["pruned"] = {k: coll.stats.get(k, 0) for k in ("score_exchanges", "hits_sent", "hits_pruned")}
    # round latency of each transport (sequential single-query fan-outs)
    lat = {}
    for name, st in (("mesh", via_mesh), ("collective", via_coll)):
        dist.barrier()
        ts = []
        for i in range(40):
            t0 = time.perf_counter()
            st.table("chunk").search(Q[i % 5:i % 5 + 1], 5, None)
            ts.append(time.perf_counter() - t0)
        lat[name] = sorted(ts)[len(ts) // 2] * 1000
    out["p50_ms"] = lat
    out["stats"] = coll.round_stats()
    if rank == 0:
        time.sleep(0.05)  # a replica that closes late: the others keep ticking until it has
    coll.close()
    mesh.close()
    out["closed"] = coll._closed.is_set()
    return out


def test_collective_transport_matches_flat_and_mesh_cpu():
    outs = run_ranks(_check, 3, "cpu", False)
    for r, o in enumerate(outs):
        assert o["mismatch"] == [], (r, o["mismatch"])
        assert o["count"] == 300
        assert o["concurrent_ok"], (r, o["concurrent_mesh"], o["concurrent_collective"])
        assert o["busy_rounds"] < 32, o["busy_rounds"]  # 32 fan-outs shared rounds
        assert o["closed"]
        assert o["stats"]["degraded_rounds"] == 0 and o["stats"]["served"] > 0
        p = o["pruned"]
        assert p["score_exchanges"] >= 1 and p["hits_pruned"] > 0, p
        # 3 ranks x 32 single-query fan-outs, k = 5: at most 5 winners per query leave the other two shards
        assert p["hits_sent"] <= 5 * 32 * 2, p
        print(f"replica {r}: round p50 mesh {o['p50_ms']['mesh']:.3f} ms, collective "
              f"{o['p50_ms']['collective']:.3f} ms; 32 concurrent fan-outs in {o['busy_rounds']} rounds")


@pytest.mark.gpu
def test_collective_transport_device_exchange_two_replicas_on_one_gpu():
    """2 replicas on cuda:0: the rounds' payloads cross through the IPC one-shot gather."""
    outs = run_ranks(_check, 2, "cuda:0", True)
    for r, o in enumerate(outs):
        assert o["mismatch"] == [], (r, o["mismatch"])
        assert o["count"] == 300 and o["closed"]
        assert o["concurrent_ok"], (r, o["concurrent_mesh"], o["concurrent_collective"], o["stats"])
        assert o["stats"]["device_exchanges"] > 0 and o["stats"].get("device_detached", 0) == 0
        print(f"replica {r}: round p50 mesh {o['p50_ms']['mesh']:.3f} ms, "
              f"collective {o['p50_ms']['collective']:.3f} ms; {o['stats']}")
