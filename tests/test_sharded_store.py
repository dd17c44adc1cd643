"""Row-sharded store (index/sharded_store.py): N shards behind one facade give
the same hits as one flat store — plain searches, filtered searches and
whole graph traversals — and writes land on the owning shard only."""
import torch

from githubrepostorag_amd.embed.service import Embedder
from githubrepostorag_amd.index.sharded_store import (LocalShardTransport, ShardedStore, load_shard, retain_shard,
                                                      shard_dir, shard_of)
from githubrepostorag_amd.index.store import VectorStore
from githubrepostorag_amd.retrieval.graph import RetrieverFactory


def _rows(n, seed=0):
    g = torch.Generator().manual_seed(seed)
    ids = [f"row{i}" for i in range(n)]
    texts = [f"text {i}" for i in range(n)]
    vecs = torch.nn.functional.normalize(torch.randn(n, 32, generator=g), dim=1)
    metas = [{"namespace": "default", "repo": f"r{i % 5}", "module": f"m{i % 7}", "file_path": f"m{i % 7}/f{i % 11}.py",
              "topics": ["cache", "retry"] if i % 3 == 0 else ["queue"]} for i in range(n)]
    return ids, texts, vecs, metas


def _stores(n_shards, n=300, kind="flat"):
    flat = VectorStore(32, "cpu", index_kind=kind, nlist=8, nprobe=8)
    tr = LocalShardTransport()
    locs = [VectorStore(32, "cpu", index_kind=kind, nlist=8, nprobe=8) for _ in range(n_shards)]
    facades = [ShardedStore(loc, r, n_shards, tr) for r, loc in enumerate(locs)]
    for r, loc in enumerate(locs):
        tr.register(r, loc)
    ids, texts, vecs, metas = _rows(n)
    for scope in ("chunk", "file"):
        flat.table(scope).upsert(ids, texts, vecs, metas)
        facades[1].table(scope).upsert(ids, texts, vecs, metas)  # ingest on replica 1: routed by owner
    return flat, locs, facades, vecs


def test_writes_land_on_owner_shard_only():
    flat, locs, facades, _ = _stores(3)
    for r, loc in enumerate(locs):
        keys = list(loc.table("chunk").rows.key_to_row)
        assert keys and all(shard_of(k, 3) == r for k in keys)
    assert sum(loc.table("chunk").count() for loc in locs) == flat.table("chunk").count() == 300
    assert facades[2].table("chunk").count() == 300
    facades[0].table("chunk").delete(["row1", "row2", "row3"])
    assert facades[1].table("chunk").count() == 297


def test_search_matches_flat_store():
    flat, _, facades, vecs = _stores(3)
    g = torch.Generator().manual_seed(9)
    Q = torch.nn.functional.normalize(torch.randn(6, 32, generator=g), dim=1)
    for flt in (None, {"repo": "r2"}, {"module": "m3", "namespace": "default"}, {"topics": "cache"},
                {"file_path": "m1/f4.py"}, {"repo": "missing"}):
        ref = [[h.row_id for h in hs] for hs in flat.table("chunk").search(Q, 7, flt)]
        for fac in facades:
            got = [[h.row_id for h in hs] for hs in fac.table("chunk").search(Q, 7, flt)]
            assert got == ref, flt


def test_graph_traversal_across_shards_matches_flat():
    flat, _, facades, _ = _stores(3)
    emb = Embedder.from_name("encoder-tiny", device="cpu", seed=3)

    class Fixed:  # the retriever embeds the query: give both sides the same 32-d vector
        dim = 32

        def __init__(self):
            self.g = torch.Generator().manual_seed(4)

        def embed_query(self, q):
            torch.manual_seed(abs(hash(q)) % (1 << 31))
            return torch.nn.functional.normalize(torch.randn(32), dim=0)

    del emb
    fixed = Fixed()
    ref_r = RetrieverFactory(flat, fixed).for_chunk(k=10, start_k=3, adjacent_k=8, max_depth=2)
    for fac in facades:
        r = RetrieverFactory(fac, fixed).for_chunk(k=10, start_k=3, adjacent_k=8, max_depth=2)
        for q in ("retry cache", "queue worker", "broker session"):
            a = [(d.id, d.metadata["_depth"]) for d in ref_r.invoke(q, {"namespace": "default"})]
            b = [(d.id, d.metadata["_depth"]) for d in r.invoke(q, {"namespace": "default"})]
            assert a == b, q
            assert any(dep > 0 for _, dep in b)  # the traversal left the seeds' shard


def test_ivf_shards_and_snapshot(tmp_path):
    flat, locs, facades, vecs = _stores(2, n=600, kind="ivf")
    for loc in locs:
        for t in loc.tables.values():
            t.compact()
    q = vecs[:4]
    got = [[h.row_id for h in hs][:1] for hs in facades[0].table("chunk").search(q, 3)]
    assert got == [["row0"], ["row1"], ["row2"], ["row3"]]
    # per-shard snapshots, and a full snapshot cut down to one shard
    for fac in facades:
        fac.save(tmp_path / "idx")
    assert (tmp_path / "idx" / shard_dir(1, 2) / "manifest.json").exists()
    back = load_shard(tmp_path / "idx", 1, 2, "cpu")
    assert back.table("chunk").count() == locs[1].table("chunk").count()
    flat.save(tmp_path / "full")
    cut = load_shard(tmp_path / "full", 0, 2, "cpu")
    assert set(cut.table("chunk").rows.key_to_row) >= set()  # loaded
    assert cut.table("chunk").count() == locs[0].table("chunk").count()
    assert retain_shard(cut, 0, 2) == 0
