"""GPU vector store semantics on CPU (fp32 reference scoring): the five
scope tables that replace the reference's Cassandra SAI tables
(helm/templates/cassandra-initdb-configmap.yaml:13-102), cosine top-k,
metadata-equality filters incl. shredded multi-valued fields, idempotent
upserts, deletes, snapshot/restore (checkpoint-resume), and IVF recall."""
import torch

from githubrepostorag_amd.index.ivf import IVFIndex
from githubrepostorag_amd.index.store import VectorStore, VectorTable
from githubrepostorag_amd.utils import synthetic


def _unit(n, d, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.nn.functional.normalize(torch.randn(n, d, generator=g), dim=1)


def _table(n=300, d=32):
    X = _unit(n, d, 0)
    t = VectorTable("embeddings", d, "cpu", capacity=16)
    md = [{"repo": f"r{i % 3}", "module": f"m{i % 5}", "topics": ["cache", "retry"] if i % 4 == 0 else "auth",
           "file_path": f"src/f{i}.py"} for i in range(n)]
    t.upsert([f"id{i}" for i in range(n)], [f"text {i}" for i in range(n)], X, md)
    return t, X, md


def test_search_matches_brute_force():
    t, X, _ = _table()
    Q = _unit(4, 32, 1)
    hits = t.search(Q, 5)
    exact = Q.to(torch.bfloat16).float() @ X.to(torch.bfloat16).float().T
    for qi, hs in enumerate(hits):
        assert len(hs) == 5
        top = exact[qi].topk(5).values
        got = torch.tensor([exact[qi, int(h.row_id[2:])] for h in hs])
        assert torch.allclose(got, top, atol=2e-2)
        assert all(abs(h.score - float(exact[qi, int(h.row_id[2:])])) < 2e-2 for h in hs)
        assert hs[0].text == f"text {hs[0].row_id[2:]}"


def test_metadata_filters_and_multivalue():
    t, X, md = _table()
    Q = _unit(3, 32, 2)
    for hs in t.search(Q, 10, {"repo": "r1", "module": "m2"}):
        assert hs and all(h.metadata["repo"] == "r1" and h.metadata["module"] == "m2" for h in hs)
    for hs in t.search(Q, 10, {"topics": "retry"}):
        assert hs and all(int(h.row_id[2:]) % 4 == 0 for h in hs)
    assert all(hs == [] for hs in t.search(Q, 10, {"repo": "nope"}))


def test_idempotent_upsert_and_delete():
    t, X, _ = _table()
    n = t.count()
    newv = _unit(1, 32, 9)
    t.upsert(["id7"], ["replaced"], newv, [{"repo": "r9"}])
    assert t.count() == n
    top = t.search(newv, 1)[0][0]
    assert top.row_id == "id7" and top.text == "replaced" and top.metadata["repo"] == "r9"
    assert t.delete(["id7", "id8", "missing"]) == 2
    assert t.count() == n - 2
    assert all(h.row_id not in ("id7", "id8") for h in t.search(newv, 20)[0])


def test_snapshot_roundtrip(tmp_path):
    store = VectorStore(32, "cpu")
    X = _unit(50, 32, 3)
    for scope in ("chunk", "file", "repo"):
        store.table(scope).upsert([f"{scope}{i}" for i in range(50)], ["t"] * 50, X, [{"scope": scope}] * 50)
    store.save(tmp_path / "idx")
    back = VectorStore.load(tmp_path / "idx", "cpu")
    assert back.counts() == store.counts()
    Q = _unit(2, 32, 4)
    a = [[h.row_id for h in hs] for hs in store.table("file").search(Q, 5)]
    b = [[h.row_id for h in hs] for hs in back.table("file").search(Q, 5)]
    assert a == b


def test_ivf_recall_cpu():
    X = synthetic.clustered_vectors(4000, 32, seed=5, device="cpu").float()
    ivf = IVFIndex(32, 16, "cpu", dtype=torch.float32)
    ivf.train(X, iters=6, seed=0)
    ivf.add(X)
    Q = torch.nn.functional.normalize(X[:20] + 0.05 * _unit(20, 32, 6), dim=1)
    ref = (Q @ torch.nn.functional.normalize(X, dim=1).T).topk(10, dim=1).indices

    def recall(nprobe):
        _, ids = ivf.search(Q, 10, nprobe=nprobe)
        return sum(len(set(a.tolist()) & set(b.tolist())) for a, b in zip(ids, ref)) / ref.numel()

    assert recall(16) >= 0.99  # probing every list is exact search (up to bf16 score ties)
    assert recall(6) >= 0.8


def test_query_embedding_batcher_coalesces_threads():
    """Concurrent embed_queries calls (one per agent job thread) are served
    by one encoder pass and return exactly the rows a direct call gives."""
    import threading

    from githubrepostorag_amd.embed.service import Embedder

    emb = Embedder.from_name("encoder-tiny", device="cpu", seed=3)
    qs = [f"how does retry policy {i} handle timeouts" for i in range(24)]
    ref = emb.embed_queries(qs)
    emb.enable_batching(window_s=0.05)
    out = [None] * len(qs)
    barrier = threading.Barrier(len(qs))

    def run(i):
        barrier.wait()
        out[i] = emb.embed_queries([qs[i]])[0]

    th = [threading.Thread(target=run, args=(i,)) for i in range(len(qs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    b = emb._batcher
    assert b.texts == len(qs) and b.batches < len(qs)
    for i in range(len(qs)):
        assert torch.allclose(out[i].float(), ref[i].float(), atol=2e-2)
    emb.close()


def test_search_concurrent_with_upsert_and_compaction_cpu():
    import importlib.util
    import os

    spec = importlib.util.spec_from_file_location("tig", os.path.join(os.path.dirname(__file__), "test_index_gpu.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod._search_while_writing(torch.device("cpu"), rounds=12)


def test_search_pairs_concurrent_with_growing_upsert_cpu():
    import importlib.util
    import os

    spec = importlib.util.spec_from_file_location("tig", os.path.join(os.path.dirname(__file__), "test_index_gpu.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod._pairs_while_writing(torch.device("cpu"), rounds=12)
