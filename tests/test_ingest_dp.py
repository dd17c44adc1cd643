"""Data-parallel ingest (`ingest --dp N`): N rank processes (gloo on CPU here) each
ingest every N-th repository, then write S shard snapshots partitioned by crc32(row id) that a sharded
front door loads (index/sharded_store.py).  Checked against a single-process ingest of the same
repositories: same chunk rows, each on the shard that owns it, every shard snapshot loadable."""
import json
import os
import subprocess
import sys

from githubrepostorag_amd.index.sharded_store import merge_into, shard_dir, shard_of, split_store
from githubrepostorag_amd.index.store import VectorStore

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(tmp, name):
    env = dict(os.environ, QWEN_MODEL="qwen2-tiny", EMBED_MODEL="encoder-tiny", DEVICE="cpu",
               CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", DATA_DIR=str(tmp / f"data-{name}"),
               PUSHGATEWAY_ADDRESS="")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT", "INDEX_DIR"):
        env.pop(k, None)
    return env


def _run(args, tmp, name):
    r = subprocess.run([sys.executable, "-m", "githubrepostorag_amd", *args], cwd=ROOT, env=_env(tmp, name),
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    return [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]


def _ids(store, scope):
    return set(store.tables[scope].rows.key_to_row)


def test_split_merge_roundtrip():
    import torch

    st = VectorStore(8, "cpu")
    ids = [f"row-{i}" for i in range(40)]
    st.table("chunk").upsert(ids, [f"t{i}" for i in ids], torch.randn(40, 8),
                             [{"repo": "r", "namespace": "n"} for _ in ids])
    st.table("chunk").delete(ids[:5])
    parts = split_store(st, 3)
    assert sum(p.table("chunk").count() for p in parts) == 35
    for s, p in enumerate(parts):
        assert all(shard_of(r, 3) == s for r in _ids(p, "chunk"))
    back = VectorStore(8, "cpu")
    for p in parts:
        merge_into(back, p)
    assert _ids(back, "chunk") == set(ids[5:])
    q = torch.randn(2, 8)
    a = [[h.row_id for h in hs] for hs in st.table("chunk").search(q, 5)]
    b = [[h.row_id for h in hs] for hs in back.table("chunk").search(q, 5)]
    assert a == b


def test_cli_ingest_dp_matches_single_process(tmp_path):
    out = _run(["ingest", "--dp", "2", "--source", "synthetic", "--n-repos", "2", "--no-extract", "--save",
                str(tmp_path / "dp")], tmp_path, "dp")
    summary = [x for x in out if "ingest_dp" in x]
    assert summary and summary[0]["shards"] == 2 and len(summary[0]["ranks"]) == 2
    assert sorted(r for x in summary[0]["ranks"] for r in x["repos"]) == ["synthetic-repo-0", "synthetic-repo-1"]
    assert not (tmp_path / "dp" / "parts").exists()
    _run(["ingest", "--source", "synthetic", "--repos", "synthetic-repo-0", "synthetic-repo-1", "--no-extract",
          "--save", str(tmp_path / "flat")], tmp_path, "flat")
    flat = VectorStore.load(tmp_path / "flat", "cpu")
    shards = [VectorStore.load(tmp_path / "dp" / shard_dir(s, 2), "cpu") for s in range(2)]
    union = set()
    for s, st in enumerate(shards):
        ids = _ids(st, "chunk")
        assert ids and all(shard_of(r, 2) == s for r in ids)
        union |= ids
    assert union == _ids(flat, "chunk")
    assert {st.tables["chunk"].rows.get(0)[2]["repo"] for st in shards} <= {"synthetic-repo-0", "synthetic-repo-1"}
