"""Ingest pipeline on CPU (reference tests: ingest/tests/test_transform_service.py,
test_jupyter_notebook_handling.py, test_code_pipeline.py semantics)."""
import json

import pytest
import torch

from githubrepostorag_amd.agent.llm import ScriptedLLM
from githubrepostorag_amd.config import Settings
from githubrepostorag_amd.embed.service import Embedder
from githubrepostorag_amd.index.store import VectorStore
from githubrepostorag_amd.ingest.controller import IngestController
from githubrepostorag_amd.ingest.notebooks import is_output_heavy, is_setup_cell, process_notebook_text
from githubrepostorag_amd.ingest.preprocess import (filter_documents, infer_component_kind, language_of,
                                                    prepare_repo_documents)
from githubrepostorag_amd.ingest.readers import Document, LocalDirReader, SyntheticRepoReader
from githubrepostorag_amd.ingest.splitters import (CodeSplitter, DynamicCodeSplitter, SentenceSplitter,
                                                   count_tokens, create_splitter)
from githubrepostorag_amd.ingest.writer import row_id_for, sanitize_metadata


def _d(path, text="x = 1\n"):
    return Document(text, {"file_path": path})


def test_filter_skips_binary_and_boilerplate():
    docs = [_d(p) for p in ("a.py", "data.csv", "LICENSE", "x/data.json", "x/conf.json", "img.PNG", "store.db",
                            "diagram.drawio", ".gitignore", "README.md")]
    kept = {d.metadata["file_path"] for d in filter_documents(docs)}
    assert kept == {"a.py", "x/conf.json", "README.md"}  # .db skipped (reference quirk fixed)


def test_filter_drops_nul_bytes():
    assert filter_documents([_d("a.txt", "ab\x00cd")]) == []


def test_language_and_kind():
    assert language_of("src/main.py") == "python"
    assert language_of("Dockerfile") == "dockerfile"
    assert language_of("deploy/docker-compose.yml") == "yaml"
    assert language_of("k.hip") == "hip"
    assert infer_component_kind([_d("nb/a.ipynb")]) == "standalone"
    assert infer_component_kind([_d("nb/a.ipynb"), _d("pyproject.toml")]) == "service"
    assert infer_component_kind([_d("a.py")]) == "service"


def _nb(cells, **md):
    return json.dumps({"cells": cells, "metadata": md, "nbformat": 4, "nbformat_minor": 5})


def test_notebook_cleanup():
    nb = _nb([
        {"cell_type": "markdown", "source": ["# Title\n", "text"]},
        {"cell_type": "code", "source": "!pip install torch", "outputs": []},
        {"cell_type": "code", "source": "%matplotlib inline", "outputs": []},
        {"cell_type": "code", "source": "print(1)", "outputs": [{"output_type": "stream", "text": "1\n"}]},
        {"cell_type": "code", "source": "df", "outputs": [{"output_type": "execute_result",
                                                             "data": {"text/plain": "9" * 600}}]},
        {"cell_type": "code", "source": "", "outputs": []},
    ], title="My NB")
    out = process_notebook_text(nb)
    assert out.startswith("# My NB")
    assert "pip install" not in out and "matplotlib" not in out
    assert "```python\nprint(1)\n```" in out and "```\n1\n\n```" in out
    assert "9" * 600 not in out and "```python\ndf\n```" in out


def test_notebook_predicates():
    assert is_setup_cell("import os\n!wget http://x")
    assert not is_setup_cell("import os")
    logs = "\n".join(f"2024-01-01 10:00:0{i} INFO step" for i in range(5))
    assert is_output_heavy([{"output_type": "stream", "text": logs}])
    assert not is_output_heavy([{"output_type": "stream", "text": "| a | b |\n" + "x" * 600}])


def test_transform_notebook_in_prepare():
    nb = _nb([{"cell_type": "code", "source": "x=1", "outputs": []}])
    docs = prepare_repo_documents([Document(nb, {"file_path": "a/b.ipynb"})])
    assert docs[0].metadata["content_type"] == "notebook" and "```python\nx=1\n```" in docs[0].text
    assert docs[0].metadata["language"] == "python"


def test_sentence_splitter_budget_and_overlap():
    text = " ".join(f"Sentence number {i} talks about widgets." for i in range(400))
    sp = SentenceSplitter(chunk_size=64, chunk_overlap=16)
    chunks = sp.split_text(text)
    assert len(chunks) > 5
    for body, s, e in chunks:
        assert count_tokens(body) <= 64
        assert text[s:e] == body
    # consecutive chunks overlap
    assert chunks[1][1] < chunks[0][2]
    with pytest.raises(ValueError):
        SentenceSplitter(10, 20)


def test_code_splitter_python_blocks():
    src = "\n".join(f"def f{i}(x):\n    return x + {i}\n" for i in range(300))
    sp = CodeSplitter("python", chunk_lines=40, max_chars=600)
    chunks = sp.split_text(src)
    assert len(chunks) > 10
    for body, s, e in chunks:
        assert len(body) <= 600 and len(body.split("\n")) <= 40
        assert body.lstrip().startswith("def ")  # never cuts a function in half here
        assert src[s:e] == body


def test_code_splitter_brace_language():
    src = "\n".join("public int m%d() {\n  if (x) {\n    return %d;\n  }\n  return 0;\n}\n" % (i, i) for i in range(200))
    chunks = CodeSplitter("java", max_chars=500).split_text(src)
    assert all(c[0].count("{") == c[0].count("}") for c in chunks)


def test_create_splitter_fallback():
    assert isinstance(create_splitter("a.unknownext"), SentenceSplitter)
    assert isinstance(create_splitter("a.py"), CodeSplitter)
    assert isinstance(create_splitter(None), SentenceSplitter)
    nb = json.dumps({"metadata": {"kernelspec": {"name": "ir", "language": "R"}}, "cells": []})
    assert isinstance(create_splitter("x.ipynb", content=nb), SentenceSplitter)  # R has no grammar here
    nodes = DynamicCodeSplitter().get_nodes_from_documents([_d("a.py", "def f():\n  pass\n")])
    assert nodes and nodes[0].metadata["source_doc_id"]


def test_writer_sanitize_and_ids():
    md = {"repo": "r", "topics": ["a", "b"], "secret": "x", "extra": {"k": 1}, "file_path": None, "path": "p.py",
          "is_standalone": True}
    out = sanitize_metadata(md, "chunk")
    assert out["topics"] == "a,b" and "secret" not in out and "extra" not in out
    assert out["scope"] == "chunk" and all(isinstance(v, str) for v in out.values())
    n1, n2 = Document("abc", {"repo": "r"}), Document("abc", {"repo": "r"})
    assert row_id_for("chunk", n1) == row_id_for("chunk", n2) != row_id_for("file", n1)


def _echo_llm():
    def reply(p):
        if "GOOD" in p and "BAD" in p:
            return "GOOD"
        if "keywords" in p.lower():
            return "alpha, beta, gamma"
        if "title" in p.lower():
            return "A Title"
        return "This component does useful things with widgets and gadgets."
    return ScriptedLLM(reply)


@pytest.fixture(scope="module")
def embedder():
    return Embedder.from_name("encoder-tiny", device="cpu", seed=3)


def test_controller_end_to_end(tmp_path, embedder):
    store = VectorStore(embedder.dim, "cpu")
    llm = _echo_llm()
    ctl = IngestController(llm=llm, store=store, embedder=embedder, settings=Settings(data_dir=str(tmp_path)))
    events = []
    ctl.on_event = lambda k, d: events.append(k)
    res = ctl.ingest_component(repo="demo", namespace="ns", source="synthetic")
    assert res["documents"] > 0 and res["nodes_written"] > 0
    per = res["nodes_per_scope"]
    assert per["catalog"] >= 1 and per["repo"] >= 1 and per["module"] >= 1 and per["file"] >= 1
    # the reference's eight stages (+ split / extract_wait of the concurrent stage DAG)
    assert set(res["stage_seconds"]) == {"preprocess", "split", "code_nodes", "catalog", "file_summaries",
                                         "module_summaries", "repo_summaries", "extract_wait", "vector_write",
                                         "audit_and_clean"}
    # extractor passes of every level ran (file/module/repo/catalog nodes carry keywords too)
    for scope in ("file", "module", "repo", "catalog"):
        hs = store.table(scope).search(embedder.embed_queries(["widgets"]), 1, {"namespace": "ns"})[0]
        assert hs and hs[0].metadata.get("repo") == "demo"
    c = store.counts()
    assert c["embeddings"] == per["chunk"] and c["embeddings_catalog"] == per["catalog"]
    # chunk metadata carries extractor outputs that survive the allow-list
    hit = store.table("chunk").search(embedder.embed_queries(["widgets"]), 3, {"namespace": "ns"})[0]
    assert hit and hit[0].metadata["repo"] == "demo" and hit[0].metadata["excerpt_keywords"] == "alpha, beta, gamma"
    assert store.audit[-1]["repo"] == "demo"
    assert (tmp_path / "ingest_runs.jsonl").exists()
    assert (tmp_path / "repos" / "demo" / "raw_documents_main.json").exists()
    assert events[0] == "ingest_start" and events[-1] == "ingest_done"
    # unchanged repo -> skipped by the resume marker; forced re-ingest is idempotent (no duplicate rows)
    assert ctl.ingest_component(repo="demo", namespace="ns")["skipped"]
    ctl.ingest_component(repo="demo", namespace="ns", force=True)
    assert store.counts() == c


def test_controller_extractor_failures_isolated(embedder):
    calls = {"n": 0}

    def flaky(p):
        calls["n"] += 1
        if "keywords" in p.lower():
            raise RuntimeError("llm down")
        return "summary text that is long enough to be useful"

    store = VectorStore(embedder.dim, "cpu")
    ctl = IngestController(llm=ScriptedLLM(flaky), store=store, embedder=embedder, settings=Settings(data_dir=None))
    docs = SyntheticRepoReader(6).load_data("r2", seed=5)
    res = ctl.ingest_component(repo="r2", namespace="ns", documents=docs)
    assert res["nodes_written"] > 0
    hit = store.table("chunk").search(embedder.embed_queries(["x"]), 1)[0][0]
    assert hit.metadata["excerpt_keywords"].startswith("Error")


def test_ingest_many_formats(embedder):
    store = VectorStore(embedder.dim, "cpu")
    ctl = IngestController(llm=_echo_llm(), store=store, embedder=embedder, settings=Settings(data_dir=None),
                           extract=False)
    out = ctl.ingest_many([{"repo": "a", "namespace": "n1"}, ("b", "n2", "layer", "coll", "standalone")])
    assert [r["repo"] for r in out] == ["a", "b"]
    assert out[1]["component_kind"] == "standalone" and out[1]["collection"] == "coll"


def test_local_reader(tmp_path):
    (tmp_path / "pkg").mkdir()
    (tmp_path / "pkg" / "m.py").write_text("def f():\n    return 1\n")
    (tmp_path / "README.md").write_text("# hi\n")
    docs = LocalDirReader(str(tmp_path)).load_data("myrepo")
    assert sorted(d.metadata["file_path"] for d in docs) == ["README.md", "pkg/m.py"]
    assert all(d.metadata["repo"] == "myrepo" for d in docs)


def test_synthetic_reader_deterministic():
    a = SyntheticRepoReader(5).load_data("same")
    b = SyntheticRepoReader(5).load_data("same")
    assert [d.text for d in a] == [d.text for d in b]
    assert torch.tensor(0).item() == 0


def test_chunk_nodes_get_module_metadata():
    """the reference never stamps ``module`` on chunk nodes,
    leaving its module edge/filter empty at code scope."""
    from githubrepostorag_amd.ingest.controller import attach_common_metadata
    from githubrepostorag_amd.ingest.readers import Node

    n = Node(text="def f(): pass", metadata={"file_path": "billing/api/handlers.py"})
    attach_common_metadata([n], namespace="default", repo="r", branch="main", collection="misc",
                           component_kind="service", is_standalone=False, run_id="0", dev_forced=False,
                           doc_type="chunk")
    assert n.metadata["module"] == "billing" and n.metadata["scope"] == "chunk"


def test_ingest_token_audit_small_repo():
    """scripts/ingest_token_audit.py (the prefill floor quoted in profiles/ingest_critical_path_r4.txt) on
    an 8-file repo: every call kind is seen, and an ideal block cache computes fewer tokens than submitted."""
    import importlib.util
    import os
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("ingest_token_audit", os.path.join(root, "scripts",
                                                                                    "ingest_token_audit.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    runner = mod.FakeRunner(mod.load_tokenizer(None, 152064), 152064)
    calls = [([1] * 40 + [2] * 10, 32), ([1] * 40 + [3] * 10, 32), ([5] * 20, 64)]
    runner.calls.extend(calls)
    u = mod.ideal_unique(runner.calls)
    assert u == [50, 50 - 32, 20]  # the second prompt shares two full 16-token blocks with the first
    old = sys.argv
    try:
        sys.argv = ["ingest_token_audit", "--files", "8"]
        mod.main()
    finally:
        sys.argv = old
