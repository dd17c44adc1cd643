"""CLI entry points on CPU with tiny random-init models: `ingest` (synthetic
repo -> index snapshot) then `ask` over the restored snapshot, `config`."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(tmp):
    return dict(os.environ, QWEN_MODEL="qwen2-tiny", EMBED_MODEL="encoder-tiny", DEVICE="cpu",
                CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", INDEX_DIR=str(tmp / "idx"), DATA_DIR=str(tmp / "data"),
                PUSHGATEWAY_ADDRESS="")


def _run(args, tmp):
    r = subprocess.run([sys.executable, "-m", "githubrepostorag_amd", *args], cwd=ROOT, env=_env(tmp),
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return r.stdout


def test_cli_ingest_then_ask(tmp_path):
    out = _run(["ingest", "--source", "synthetic", "--no-extract"], tmp_path)
    lines = [json.loads(x) for x in out.splitlines() if x.startswith("{")]
    assert lines[0]["ok"] and lines[0]["nodes_per_scope"]["chunk"] > 0
    assert lines[-1]["counts"]["embeddings"] > 0
    assert (tmp_path / "idx" / "manifest.json").exists()
    ans = json.loads(_run(["ask", "where is the retry policy?"], tmp_path))
    assert ans["answer"] and ans["sources"]
    assert all(s["repo"] == "synthetic-repo" for s in ans["sources"])


def test_cli_config(tmp_path):
    cfg = json.loads(_run(["config"], tmp_path))
    assert cfg["qwen_model"] == "qwen2-tiny" and cfg["max_rag_attempts"] == 3 and "github_token" not in cfg
