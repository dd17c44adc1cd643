"""Filtering, special-file transforms, language tagging and component-kind
inference (ingest/src/app/services/transform_service.py:10-127,
preprocess_service.py:23-56, scope_utils.py:8-27).

Deviation, on purpose: the reference's SKIP_EXT has a missing comma that
fuses ``".drawio" ".db"`` into one string, so ``.db`` files were NOT skipped
(SURVEY §2.11); here ``.db`` is skipped like the other binary stores.
Notebooks are cleaned from the fetched document text (the reference opened a
local path that does not exist for GitHub documents, quirk 14).
"""
from __future__ import annotations

import logging
from collections import defaultdict
from pathlib import PurePosixPath

from .notebooks import process_notebook_text
from .readers import Document

log = logging.getLogger(__name__)

SKIP_EXT = {
    ".csv", ".tsv", ".xlsx", ".xls", ".parquet", ".feather", ".xml", ".jsonl", ".ndjson",
    ".png", ".jpg", ".jpeg", ".gif", ".bmp", ".svg", ".webp", ".ico", ".tiff", ".tif", ".psd", ".drawio",
    ".mp3", ".wav", ".mp4", ".avi", ".mov", ".mkv", ".flv", ".zip", ".tar", ".gz", ".rar", ".7z", ".bz2",
    ".exe", ".dll", ".so", ".dylib", ".bin", ".log", ".dump", ".backup", ".db", ".sqlite", ".sqlite3",
}
SKIP_JSON_PATTERNS = {"data.json", "test-data.json", "sample.json", "mock.json", "responses.json", "fixtures.json"}
SKIP_NAMES = {
    "license", "license.txt", "license.md", "changelog", "changelog.txt", "changelog.md", "authors", "authors.txt",
    "authors.md", "contributors", "contributors.txt", "contributors.md", "copying", "copying.txt", "copying.md",
    "notice", "notice.txt", "notice.md", ".gitignore", ".gitattributes", ".gitmodules", ".dockerignore",
    ".eslintignore", ".prettierignore",
}
EXTENSION_TO_LANGUAGE = {
    ".py": "python", ".java": "java", ".kt": "kotlin", ".go": "go", ".js": "javascript", ".jsx": "javascript",
    ".ts": "typescript", ".tsx": "typescript", ".rb": "ruby", ".rs": "rust", ".c": "c", ".h": "c", ".cpp": "cpp",
    ".hpp": "cpp", ".cs": "csharp", ".php": "php", ".scala": "scala", ".swift": "swift", ".sh": "bash",
    ".bash": "bash", ".zsh": "zsh", ".yml": "yaml", ".yaml": "yaml", ".toml": "toml", ".ini": "ini", ".cfg": "ini",
    ".sql": "sql", ".md": "markdown", ".rst": "rst", ".proto": "protobuf", ".gradle": "gradle", ".groovy": "groovy",
    ".xml": "xml", ".json": "json", ".hip": "hip", ".cu": "cuda", ".ipynb": "python",
}


def _ext(path: str) -> str:
    return ("." + path.rsplit(".", 1)[-1].lower()) if "." in path.split("/")[-1] else ""


def filter_documents(docs: list[Document]) -> list[Document]:
    out = []
    for d in docs:
        path = d.metadata.get("file_path", "")
        ext, name = _ext(path), path.split("/")[-1].lower()
        if ext == ".json" and name in SKIP_JSON_PATTERNS:
            continue
        if ext in SKIP_EXT or name in SKIP_NAMES:
            continue
        if "\x00" in d.text[:4096]:  # binary content fetched as text
            continue
        out.append(d)
    log.info("filter: %d kept, %d skipped", len(out), len(docs) - len(out))
    return out


def transform_special_files(docs: list[Document]) -> list[Document]:
    out = []
    for d in docs:
        if d.metadata.get("file_path", "").endswith(".ipynb"):
            try:
                out.append(Document(process_notebook_text(d.text),
                                    {**d.metadata, "content_type": "notebook", "is_processed": True}, d.id))
            except Exception:
                log.warning("notebook transform failed for %s; keeping raw text", d.metadata.get("file_path"))
                out.append(d)
        else:
            out.append(d)
    return out


def language_of(path: str) -> str:
    name = path.split("/")[-1].lower()
    if name == "dockerfile":
        return "dockerfile"
    if "docker-compose" in name and name.endswith((".yml", ".yaml")):
        return "yaml"
    ext = _ext(path)
    return EXTENSION_TO_LANGUAGE.get(ext, ext.lstrip(".") or name)


def prepare_repo_documents(raw: list[Document]) -> list[Document]:
    docs = transform_special_files(filter_documents(raw))
    for d in docs:
        fp = (d.metadata.get("file_path") or "").strip()
        if fp and "language" not in d.metadata:
            d.metadata["language"] = language_of(fp)
    return docs


def infer_component_kind(docs: list[Document]) -> str:
    has_nb = has_manifest = has_openapi = False
    for d in docs:
        p = d.metadata.get("file_path", "").lower()
        has_nb |= p.endswith(".ipynb")
        has_manifest |= p.endswith(("package.json", "pyproject.toml", "pom.xml"))
        has_openapi |= p.endswith(("openapi.yaml", "openapi.yml", "openapi.json"))
    return "standalone" if has_nb and not (has_manifest or has_openapi) else "service"


def top_directory(path: str, depth: int = 1) -> str:
    parts = [x for x in PurePosixPath(path or "").parts if x not in (".", "")]
    return "/".join(parts[:depth]) if parts else ""


def group_nodes_by_file(nodes) -> dict:
    by = defaultdict(list)
    for n in nodes:
        by[(n.metadata.get("file_path") or n.metadata.get("path") or "").strip()].append(n)
    return by


def group_files_by_module(paths, depth: int = 1) -> dict:
    by = defaultdict(list)
    for p in paths:
        by[top_directory(p, depth)].append(p)
    return by
