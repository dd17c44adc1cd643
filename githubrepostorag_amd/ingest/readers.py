"""Document model and repository readers.

* ``GithubReader`` — the reference's LlamaIndex ``GithubRepositoryReader``
  (ingest/src/app/services/github_service.py:10-25): resolve the branch, list
  the recursive tree, fetch blobs (base64) with bounded concurrency (6), one
  Document per text file with ``file_path``/``file_name``/``url`` metadata;
  ``fetch_repositories`` = the GraphQL listing of a user's public, non-fork,
  non-archived repositories (github_service.py:28-79).
* ``LocalDirReader`` — same Documents from a checked-out directory.
* ``SyntheticRepoReader`` — deterministic repos (no network on GPU boxes).
"""
from __future__ import annotations

import base64
import logging
import os
import uuid
import zlib
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field
from pathlib import Path

log = logging.getLogger(__name__)


@dataclass
class Node:
    text: str
    metadata: dict = field(default_factory=dict)
    id: str = field(default_factory=lambda: uuid.uuid4().hex)

    def get_content(self) -> str:
        return self.text


Document = Node


def _doc(path: str, text: str, **md) -> Document:
    return Document(text, {"file_path": path, "file_name": path.split("/")[-1], **md})


class GithubReader:
    API = "https://api.github.com"

    def __init__(self, owner: str, token: str = "", concurrent_requests: int = 6, timeout: float = 60.0):
        self.owner = owner
        self.token = token
        self.concurrency = concurrent_requests
        self.timeout = timeout

    def _headers(self):
        h = {"Accept": "application/vnd.github+json"}
        if self.token:
            h["Authorization"] = f"Bearer {self.token}"
        return h

    def load_data(self, repo: str, branch: str = "main") -> list[Document]:
        import requests

        r = requests.get(f"{self.API}/repos/{self.owner}/{repo}/git/trees/{branch}?recursive=1",
                         headers=self._headers(), timeout=self.timeout)
        r.raise_for_status()
        blobs = [t for t in r.json().get("tree", []) if t.get("type") == "blob"]

        def fetch(t):
            try:
                b = requests.get(t["url"], headers=self._headers(), timeout=self.timeout)
                b.raise_for_status()
                raw = base64.b64decode(b.json().get("content", ""))
                try:
                    text = raw.decode("utf-8")
                except UnicodeDecodeError:
                    return None  # binary
                return _doc(t["path"], text, url=t.get("url", ""), repo=repo, branch=branch)
            except Exception as e:
                log.warning("blob fetch failed for %s: %s", t.get("path"), e)
                return None

        with ThreadPoolExecutor(max_workers=self.concurrency) as ex:
            return [d for d in ex.map(fetch, blobs) if d is not None]


def fetch_repositories(username: str, token: str, timeout: float = 30.0) -> list[str]:
    import requests

    query = """query($login: String!, $after: String) { user(login: $login) {
      repositories(first: 100, after: $after, isFork: false, privacy: PUBLIC) {
        pageInfo { endCursor hasNextPage } nodes { name isArchived isPrivate } } } }"""
    out, after = [], None
    while True:
        r = requests.post("https://api.github.com/graphql", json={"query": query,
                                                                  "variables": {"login": username, "after": after}},
                          headers={"Authorization": f"Bearer {token}"}, timeout=timeout)
        r.raise_for_status()
        data = r.json()["data"]["user"]["repositories"]
        out += [n["name"] for n in data["nodes"] if not n["isArchived"] and not n["isPrivate"]]
        if not data["pageInfo"]["hasNextPage"]:
            return out
        after = data["pageInfo"]["endCursor"]


class LocalDirReader:
    def __init__(self, root: str, max_file_bytes: int = 2_000_000):
        self.root = Path(root)
        self.max_file_bytes = max_file_bytes

    def load_data(self, repo: str | None = None, branch: str = "main") -> list[Document]:
        out = []
        for p in sorted(self.root.rglob("*")):
            if not p.is_file() or ".git" in p.parts or p.stat().st_size > self.max_file_bytes:
                continue
            try:
                text = p.read_text(encoding="utf-8")
            except (UnicodeDecodeError, OSError):
                continue
            out.append(_doc(str(p.relative_to(self.root)).replace(os.sep, "/"), text, repo=repo or self.root.name,
                            branch=branch))
        return out


class SyntheticRepoReader:
    def __init__(self, n_files: int = 24):
        self.n_files = n_files

    def load_data(self, repo: str, branch: str = "main", seed: int | None = None) -> list[Document]:
        from ..utils.synthetic import synthetic_repo

        seed = seed if seed is not None else zlib.crc32(repo.encode()) & 0x3FFFFFFF
        _, files = synthetic_repo(seed, self.n_files, repo)
        return [_doc(f["file_path"], f["text"], repo=repo, branch=branch) for f in files]
