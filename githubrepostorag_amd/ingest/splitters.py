"""Text and code splitters (reference call sites
ingest/src/app/langauge_detector.py:76-137, pipelines/code_pipeline.py:14-54,
pipelines/catalog_pipeline.py:17-18).

* ``SentenceSplitter(chunk_size, chunk_overlap)`` — token-budgeted: split by
  paragraph -> sentence -> word until every piece fits, greedily pack pieces
  up to ``chunk_size`` tokens, carry ``chunk_overlap`` tokens of trailing
  pieces into the next chunk; nodes keep start/end char offsets and the
  source document id.
* ``CodeSplitter(language, chunk_lines=200, chunk_lines_overlap=10,
  max_chars=4000)`` — structure-aware packing of top-level blocks (brace depth
  for C-family languages, indentation for Python-like ones, headings for
  markdown), recursing into blocks larger than ``max_chars``; unsupported
  languages raise ``LookupError`` so the caller falls back to
  ``SentenceSplitter(4000, 200)`` exactly like the reference.
* ``DynamicCodeSplitter`` — per-document splitter choice from the language
  detected from the path (notebooks: kernel language).
Token counts use a BPE-granularity regex (no tokenizer download needed).
"""
from __future__ import annotations

import json
import re
from pathlib import Path

from .readers import Document, Node

_TOK = re.compile(r"[A-Za-z]{1,8}|\d{1,3}|[^\sA-Za-z\d]")
_SENT = re.compile(r"[^,.;。？！?!\n]+[,.;。？！?!]?\s*|\n")


def count_tokens(s: str) -> int:
    return len(_TOK.findall(s))


class SentenceSplitter:
    def __init__(self, chunk_size: int = 1024, chunk_overlap: int = 200, paragraph_separator: str = "\n\n"):
        if chunk_overlap > chunk_size:
            raise ValueError("chunk_overlap > chunk_size")
        self.chunk_size = chunk_size
        self.chunk_overlap = chunk_overlap
        self.para = paragraph_separator

    def _pieces(self, text: str, budget: int) -> list[str]:
        if count_tokens(text) <= budget:
            return [text]
        for splitter in (lambda t: _keep_sep(t, self.para), lambda t: _SENT.findall(t),
                         lambda t: re.findall(r"\S+\s*|\s+", t)):
            parts = [p for p in splitter(text) if p]
            if len(parts) > 1:
                out = []
                for p in parts:
                    out.extend(self._pieces(p, budget))
                return out
        # a single huge token run: hard-cut by characters
        step = max(1, budget * 3)
        return [text[i:i + step] for i in range(0, len(text), step)]

    def split_text(self, text: str) -> list[tuple[str, int, int]]:
        if not text:
            return []
        pieces = self._pieces(text, self.chunk_size)
        chunks, cur, cur_tok = [], [], 0
        pos = 0
        spans = []
        for p in pieces:
            spans.append((p, pos, pos + len(p), count_tokens(p)))
            pos += len(p)
        i = 0
        while i < len(spans):
            cur, cur_tok = [], 0
            j = i
            while j < len(spans) and (cur_tok + spans[j][3] <= self.chunk_size or not cur):
                cur.append(spans[j])
                cur_tok += spans[j][3]
                j += 1
            s, e = cur[0][1], cur[-1][2]
            body = text[s:e].strip()
            if body:
                off = text.find(body, s)
                chunks.append((body, off, off + len(body)))
            if j >= len(spans):
                break
            # overlap: step back over trailing pieces worth <= chunk_overlap tokens
            back, tok = j, 0
            while back - 1 > i and tok + spans[back - 1][3] <= self.chunk_overlap:
                back -= 1
                tok += spans[back][3]
            i = back if back > i else j
        return chunks

    def get_nodes_from_documents(self, docs: list[Document]) -> list[Node]:
        out = []
        for d in docs:
            for body, s, e in self.split_text(d.text):
                out.append(Node(body, {**d.metadata, "start_char_idx": s, "end_char_idx": e, "source_doc_id": d.id}))
        return out


def _keep_sep(text: str, sep: str) -> list[str]:
    parts = text.split(sep)
    return [p + (sep if k < len(parts) - 1 else "") for k, p in enumerate(parts)]


BRACE_LANGS = {"java", "javascript", "typescript", "go", "c", "cpp", "c_sharp", "csharp", "rust", "kotlin", "scala",
               "swift", "php", "hip", "cuda", "groovy", "gradle", "protobuf"}
INDENT_LANGS = {"python", "yaml", "ruby"}
TEXT_LANGS = {"markdown"}
LINE_LANGS = {"bash", "sql", "json", "toml", "ini", "dockerfile", "html", "css", "xml"}


class CodeSplitter:
    def __init__(self, language: str, chunk_lines: int = 200, chunk_lines_overlap: int = 10, max_chars: int = 4000):
        lang = (language or "").lower()
        if lang not in BRACE_LANGS | INDENT_LANGS | TEXT_LANGS | LINE_LANGS:
            raise LookupError(f"no code grammar for language {language!r}")
        self.language = lang
        self.chunk_lines = chunk_lines
        self.overlap = chunk_lines_overlap
        self.max_chars = max_chars

    def _blocks(self, lines: list[str]) -> list[list[str]]:
        blocks, cur = [], []
        if self.language in BRACE_LANGS:
            depth = 0
            for ln in lines:
                cur.append(ln)
                code = re.sub(r"//.*|\"(?:\\.|[^\"])*\"|'(?:\\.|[^'])*'", "", ln)
                depth += code.count("{") - code.count("}")
                depth = max(depth, 0)
                if depth == 0 and (code.strip().endswith(("}", ";")) or not code.strip()):
                    blocks.append(cur)
                    cur = []
        elif self.language in INDENT_LANGS:
            for ln in lines:
                top = ln and not ln[0].isspace() and not ln.startswith((")", "]", "}"))
                starts_block = top and not (cur and cur[-1].rstrip().endswith(("\\", ",", "(")))
                if starts_block and cur and not (cur[-1].lstrip().startswith("@")):
                    blocks.append(cur)
                    cur = []
                cur.append(ln)
        elif self.language in TEXT_LANGS:
            for ln in lines:
                if ln.startswith("#") and cur:
                    blocks.append(cur)
                    cur = []
                cur.append(ln)
        else:
            for ln in lines:
                cur.append(ln)
                if not ln.strip():
                    blocks.append(cur)
                    cur = []
        if cur:
            blocks.append(cur)
        return [b for b in blocks if b]

    def _split_big(self, block: list[str]) -> list[list[str]]:
        """Descend into an oversized block: split at its inner blank lines /
        dedents, then by line count."""
        if len("\n".join(block)) <= self.max_chars and len(block) <= self.chunk_lines:
            return [block]
        out, cur, size = [], [], 0
        for ln in block:
            if cur and (size + len(ln) + 1 > self.max_chars or len(cur) >= self.chunk_lines):
                out.append(cur)
                cur, size = [], 0
            cur.append(ln)
            size += len(ln) + 1
        if cur:
            out.append(cur)
        return out

    def split_text(self, text: str) -> list[tuple[str, int, int]]:
        lines = text.split("\n")
        blocks = []
        for b in self._blocks(lines):
            blocks.extend(self._split_big(b))
        chunks, cur, size = [], [], 0
        for b in blocks:
            bsize = len("\n".join(b)) + 1
            if cur and (size + bsize > self.max_chars or len(cur) + len(b) > self.chunk_lines):
                chunks.append(cur)
                cur, size = [], 0
            cur = cur + b
            size += bsize
        if cur:
            chunks.append(cur)
        out, pos = [], 0
        for c in chunks:
            body = "\n".join(c).strip("\n")
            if not body.strip():
                continue
            s = text.find(body, pos)
            s = s if s >= 0 else pos
            out.append((body, s, s + len(body)))
            pos = s + len(body)
        return out

    def get_nodes_from_documents(self, docs: list[Document]) -> list[Node]:
        out = []
        for d in docs:
            for body, s, e in self.split_text(d.text):
                out.append(Node(body, {**d.metadata, "start_char_idx": s, "end_char_idx": e, "source_doc_id": d.id}))
        return out


EXT_TO_GRAMMAR = {".py": "python", ".js": "javascript", ".ts": "typescript", ".java": "java", ".cpp": "cpp",
                  ".c": "c", ".cs": "c_sharp", ".php": "php", ".rb": "ruby", ".go": "go", ".rs": "rust",
                  ".swift": "swift", ".kt": "kotlin", ".scala": "scala", ".sh": "bash", ".sql": "sql", ".html": "html",
                  ".css": "css", ".json": "json", ".xml": "xml", ".yaml": "yaml", ".yml": "yaml", ".md": "markdown",
                  ".dockerfile": "dockerfile", ".ipynb": "python", ".hip": "hip", ".cu": "cuda", ".tsx": "typescript",
                  ".jsx": "javascript", ".h": "c", ".hpp": "cpp"}


def detect_notebook_language(content: str) -> str:
    try:
        ks = (json.loads(content).get("metadata") or {}).get("kernelspec") or {}
        name, lang = ks.get("name", "").lower(), ks.get("language", "").lower()
        m = {"python3": "python", "python2": "python", "ir": "r", "scala": "scala", "julia": "julia",
             "javascript": "javascript", "typescript": "typescript"}
        if name in m:
            return m[name]
        if lang in ("python", "r", "scala", "julia", "javascript"):
            return lang
    except Exception:
        pass
    return "python"


def create_splitter(file_path: str | None, language: str | None = None, content: str | None = None):
    """The reference's ``create_code_splitter_safely`` semantics."""
    lang = language
    if lang in (None, "auto") and file_path:
        lang = EXT_TO_GRAMMAR.get(Path(file_path).suffix.lower())
        if file_path.endswith(".ipynb") and content:
            lang = detect_notebook_language(content)
    if not lang:
        return SentenceSplitter(4000, 200)
    try:
        return CodeSplitter(lang, chunk_lines=200, chunk_lines_overlap=10, max_chars=4000)
    except LookupError:
        return SentenceSplitter(4000, 200)


class DynamicCodeSplitter:
    def get_nodes_from_documents(self, docs: list[Document]) -> list[Node]:
        out = []
        for d in docs:
            fp = d.metadata.get("file_path") or d.metadata.get("path")
            lang = d.metadata.get("language")
            sp = create_splitter(fp, EXT_TO_GRAMMAR.get(Path(fp or "").suffix.lower()) if lang else None, d.text)
            out.extend(sp.get_nodes_from_documents([d]))
        return out
