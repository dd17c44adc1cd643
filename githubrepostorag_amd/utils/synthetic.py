"""Deterministic synthetic data (no network on the GPU box): code-repo files,
chunk texts addressed by id (so a 10M-row index needs no host text store),
questions, and clustered embedding matrices for index benchmarks."""
from __future__ import annotations

import random

import torch

_WORDS = ("cache retry broker session token config handler queue worker index vector embed chunk module "
          "service client request response timeout reconnect policy schema table stream event job cancel "
          "health metrics summary parser splitter encoder decoder attention kernel batch shard gather merge "
          "repository branch commit pipeline deploy helm redis cassandra graph traverse scope file package").split()
_LANGS = (("py", "python"), ("java", "java"), ("ts", "typescript"), ("go", "go"), ("md", "markdown"),
          ("yaml", "yaml"), ("sql", "sql"))


def _rng(seed: int) -> random.Random:
    return random.Random(seed * 2654435761 % (1 << 32))


def words(r: random.Random, n: int) -> str:
    return " ".join(r.choice(_WORDS) for _ in range(n))


def code_file(r: random.Random, ext: str, n_funcs: int = 4) -> str:
    out = []
    for f in range(n_funcs):
        name = f"{r.choice(_WORDS)}_{r.choice(_WORDS)}_{f}"
        if ext == "py":
            out.append(f"def {name}(self, {r.choice(_WORDS)}, timeout=30):\n    \"\"\"{words(r, 12)}.\"\"\"\n"
                       f"    result = self.{r.choice(_WORDS)}.{r.choice(_WORDS)}({r.choice(_WORDS)})\n"
                       f"    if result is None:\n        raise RuntimeError('{words(r, 5)}')\n    return result\n")
        elif ext == "java":
            out.append(f"public class {name.title().replace('_', '')} {{\n  // {words(r, 10)}\n"
                       f"  public void {name}(String {r.choice(_WORDS)}) {{ log.info(\"{words(r, 4)}\"); }}\n}}\n")
        elif ext == "ts":
            out.append(f"export function {name}(opts: Options): Promise<Result> {{\n  // {words(r, 10)}\n"
                       f"  return client.{r.choice(_WORDS)}(opts).then((r) => r.{r.choice(_WORDS)});\n}}\n")
        elif ext == "go":
            out.append(f"func {name.title().replace('_', '')}(ctx context.Context) error {{\n\t// {words(r, 10)}\n"
                       f"\treturn nil\n}}\n")
        elif ext == "md":
            out.append(f"## {words(r, 3).title()}\n\n{words(r, 40)}.\n")
        elif ext == "yaml":
            out.append(f"{r.choice(_WORDS)}:\n  {r.choice(_WORDS)}: {r.randint(1, 100)}\n  name: {words(r, 2)}\n")
        else:
            out.append(f"SELECT {r.choice(_WORDS)}, {r.choice(_WORDS)} FROM {r.choice(_WORDS)} WHERE id = {f};\n")
    return "\n".join(out)


def synthetic_repo(seed: int, n_files: int = 24, repo: str | None = None) -> tuple[str, list[dict]]:
    """-> (repo name, [{"file_path", "text"}]) with a README, modules and a notebook."""
    r = _rng(seed)
    repo = repo or f"{r.choice(_WORDS)}-{r.choice(_WORDS)}-{seed}"
    files = [{"file_path": "README.md",
              "text": f"# {repo}\n\nThis service handles {words(r, 30)}.\n\n## Usage\n\n{words(r, 40)}.\n"}]
    mods = [r.choice(_WORDS) for _ in range(max(1, n_files // 6))]
    for i in range(n_files - 1):
        ext, _ = _LANGS[i % len(_LANGS)]
        mod = mods[i % len(mods)]
        files.append({"file_path": f"{mod}/{r.choice(_WORDS)}_{i}.{ext}", "text": code_file(r, ext, 3 + i % 4)})
    files.append({"file_path": "LICENSE", "text": "MIT License\n" + words(r, 50)})
    files.append({"file_path": "assets/logo.png", "text": "\x89PNG binary"})
    return repo, files


def chunk_text(doc_id: int, n_chars: int = 800) -> str:
    """Text of synthetic index row `doc_id` (regenerated on demand)."""
    r = _rng(doc_id + 1)
    out = []
    while sum(len(x) + 1 for x in out) < n_chars:
        out.append(code_file(r, _LANGS[r.randrange(len(_LANGS))][0], 1))
    return "\n".join(out)[:n_chars]


def question(i: int) -> str:
    r = _rng(10_000_019 + i)
    return (f"How does the {r.choice(_WORDS)} {r.choice(_WORDS)} handle {r.choice(_WORDS)} "
            f"{r.choice(_WORDS)} when the {r.choice(_WORDS)} {r.choice(_WORDS)} times out?")


@torch.inference_mode()
def clustered_vectors(n: int, d: int, n_centers: int = 4096, noise: float = 0.35, seed: int = 0,
                      device="cuda", chunk: int = 1 << 20, center_seed: int | None = None) -> torch.Tensor:
    """bf16 [n, d] unit vectors drawn around random unit centres.  ``center_seed``: draw the centres from
    their own seed, so the shards of one corpus (one ``seed`` per rank) share ONE set of clusters -- with
    per-shard centres a W-way sharded corpus would hold W x n_centers clusters and a fixed nlist would
    cover W times as many clusters per list as on one GPU."""
    g = torch.Generator(device=device)
    g.manual_seed(seed if center_seed is None else center_seed)
    C = torch.randn(n_centers, d, generator=g, device=device)
    if center_seed is not None and center_seed != seed:  # (center_seed == seed: one stream, as without it)
        g.manual_seed(seed)
    C = C / C.norm(dim=1, keepdim=True)
    out = torch.empty(n, d, dtype=torch.bfloat16, device=device)
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        c = torch.randint(0, n_centers, (m,), generator=g, device=device)
        x = C[c] + noise * torch.randn(m, d, generator=g, device=device) / d ** 0.5
        out[s:s + m] = (x / x.norm(dim=1, keepdim=True)).to(torch.bfloat16)
    return out


class SyntheticCorpus:
    """Virtual rows of a vector table (index/store.py ``RowStore`` segments): row i
    of a bulk-loaded synthetic corpus gets a deterministic row_id, chunk text and
    metadata (namespace / repo / module / file_path / language / scope), so a
    10M-row table carries its host rows as a recipe instead of 10M objects.
    ``columns(n, device)`` returns the matching dictionary-coded filter columns."""

    def __init__(self, n: int, seed: int = 0, n_repos: int = 64, n_modules: int = 8, files_per_module: int = 64,
                 namespace: str = "default", scope: str = "chunk", text_chars: int = 800):
        self.n, self.seed = int(n), int(seed)
        self.n_repos, self.n_modules, self.fpm = n_repos, n_modules, files_per_module
        self.namespace, self.scope, self.text_chars = namespace, scope, text_chars
        self.prefix = f"syn{self.seed}-"

    def spec(self) -> dict:
        return {"kind": "synthetic", "n": self.n, "seed": self.seed, "n_repos": self.n_repos,
                "n_modules": self.n_modules, "files_per_module": self.fpm, "namespace": self.namespace,
                "scope": self.scope, "text_chars": self.text_chars}

    # row i -> (repo, module, file, language) indices
    def _parts(self, i: int):
        repo = i % self.n_repos
        mod = (i // self.n_repos) % self.n_modules
        f = (i // (self.n_repos * self.n_modules)) % self.fpm
        return repo, mod, f, (repo + mod + f) % len(_LANGS)

    def repo_name(self, j: int) -> str:
        return f"{_WORDS[j % len(_WORDS)]}-{_WORDS[(j * 7 + 3) % len(_WORDS)]}-{j}"

    def module_name(self, j: int) -> str:
        return _WORDS[(j * 5 + 1) % len(_WORDS)] + f"{j}"

    def row_id(self, i: int) -> str:
        return f"{self.prefix}{i}"

    def index_of(self, row_id: str):
        if not row_id.startswith(self.prefix):
            return None
        try:
            return int(row_id[len(self.prefix):])
        except ValueError:
            return None

    def text(self, i: int) -> str:
        return chunk_text(self.seed * 1_000_003 + i, self.text_chars)

    def meta(self, i: int) -> dict:
        repo, mod, f, lang = self._parts(i)
        ext, language = _LANGS[lang]
        m = self.module_name(mod)
        return {"namespace": self.namespace, "repo": self.repo_name(repo), "module": m,
                "file_path": f"{m}/{_WORDS[f % len(_WORDS)]}_{f}.{ext}", "language": language,
                "scope": self.scope, "doc_type": self.scope}

    def register(self, table) -> None:
        """Register every dictionary value this corpus uses, in a fixed order, so
        ``columns`` can encode rows arithmetically."""
        self._codes = {}
        for fld, vals in (("namespace", [self.namespace]), ("scope", [self.scope]), ("doc_type", [self.scope]),
                          ("repo", [self.repo_name(j) for j in range(self.n_repos)]),
                          ("module", [self.module_name(j) for j in range(self.n_modules)]),
                          ("language", [lang for _, lang in _LANGS])):
            self._codes[fld] = torch.tensor([table._code(fld, v) for v in vals], dtype=torch.int32)
        fp = []
        for mod in range(self.n_modules):
            for f in range(self.fpm):
                for lang in range(len(_LANGS)):
                    m = self.module_name(mod)
                    fp.append(table._code("file_path", f"{m}/{_WORDS[f % len(_WORDS)]}_{f}.{_LANGS[lang][0]}"))
        self._codes["file_path"] = torch.tensor(fp, dtype=torch.int32)

    def columns(self, device) -> dict:
        i = torch.arange(self.n, device=device, dtype=torch.int64)
        repo = i % self.n_repos
        mod = (i // self.n_repos) % self.n_modules
        f = (i // (self.n_repos * self.n_modules)) % self.fpm
        lang = (repo + mod + f) % len(_LANGS)
        c = {k: v.to(device) for k, v in self._codes.items()}
        return {"namespace": c["namespace"][torch.zeros_like(i)], "scope": c["scope"][torch.zeros_like(i)],
                "doc_type": c["doc_type"][torch.zeros_like(i)], "repo": c["repo"][repo], "module": c["module"][mod],
                "language": c["language"][lang],
                "file_path": c["file_path"][(mod * self.fpm + f) * len(_LANGS) + lang]}


def provider_from_spec(spec: dict):
    if spec.get("kind") == "shard":
        from ..index.sharded import ShardView

        return ShardView(provider_from_spec(spec["corpus"]), spec["rank"], spec["world"])
    if spec.get("kind") == "synthetic":
        kw = {k: v for k, v in spec.items() if k not in ("kind", "n", "seed")}
        kw["files_per_module"] = kw.pop("files_per_module", 64)
        return SyntheticCorpus(spec["n"], spec["seed"], **kw)
    raise ValueError(f"unknown virtual row provider {spec!r}")


def code_question(i: int) -> str:
    """A debugging-style question: the agent's planner routes it to the code scope
    (agent_graph.py:33-38 keyword fallback), so every refinement round searches
    the chunk table."""
    r = _rng(20_000_033 + i)
    return (f"Why does {r.choice(_WORDS)}_{r.choice(_WORDS)} raise an exception on retry when the "
            f"{r.choice(_WORDS)} {r.choice(_WORDS)} hits a timeout?")


def scope_rows(corpus: SyntheticCorpus, scope: str) -> tuple[list[str], list[str], list[dict]]:
    """The hierarchy-summary rows (ingest/hierarchy.py's repo / module / file documents) that an
    ingest of ``corpus``'s chunks would have produced: one REPO OVERVIEW per repo, one MODULE
    SUMMARY per (repo, module), one FILE SUMMARY per (repo, module, file) — the project /
    package / file tables the agent's scope retrievers search (reference agent_graph.py:158-176)."""
    ids, texts, metas = [], [], []
    langs = _LANGS
    for rp in range(corpus.n_repos):
        repo = corpus.repo_name(rp)
        base = {"namespace": corpus.namespace, "repo": repo}
        if scope == "repo":
            r = _rng(corpus.seed * 7919 + rp)
            ids.append(f"{corpus.prefix}repo-{rp}")
            texts.append(f"REPO OVERVIEW {repo}: this project handles {words(r, 40)}.")
            metas.append({**base, "scope": "repo", "doc_type": "repo"})
            continue
        for md in range(corpus.n_modules):
            m = corpus.module_name(md)
            if scope == "module":
                r = _rng(corpus.seed * 7919 + rp * 131 + md)
                ids.append(f"{corpus.prefix}module-{rp}-{md}")
                texts.append(f"MODULE SUMMARY {repo}/{m}: {words(r, 30)}.")
                metas.append({**base, "module": m, "scope": "module", "doc_type": "module"})
                continue
            for f in range(corpus.fpm):
                ext = langs[(rp + md + f) % len(langs)][0]
                fp = f"{m}/{_WORDS[f % len(_WORDS)]}_{f}.{ext}"
                r = _rng(corpus.seed * 7919 + (rp * 131 + md) * 4099 + f)
                ids.append(f"{corpus.prefix}file-{rp}-{md}-{f}")
                texts.append(f"FILE SUMMARY {fp}: {words(r, 20)}.")
                metas.append({**base, "module": m, "file_path": fp, "scope": "file", "doc_type": "file",
                              "language": langs[(rp + md + f) % len(langs)][1]})
    return ids, texts, metas


def overview_question(i: int, corpus: SyntheticCorpus) -> str:
    """A project-level question: the planner falls back to the project scope (no code keywords), and
    the judge's stage-down walks project -> package -> file (agent_graph.py:346-378)."""
    r = _rng(30_000_041 + i)
    repo = corpus.repo_name(r.randrange(corpus.n_repos))
    return (f"Tell me about the {repo} project: how are its {r.choice(_WORDS)} and {r.choice(_WORDS)} "
            f"parts organised?")
