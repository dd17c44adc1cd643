"""Prompt-token audit of the bench's agent phase (no model, no GPU): the real GraphAgent (plan -> retrieve ->
judge -> rewrite -> synthesize, reference prompts) over an in-memory store of the bench's synthetic corpus
(chunk table + repo / module / file summary rows, random unit vectors) with a fake LLM that answers every
call with random text of exactly its token cap (what random-init weights do: JSON never parses, so the
fallbacks run as in the bench).  Reports per call purpose the prompt tokens and what an IDEAL block prefix
cache (16-token blocks, chained hashes, unbounded, submission order) would still prefill, and the shared
prefix between consecutive calls of the same job -- the floor for the engine's prefix_hit_tokens in
agent_e2e.engine.

python scripts/agent_token_audit.py [--jobs 256] [--out profiles/agent_token_audit_r5.json]
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from githubrepostorag_amd.agent.graph_agent import GraphAgent  # noqa: E402
from githubrepostorag_amd.agent.llm import EngineLLM  # noqa: E402
from githubrepostorag_amd.engine.tokenizer import load_tokenizer  # noqa: E402
from githubrepostorag_amd.index.store import VectorStore  # noqa: E402
from githubrepostorag_amd.retrieval.graph import RetrieverFactory  # noqa: E402
from githubrepostorag_amd.utils import synthetic  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ingest_token_audit import FakeRunner, ideal_unique  # noqa: E402

PURPOSE = (("Choose the best search scope", "plan"), ("Generate 3-4", "expand"), ("Judge if", "judge"),
           ("Rewrite this", "rewrite"), ("You are a helpful developer assistant", "synthesize_retry"),
           ("You are a senior developer assistant", "synthesize"))


def purpose_of(prompt: str) -> str:
    for pre, name in PURPOSE:
        if pre in prompt:  # (judge / synthesize prompts lead with the shared context blocks)
            return name
    return "other"


class _Emb:
    dim = 64

    def __init__(self):
        self.g = torch.Generator().manual_seed(3)

    def embed_queries(self, texts, **kw):
        return torch.nn.functional.normalize(torch.randn(len(texts), self.dim, generator=self.g), dim=1)

    embed_documents = embed_queries

    def embed_query(self, text):
        return self.embed_queries([text])[0]


def build_store(rows: int, emb: _Emb):
    corpus = synthetic.SyntheticCorpus(rows, seed=7)
    store = VectorStore(emb.dim, "cpu")
    ids = [corpus.row_id(i) for i in range(rows)]
    store.table("chunk").upsert(ids, [corpus.text(i) for i in range(rows)], emb.embed_documents(ids),
                                [corpus.meta(i) for i in range(rows)])
    for scope in ("repo", "module", "file"):
        sid, texts, metas = synthetic.scope_rows(corpus, scope)
        store.table(scope).upsert(sid, texts, emb.embed_documents(sid), metas)
    return corpus, store


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=256)
    ap.add_argument("--rows", type=int, default=20000)
    ap.add_argument("--gen-len", type=int, default=32)
    ap.add_argument("--synth-len", type=int, default=256)
    ap.add_argument("--vocab", type=int, default=152064)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    tok = load_tokenizer(None, a.vocab)
    runner = FakeRunner(tok, a.vocab)
    runner.engine.cfg.max_model_len = 4096  # the bench's serving engine
    llm = EngineLLM(runner, tok, max_tokens=a.gen_len, mode="worker", retries=0)
    emb = _Emb()
    corpus, store = build_store(a.rows, emb)
    rf = RetrieverFactory(store, emb)
    per_job, purposes = [], []
    for i in range(a.jobs):
        q = synthetic.code_question(50_000_000 + i) if i % 2 == 0 else \
            synthetic.overview_question(50_000_000 + i, corpus)
        n0 = len(runner.calls)
        agent = GraphAgent(llm, rf.scope_retrievers(), namespace=corpus.namespace, synth_max_tokens=a.synth_len)
        agent.run(q)
        per_job.append((n0, len(runner.calls)))
    # purposes, recovered from the prompt text (the fake runner only sees token ids)
    for ids, _ in runner.calls:
        purposes.append(purpose_of(tok.decode(ids)))
    uniq = ideal_unique(runner.calls)
    by = collections.defaultdict(lambda: [0, 0, 0])
    for (ids, _), u, p in zip(runner.calls, uniq, purposes):
        r = by[p]
        r[0] += 1
        r[1] += len(ids)
        r[2] += u
    # the same ideal cache, restricted to each job's own calls (what sharing WITHIN a job is worth)
    within = 0
    for a0, a1 in per_job:
        within += sum(ideal_unique(runner.calls[a0:a1]))
    tot = sum(len(i) for i, _ in runner.calls)
    res = {"jobs": a.jobs, "llm_calls": len(runner.calls), "calls_per_job": round(len(runner.calls) / a.jobs, 2),
           "prompt_tokens": tot, "prompt_tokens_per_job": round(tot / a.jobs, 1),
           "ideal_prefill_tokens": sum(uniq), "ideal_prefix_hit_share": round(1 - sum(uniq) / max(1, tot), 4),
           "ideal_prefill_tokens_within_jobs_only": within,
           "by_purpose": {k: {"calls": v[0], "prompt_tokens": v[1], "ideal_prefill_tokens": v[2],
                              "mean_prompt_tokens": round(v[1] / max(1, v[0]), 1)} for k, v in sorted(by.items())}}
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    random.seed(0)
    main()
