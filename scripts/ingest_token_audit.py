"""Prompt-token audit of the bench's ingest (no model, no GPU): the FULL ingest pipeline on the 192-file
synthetic repo with a fake engine runner that answers every call with random text of exactly its token cap
(what random-init weights do), recording every prompt's token ids in submission order.  Reports per call
kind (by token cap) the prompt tokens and the tokens an IDEAL block-granular prefix cache (16-token blocks,
chained hashes, unbounded, no timing) would still have to prefill -- the floor for the engine's
``prefill_tokens`` in the bench JSON (its ``prefix_hit_tokens`` is what the real cache saved).

python scripts/ingest_token_audit.py [--files 192] [--out profiles/ingest_token_audit_r4.json]
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import random
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from githubrepostorag_amd.agent.llm import EngineLLM  # noqa: E402
from githubrepostorag_amd.config import Settings  # noqa: E402
from githubrepostorag_amd.engine.sequence import Completion  # noqa: E402
from githubrepostorag_amd.engine.tokenizer import load_tokenizer  # noqa: E402
from githubrepostorag_amd.ingest.controller import IngestController  # noqa: E402
from githubrepostorag_amd.ingest.readers import Document  # noqa: E402
from githubrepostorag_amd.utils.synthetic import synthetic_repo  # noqa: E402

BS = 16


class _Handle:
    def __init__(self, c):
        self.c = c
        self.done = threading.Event()
        self.done.set()

    def wait(self, timeout=None):
        return self.c

    def cancel(self):
        pass


class _Cfg:
    max_model_len = 8192


class _Eng:
    cfg = _Cfg()


class FakeRunner:
    engine = _Eng()

    def __init__(self, tok, vocab):
        self.tok, self.vocab = tok, vocab
        self.rng = random.Random(0)
        self.calls = []  # (ids, max_tokens)
        self.lock = threading.Lock()

    def submit(self, ids, sp, on_token=None, interactive=True):
        ids = list(ids) if not isinstance(ids, str) else self.tok.encode(ids)
        out = [self.rng.randrange(256, self.vocab - 1) for _ in range(sp.max_tokens)]
        with self.lock:
            self.calls.append((ids, sp.max_tokens))
        return _Handle(Completion("x", self.tok.decode(out), out, "length", len(ids), 0.0, 0.0))

    def generate(self, ids, sp, on_token=None, timeout=None):
        return self.submit(ids, sp).wait()


def ideal_unique(calls):
    """Tokens an unbounded block cache still prefills (chained block hashes, submission order; the last
    prompt token is always computed, as in the engine's match_prefix)."""
    seen = set()
    out = []
    for ids, _ in calls:
        usable = (len(ids) - 1) // BS
        h = 0
        hit = 0
        for b in range(usable):
            h = hash((h, tuple(ids[b * BS:(b + 1) * BS])))
            if h in seen:
                hit += 1
            else:
                break
        # register every full block of this prompt
        h = 0
        for b in range(len(ids) // BS):
            h = hash((h, tuple(ids[b * BS:(b + 1) * BS])))
            seen.add(h)
        out.append(len(ids) - hit * BS)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=192)
    ap.add_argument("--vocab", type=int, default=152064)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    tok = load_tokenizer(None, a.vocab)
    runner = FakeRunner(tok, a.vocab)
    llm = EngineLLM(runner, tok, max_tokens=128, mode="ingest", timeout_s=3600.0, retries=0)

    class _Emb:
        dim = 32

        def embed_documents(self, texts, **kw):
            import torch

            return torch.nn.functional.normalize(torch.randn(len(texts), 32), dim=1)

        embed_queries = embed_documents

    from githubrepostorag_amd.index.store import VectorStore

    ctl = IngestController(llm=llm, store=VectorStore(32, "cpu"), embedder=_Emb(), settings=Settings(data_dir=None),
                           summary_tokens=128)
    _, files = synthetic_repo(0, a.files, "bench-repo-0")
    docs = [Document(f["text"], {"file_path": f["file_path"], "file_name": f["file_path"].split("/")[-1]})
            for f in files]
    t0 = time.perf_counter()
    ctl.ingest_component(repo="bench-repo-0", namespace="bench", documents=docs, force=True)
    calls = runner.calls
    uniq = ideal_unique(calls)
    by = collections.defaultdict(lambda: [0, 0, 0, 0])
    for (ids, mt), u in zip(calls, uniq):
        r = by[mt]
        r[0] += 1
        r[1] += len(ids)
        r[2] += u
        r[3] += mt
    res = {"files": a.files, "llm_calls": len(calls), "prompt_tokens": sum(len(i) for i, _ in calls),
           "ideal_prefill_tokens": sum(uniq), "decode_tokens": sum(m for _, m in calls),
           "by_token_cap": {str(k): {"calls": v[0], "prompt_tokens": v[1], "ideal_prefill_tokens": v[2],
                                     "decode_tokens": v[3]} for k, v in sorted(by.items())},
           "seconds": round(time.perf_counter() - t0, 1)}
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
