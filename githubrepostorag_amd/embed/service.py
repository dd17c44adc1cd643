"""Embedding service: the reference's ``HuggingFaceEmbeddings.embed_query /
embed_documents`` (graph_rag_retrievers.py:53, vector_write_service.py:117)
on the GPU encoder.  Documents are length-sorted and packed into token-budget
batches (varlen: no padding compute), truncated to the model's
``max_seq_length`` like sentence-transformers does."""
from __future__ import annotations

import contextlib
import os
import threading

import torch

from ..engine.tokenizer import WordPieceTokenizer
from ..ops.gemm import WS
from ..utils.gpu_guard import gpu_guard, gpu_shared, set_device_of, side_stream
from ..models.configs import EncoderConfig, encoder_config
from ..models.encoder import BertEncoder, EncoderGraphs


class Embedder:
    def __init__(self, encoder: BertEncoder, tokenizer: WordPieceTokenizer | None = None,
                 max_tokens_per_batch: int = 65536, max_batch: int = 1024):
        self.encoder = encoder
        self.cfg: EncoderConfig = encoder.cfg
        self.tok = tokenizer or WordPieceTokenizer(self.cfg.vocab_size)
        self.max_tokens = max_tokens_per_batch
        self.max_batch = max_batch
        self.dim = self.cfg.hidden_size
        self.lock = threading.Lock()  # one encoder stream at a time
        self.stats = {"texts": 0, "tokens": 0, "graph_batches": 0}
        # query-sized batches replay captured encoder graphs (GRAG_ENCODER_GRAPHS=0: eager)
        self.graphs = (EncoderGraphs(encoder) if encoder.device.type == "cuda"
                       and os.environ.get("GRAG_ENCODER_GRAPHS", "1") != "0" else None)
        # The encoder's launches -- eager batches, graph captures and replays, from whichever thread embeds --
        # all go to ONE stream the embedder owns, with split-K slabs / stream-K tickets it owns (ops/gemm.py
        # WS.owned_by): a captured bucket graph and the eager batches that share its workspace are then
        # ordered by that stream instead of racing on two callers' streams.  Callers' streams wait on an event.
        self._ws: dict = {}
        self._stream = None

    @classmethod
    def from_name(cls, name: str, device="cuda", seed: int = 0, **kw) -> "Embedder":
        cfg = encoder_config(name)
        return cls(BertEncoder(cfg, device=device, seed=seed), WordPieceTokenizer(cfg.vocab_size), **kw)

    def tokenize(self, texts: list[str], prefix: str = "") -> list[list[int]]:
        L = min(self.cfg.max_seq_length, self.cfg.max_position)
        return [self.tok.encode(prefix + (t or ""), L) for t in texts]

    @contextlib.contextmanager
    def _on_encoder(self):
        """The embedder's stream and workspace owner for the block (the caller holds ``self.lock``); the
        caller's stream waits for the block's work on exit (an event, no host sync)."""
        dev = self.encoder.device
        if dev.type != "cuda":
            yield None
            return
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        if self._stream is None:
            lo, hi = torch.cuda.Stream.priority_range()  # latency-bound query embedding: high priority
            self._stream = torch.cuda.Stream(device=dev, priority=min(lo, hi))
        caller = torch.cuda.current_stream(dev)
        with torch.cuda.stream(self._stream), WS.owned_by(self._ws):
            yield self._stream
        if caller != self._stream:
            caller.wait_stream(self._stream)

    @torch.inference_mode()
    def embed_ids(self, ids: list[list[int]]) -> torch.Tensor:
        """-> bf16 [n, d] L2-normalised on the encoder's device (input order), ready on the caller's stream."""
        n = len(ids)
        if n == 0:
            return torch.empty(0, self.dim, dtype=torch.bfloat16, device=self.encoder.device)
        if self.graphs is not None and n <= EncoderGraphs.B_BUCKETS[-1]:
            bk = self.graphs.bucket_for(ids)
            if bk is not None and not self.graphs.has(bk):
                with gpu_guard(), self.lock, self._on_encoder():  # capture: exclusive
                    self.graphs.capture(*bk)
            with gpu_shared(), self.lock:
                with self._on_encoder():
                    r = self.graphs.run(ids, allow_capture=False)
                    if r is not None:
                        # allocated on the embedder's stream, which also writes it; the caller's stream waits
                        # for that stream, and record_stream keeps the block from being reused on the
                        # embedder's stream before the caller is done with it
                        out = r[1].clone()
                if r is not None:
                    if out.is_cuda:
                        out.record_stream(torch.cuda.current_stream(out.device))
                    self.stats["graph_batches"] += 1
                    self.stats["tokens"] += sum(len(x) for x in ids)
                    self.stats["texts"] += n
                    return out
        order = sorted(range(n), key=lambda i: len(ids[i]))
        with gpu_shared(), self.lock:
            with self._on_encoder():
                out = torch.empty(n, self.dim, dtype=torch.bfloat16, device=self.encoder.device)
                i = 0
                while i < n:
                    j, tok = i, 0
                    while j < n and j - i < self.max_batch and (tok + len(ids[order[j]]) <= self.max_tokens
                                                                or j == i):
                        tok += len(ids[order[j]])
                        j += 1
                    idx = order[i:j]
                    _, vb = self.encoder.encode_ids([ids[t] for t in idx], want_bf16=True)
                    out[torch.as_tensor(idx, device=out.device)] = vb
                    self.stats["tokens"] += tok
                    i = j
            if out.is_cuda:
                out.record_stream(torch.cuda.current_stream(out.device))
        self.stats["texts"] += n
        return out

    def embed_documents(self, texts: list[str]) -> torch.Tensor:
        return self.embed_ids(self.tokenize(texts))

    def embed_queries(self, texts: list[str]) -> torch.Tensor:
        ids = self.tokenize(texts, self.cfg.query_prefix)
        b = self._batcher
        if b is not None:
            return b.submit(ids)
        return self.embed_ids(ids)

    def embed_query(self, text: str) -> torch.Tensor:
        return self.embed_queries([text])[0]

    _batcher = None

    def enable_batching(self, window_s: float = 0.001, max_texts: int = 256) -> None:
        """Coalesce concurrent query embeddings (the service's job threads each
        embed one query per retriever hop) into one varlen encoder pass:
        64 concurrent jobs cost one launch sequence instead of 64."""
        if self._batcher is None:
            self._batcher = _QueryBatcher(self, window_s, max_texts)

    def close(self) -> None:
        if self._batcher is not None:
            self._batcher.stop()
            self._batcher = None


class _QueryBatcher:
    """One worker thread gathers query-embedding requests for ``window_s``
    after the first arrives (or until ``max_texts``), runs them as a single
    ``embed_ids`` call on its own side stream, synchronises that stream and
    hands every caller its rows (complete in memory, so any stream may read
    them)."""

    def __init__(self, emb: Embedder, window_s: float, max_texts: int):
        import queue

        self.emb, self.window, self.max_texts = emb, window_s, max_texts
        self.q: "queue.Queue" = queue.Queue()
        self.batches = 0
        self.texts = 0
        self._stop = False
        self._t = threading.Thread(target=self._loop, name="embed-batcher", daemon=True)
        self._t.start()

    def submit(self, ids: list[list[int]]) -> torch.Tensor:
        from concurrent.futures import Future

        f: Future = Future()
        self.q.put((ids, f))
        out = f.result()
        if out.is_cuda:  # the rows live in the batcher stream's pool: keep them until this stream is done
            out.record_stream(torch.cuda.current_stream(out.device))
        return out

    def stop(self) -> None:
        self._stop = True
        self.q.put(None)
        self._t.join(timeout=5)

    def _loop(self) -> None:
        import queue
        import time

        if self.emb.encoder.device.type == "cuda":
            set_device_of(self.emb.encoder.device)
        while not self._stop:
            first = self.q.get()
            if first is None:
                break
            items = [first]
            n = len(first[0])
            t_end = time.perf_counter() + self.window
            while n < self.max_texts:
                left = t_end - time.perf_counter()
                if left <= 0:
                    break
                try:
                    it = self.q.get(timeout=left)
                except queue.Empty:
                    break
                if it is None:
                    self._stop = True
                    break
                items.append(it)
                n += len(it[0])
            try:
                flat = [x for ids, _ in items for x in ids]
                with side_stream(self.emb.encoder.device):
                    out = self.emb.embed_ids(flat)
                    if out.is_cuda:
                        with gpu_shared():  # the sync must not land inside a graph capture
                            torch.cuda.current_stream(out.device).synchronize()
                self.batches += 1
                self.texts += len(flat)
                o = 0
                for ids, f in items:
                    f.set_result(out[o:o + len(ids)])
                    o += len(ids)
            except BaseException as e:  # fail the callers, keep serving
                for _, f in items:
                    if not f.done():
                        f.set_exception(e)
