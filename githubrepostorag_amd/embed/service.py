"""Embedding service: the reference's ``HuggingFaceEmbeddings.embed_query /
embed_documents`` (graph_rag_retrievers.py:53, vector_write_service.py:117)
on the GPU encoder.  Documents are length-sorted and packed into token-budget
batches (varlen: no padding compute), truncated to the model's
``max_seq_length`` like sentence-transformers does."""
from __future__ import annotations

import threading

import torch

from ..engine.tokenizer import WordPieceTokenizer
from ..utils.gpu_guard import guarded, side_stream
from ..models.configs import EncoderConfig, encoder_config
from ..models.encoder import BertEncoder


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
        self.stats = {"texts": 0, "tokens": 0}

    @classmethod
    def from_name(cls, name: str, device="cuda", seed: int = 0, **kw) -> "Embedder":
        cfg = encoder_config(name)
        return cls(BertEncoder(cfg, device=device, seed=seed), WordPieceTokenizer(cfg.vocab_size), **kw)

    def tokenize(self, texts: list[str], prefix: str = "") -> list[list[int]]:
        L = min(self.cfg.max_seq_length, self.cfg.max_position)
        return [self.tok.encode(prefix + (t or ""), L) for t in texts]

    @guarded
    @torch.inference_mode()
    def embed_ids(self, ids: list[list[int]]) -> torch.Tensor:
        """-> bf16 [n, d] L2-normalised on the encoder's device (input order)."""
        n = len(ids)
        out = torch.empty(n, self.dim, dtype=torch.bfloat16, device=self.encoder.device)
        if n == 0:
            return out
        order = sorted(range(n), key=lambda i: len(ids[i]))
        with self.lock, side_stream(self.encoder.device):
            i = 0
            while i < n:
                j, tok = i, 0
                while j < n and j - i < self.max_batch and (tok + len(ids[order[j]]) <= self.max_tokens or j == i):
                    tok += len(ids[order[j]])
                    j += 1
                idx = order[i:j]
                _, vb = self.encoder.encode_ids([ids[t] for t in idx], want_bf16=True)
                out[torch.as_tensor(idx, device=out.device)] = vb
                self.stats["tokens"] += tok
                i = j
        self.stats["texts"] += n
        return out

    def embed_documents(self, texts: list[str]) -> torch.Tensor:
        return self.embed_ids(self.tokenize(texts))

    def embed_queries(self, texts: list[str]) -> torch.Tensor:
        return self.embed_ids(self.tokenize(texts, self.cfg.query_prefix))

    def embed_query(self, text: str) -> torch.Tensor:
        return self.embed_queries([text])[0]
