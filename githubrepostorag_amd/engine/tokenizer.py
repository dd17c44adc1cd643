"""Tokenizers.

* ``ByteBPETokenizer`` — byte-level BPE on the native runtime (C++), trained
  offline from a built-in code/prose corpus when no vocabulary is available
  (the GPU box has no network), with Qwen ChatML special tokens.  When the
  model vocabulary is Qwen-sized the special tokens take Qwen's real ids
  (151643-151645) so prompts are laid out exactly as Qwen expects.
* ``HFTokenizer`` — loads a real ``tokenizer.json`` with the installed
  ``tokenizers`` wheel when a model directory provides one.
* ``WordPieceTokenizer`` — BERT WordPiece (C++) for the encoders; hashing
  mode when no ``vocab.txt`` is present.
"""
from __future__ import annotations

import codecs
import ctypes
import os
import threading
from pathlib import Path

import numpy as np

from ..utils.runtime import rt

IM_START, IM_END, ENDOFTEXT = "<|im_start|>", "<|im_end|>", "<|endoftext|>"
QWEN_SPECIAL_IDS = {ENDOFTEXT: 151643, IM_START: 151644, IM_END: 151645}

_BUILTIN_CORPUS = """
def retrieve(self, query, filters=None, k=10):
    docs = self.store.search(query, k=k, filter=filters)
    return [d for d in docs if d.score > self.threshold]

class VectorStore:
    def __init__(self, dim, metric="cosine"):
        self.dim = dim
        self.metric = metric
        self.rows = []

import os, json, logging
from typing import List, Dict, Optional
logger = logging.getLogger(__name__)

public class OrderService {
    private final PaymentClient paymentClient;
    public OrderService(PaymentClient paymentClient) { this.paymentClient = paymentClient; }
    public Order placeOrder(Cart cart) throws PaymentException {
        return paymentClient.charge(cart.total());
    }
}

function fetchJobs(url, options = {}) {
  return fetch(url, { method: "POST", headers: { "Content-Type": "application/json" }, ...options })
    .then((response) => response.json());
}

The repository contains a service that ingests GitHub repositories, splits the source files into chunks,
summarises every file, module and repository with a language model, embeds the summaries and stores them
in a vector index. Questions are answered by retrieving the most relevant context and synthesising an answer
that cites the source blocks. The configuration is read from environment variables such as REDIS_URL,
QWEN_ENDPOINT and CASSANDRA_HOST. Use the retry policy with exponential backoff when the broker reconnects.
Authentication tokens are cached for ten minutes; the cache is invalidated when the user logs out.
SELECT id, name, created_at FROM users WHERE active = true ORDER BY created_at DESC LIMIT 100;
docker build -t rag-worker . && kubectl apply -f deployment.yaml
""" * 4


_LETTERS = b"etaoinshrdlucmfwypvbgkqjxz"


def _synthetic_piece(i: int) -> bytes:
    out = bytearray(b" ")
    for _ in range(2 + i % 4):
        out.append(_LETTERS[i % 26])
        i //= 26
    return bytes(out)


class ByteBPETokenizer:
    def __init__(self, model_vocab_size: int, num_merges: int = 2000, corpus: str | None = None,
                 merges: list[tuple[int, int]] | None = None):
        self._lock = threading.Lock()
        self._h = rt().grag_bpe_create()
        if model_vocab_size >= 151646:
            self.special = dict(QWEN_SPECIAL_IDS)
        else:
            self.special = {ENDOFTEXT: model_vocab_size - 3, IM_START: model_vocab_size - 2,
                            IM_END: model_vocab_size - 1}
        cap = max(0, min(num_merges, min(self.special.values()) - 256))
        if merges is not None:
            arr = np.asarray(merges[:cap], dtype=np.int32).reshape(-1)
            rt().grag_bpe_set_merges(self._h, arr.ctypes.data, len(arr) // 2)
        elif cap > 0:
            text = (corpus or _BUILTIN_CORPUS).encode("utf-8")
            rt().grag_bpe_train(self._h, text, len(text), cap)
        for tok, tid in self.special.items():
            rt().grag_bpe_add_special(self._h, tok.encode(), tid)
        self.model_vocab_size = model_vocab_size
        self.eos_token_ids = {self.special[IM_END], self.special[ENDOFTEXT]}
        self.pad_token_id = self.special[ENDOFTEXT]
        # id -> bytes table for the streaming detokenizer: bytes, merge products, specials
        table = [b""] * max(model_vocab_size, max(self.special.values()) + 1)
        for i in range(256):
            table[i] = bytes([i])
        merges = self.merges()
        for k, (a, b) in enumerate(merges):
            table[256 + k] = table[a] + table[b]
        self._known = 256 + len(merges)
        # ids the offline vocabulary does not cover (a random-init model with
        # the real 152K vocab samples them all the time) still decode to text,
        # as they would with the real tokenizer: a deterministic short word
        for i in range(self._known, len(table)):
            table[i] = _synthetic_piece(i)
        for tok, tid in self.special.items():
            table[tid] = tok.encode()
        self._table = table

    def __del__(self):
        try:
            rt().grag_bpe_destroy(self._h)
        except Exception:
            pass

    @property
    def base_vocab_size(self) -> int:
        return rt().grag_bpe_vocab_size(self._h)

    def merges(self) -> list[tuple[int, int]]:
        n = rt().grag_bpe_get_merges(self._h, None, 0)
        buf = np.zeros(2 * max(n, 1), dtype=np.int32)
        rt().grag_bpe_get_merges(self._h, buf.ctypes.data, n)
        return [(int(buf[2 * i]), int(buf[2 * i + 1])) for i in range(n)]

    def encode(self, text: str) -> list[int]:
        b = text.encode("utf-8", errors="replace")
        cap = len(b) + 16
        out = np.empty(cap, dtype=np.int32)
        n = rt().grag_bpe_encode(self._h, b, len(b), out.ctypes.data, cap)
        if n > cap:
            out = np.empty(n, dtype=np.int32)
            rt().grag_bpe_encode(self._h, b, len(b), out.ctypes.data, n)
        return out[:n].tolist()

    def decode_bytes(self, ids) -> bytes:
        arr = np.asarray(list(ids), dtype=np.int32)
        if arr.size == 0:
            return b""
        if int(arr.max()) >= self._known:  # specials / ids outside the trained vocabulary
            return b"".join(self.token_bytes(int(t)) for t in arr)
        cap = 16 * arr.size + 64
        buf = ctypes.create_string_buffer(cap)
        n = rt().grag_bpe_decode(self._h, arr.ctypes.data, arr.size, buf, cap)
        if n > cap:
            buf = ctypes.create_string_buffer(n)
            rt().grag_bpe_decode(self._h, arr.ctypes.data, arr.size, buf, n)
        return buf.raw[:n]

    def decode(self, ids) -> str:
        return self.decode_bytes(ids).decode("utf-8", errors="replace")

    def token_bytes(self, tid: int) -> bytes:
        """Raw bytes of one token (table lookup: the streaming detokenizer's per-token path)."""
        return self._table[tid] if 0 <= tid < len(self._table) else b""

    def apply_chat_template(self, messages: list[dict], add_generation_prompt: bool = True,
                            enable_thinking: bool | None = None) -> str:
        return chatml(messages, add_generation_prompt, enable_thinking)


class HFTokenizer:
    def __init__(self, path: str):
        from tokenizers import Tokenizer

        p = Path(path)
        self._tok = Tokenizer.from_file(str(p / "tokenizer.json" if p.is_dir() else p))
        self.special = {t: self._tok.token_to_id(t) for t in (ENDOFTEXT, IM_START, IM_END)
                        if self._tok.token_to_id(t) is not None}
        self.eos_token_ids = set(self.special.values())
        self.pad_token_id = self.special.get(ENDOFTEXT, 0)
        self._tok_bytes: dict[int, bytes] = {}

    def encode(self, text: str) -> list[int]:
        return self._tok.encode(text, add_special_tokens=False).ids

    def decode(self, ids) -> str:
        return self._tok.decode(list(ids), skip_special_tokens=True)

    def token_bytes(self, tid: int) -> bytes:
        b = self._tok_bytes.get(tid)
        if b is None:
            piece = self._tok.id_to_token(tid)
            if piece is None or tid in self.eos_token_ids or piece in self.special:
                b = b""
            elif all(ch in _BYTE_DECODER for ch in piece):  # byte-level BPE piece (GPT-2 byte->unicode map)
                b = bytes(_BYTE_DECODER[ch] for ch in piece)
            else:
                b = self._tok.decode([tid], skip_special_tokens=True).encode("utf-8")
            self._tok_bytes[tid] = b
        return b

    def apply_chat_template(self, messages, add_generation_prompt=True, enable_thinking=None) -> str:
        return chatml(messages, add_generation_prompt, enable_thinking)


def _bytes_to_unicode() -> dict[int, str]:
    """GPT-2 / Qwen byte-level BPE alphabet: every byte maps to a printable code point."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("\xa1"), ord("\xac") + 1)) + \
        list(range(ord("\xae"), ord("\xff") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, map(chr, cs)))


_BYTE_DECODER = {c: b for b, c in _bytes_to_unicode().items()}


class IncrementalDetokenizer:
    """Per-sequence streaming detokenizer: token bytes go through an incremental
    UTF-8 decoder, so a character split across tokens is emitted once complete
    (decoding each token on its own would emit replacement characters)."""

    __slots__ = ("tok", "_dec")

    def __init__(self, tok):
        self.tok = tok
        self._dec = codecs.getincrementaldecoder("utf-8")(errors="replace")

    def push(self, tid: int) -> str:
        tb = getattr(self.tok, "token_bytes", None)
        if tb is None:
            return self.tok.decode([tid])
        return self._dec.decode(tb(tid))

    def flush(self) -> str:
        return self._dec.decode(b"", final=True)


def chatml(messages: list[dict], add_generation_prompt: bool = True, enable_thinking: bool | None = None) -> str:
    """Qwen ChatML layout: <|im_start|>role\\ncontent<|im_end|>\\n ..."""
    parts = [f"{IM_START}{m['role']}\n{m['content']}{IM_END}\n" for m in messages]
    if add_generation_prompt:
        parts.append(f"{IM_START}assistant\n")
        if enable_thinking is False:
            parts.append("<think>\n\n</think>\n\n")
    return "".join(parts)


def plain_template(messages: list[dict], add_generation_prompt: bool = True, enable_thinking: bool | None = None) -> str:
    """Prompt layout for base LMs without chat special tokens (GPT-2):
    ``Role: content`` turns separated by blank lines, ending in ``Assistant:``."""
    parts = [f"{m['role'].capitalize()}: {m['content']}\n\n" for m in messages]
    if add_generation_prompt:
        parts.append("Assistant:")
    return "".join(parts)


def load_tokenizer(model_dir: str | None, model_vocab_size: int, arch: str = "qwen2"):
    if model_dir and (Path(model_dir) / "tokenizer.json").exists():
        tok = HFTokenizer(model_dir)
    else:
        cache = os.environ.get("GRAG_BPE_MERGES")
        if cache and Path(cache).exists():
            pairs = [tuple(map(int, ln.split())) for ln in Path(cache).read_text().splitlines() if ln.strip()]
            tok = ByteBPETokenizer(model_vocab_size, merges=pairs)
        else:
            tok = ByteBPETokenizer(model_vocab_size)
    if arch == "gpt2":  # base LM: no ChatML tokens; <|endoftext|> ends generation
        tok.apply_chat_template = plain_template
    return tok


class WordPieceTokenizer:
    CLS, SEP, UNK, PAD = 101, 102, 100, 0

    def __init__(self, vocab_size: int = 30522, vocab_file: str | None = None, lowercase: bool = True):
        self._h = rt().grag_wp_create(vocab_size, self.UNK, 1 if lowercase else 0)
        self.vocab_size = vocab_size
        if vocab_size < 2000:  # tiny test encoders: keep specials inside the table
            self.CLS, self.SEP, self.UNK = 1, 2, 3
        if vocab_file and Path(vocab_file).exists():
            data = Path(vocab_file).read_bytes()
            rt().grag_wp_load_vocab(self._h, data, len(data))

    def __del__(self):
        try:
            rt().grag_wp_destroy(self._h)
        except Exception:
            pass

    def encode(self, text: str, max_len: int = 512) -> list[int]:
        b = text.encode("utf-8", errors="replace")
        cap = len(b) + 8
        out = np.empty(cap, dtype=np.int32)
        n = rt().grag_wp_encode(self._h, b, len(b), out.ctypes.data, cap)
        ids = out[:min(n, cap)].tolist()
        if self.vocab_size < 2000:
            ids = [4 + (i % (self.vocab_size - 4)) for i in ids]
        return [self.CLS] + ids[: max(0, max_len - 2)] + [self.SEP]
