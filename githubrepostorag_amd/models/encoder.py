"""BERT-family sentence encoder (all-MiniLM-L6-v2 / e5 / bge) — replaces the
reference's CPU ``HuggingFaceEmbeddings`` (call sites
rag_worker/src/worker/services/graph_rag_retrievers.py:53,
ingest/src/app/services/vector_write_service.py:117).

Varlen packing: sequences are concatenated token-major (no pad tokens are
ever computed — the reference pads each sentence-transformers batch of 32 to
its longest member).  Per layer:
  qkv = h W_qkv^T + b                      (hipBLASLt, bias epilogue)
  a   = bidirectional MFMA attention       [grag_varlen_attention]
  h   = LN(a W_o^T + b_o + h)              [grag_layernorm: bias+residual+LN]
  f   = GELU(h W_1^T + b_1)                [grag_bias_act]
  h   = LN(f W_2^T + b_2 + h)              [grag_layernorm]
then masked-mean or CLS pooling + L2 normalisation [grag_pool_l2norm] writing
the fp32 vector and the bf16 copy the index stores.
"""
from __future__ import annotations

import torch

from ..ops.attention import varlen_attention
from ..ops.elementwise import ACT_GELU, POOL_CLS, POOL_MEAN, bias_act, pool_l2norm
from ..ops import gemm as _tile
from ..ops.linear import linear
from ..ops.norm import bert_embed_ln, layernorm
from ..utils.gpu_guard import no_gc
from .configs import EncoderConfig


class _ELayer:
    __slots__ = ("qkv_w", "qkv_b", "o_w", "o_b", "ln1_g", "ln1_b", "f1_w", "f1_b", "f2_w", "f2_b", "ln2_g", "ln2_b")


class BertEncoder:
    def __init__(self, cfg: EncoderConfig, device="cuda", dtype=torch.bfloat16, seed: int = 0,
                 state_dict: dict | None = None, init_std: float = 0.02):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.scale = cfg.head_dim ** -0.5
        if state_dict is not None:
            self._load(state_dict)
        else:
            self._init_random(seed, init_std)

    def _rand(self, g, *shape, std):
        t = torch.empty(*shape, dtype=self.dtype, device=self.device)
        if self.device.type == "cuda":
            t.normal_(0.0, std, generator=g)
        else:
            t.copy_(torch.randn(*shape, generator=g) * std)
        return t

    def _init_random(self, seed, std):
        cfg, dev, dt = self.cfg, self.device, self.dtype
        g = torch.Generator(device=dev if dev.type == "cuda" else "cpu")
        g.manual_seed(seed * 7919 + 3)
        H, I = cfg.hidden_size, cfg.intermediate_size
        self.word = self._rand(g, cfg.vocab_size, H, std=std)
        self.pos = self._rand(g, cfg.max_position, H, std=std)
        self.typ = self._rand(g, cfg.type_vocab_size, H, std=std)
        self.emb_g = torch.ones(H, dtype=dt, device=dev)
        self.emb_b = torch.zeros(H, dtype=dt, device=dev)
        self.layers = []
        for _ in range(cfg.num_layers):
            L = _ELayer()
            L.qkv_w = self._rand(g, 3 * H, H, std=std)
            L.qkv_b = self._rand(g, 3 * H, std=std)
            L.o_w = self._rand(g, H, H, std=std)
            L.o_b = self._rand(g, H, std=std)
            L.ln1_g = torch.ones(H, dtype=dt, device=dev)
            L.ln1_b = torch.zeros(H, dtype=dt, device=dev)
            L.f1_w = self._rand(g, I, H, std=std)
            L.f1_b = self._rand(g, I, std=std)
            L.f2_w = self._rand(g, H, I, std=std)
            L.f2_b = self._rand(g, H, std=std)
            L.ln2_g = torch.ones(H, dtype=dt, device=dev)
            L.ln2_b = torch.zeros(H, dtype=dt, device=dev)
            self.layers.append(L)

    def _load(self, sd):
        """HF BertModel naming (with or without a ``bert.``/``0.auto_model.`` prefix)."""
        keys = list(sd.keys())
        pre = ""
        for cand in ("bert.", "0.auto_model.", "model.", ""):
            if any(k.startswith(cand + "embeddings.word_embeddings") for k in keys):
                pre = cand
                break

        def get(n):
            return sd[pre + n].to(device=self.device, dtype=self.dtype)

        self.word = get("embeddings.word_embeddings.weight")
        self.pos = get("embeddings.position_embeddings.weight")
        self.typ = get("embeddings.token_type_embeddings.weight")
        self.emb_g = get("embeddings.LayerNorm.weight")
        self.emb_b = get("embeddings.LayerNorm.bias")
        self.layers = []
        for i in range(self.cfg.num_layers):
            p = f"encoder.layer.{i}."
            L = _ELayer()
            L.qkv_w = torch.cat([get(p + f"attention.self.{n}.weight") for n in ("query", "key", "value")], 0)
            L.qkv_b = torch.cat([get(p + f"attention.self.{n}.bias") for n in ("query", "key", "value")], 0)
            L.o_w = get(p + "attention.output.dense.weight")
            L.o_b = get(p + "attention.output.dense.bias")
            L.ln1_g = get(p + "attention.output.LayerNorm.weight")
            L.ln1_b = get(p + "attention.output.LayerNorm.bias")
            L.f1_w = get(p + "intermediate.dense.weight")
            L.f1_b = get(p + "intermediate.dense.bias")
            L.f2_w = get(p + "output.dense.weight")
            L.f2_b = get(p + "output.dense.bias")
            L.ln2_g = get(p + "output.LayerNorm.weight")
            L.ln2_b = get(p + "output.LayerNorm.bias")
            self.layers.append(L)

    @torch.inference_mode()
    def encode_ids(self, batch: list[list[int]], want_bf16: bool = True):
        """Token-id lists -> (fp32 [B, H], bf16 [B, H]) L2-normalised embeddings."""
        cfg = self.cfg
        dev = self.device
        lens = [max(1, min(len(x), cfg.max_position)) for x in batch]
        flat = []
        for x, n in zip(batch, lens):
            flat.extend(x[:n] if x else [0])
        starts = [0]
        for n in lens:
            starts.append(starts[-1] + n)
        ids = torch.tensor(flat, dtype=torch.int32, device=dev)
        pos_ids = torch.cat([torch.arange(n, dtype=torch.int32) for n in lens]).to(dev)
        seq_start = torch.tensor(starts, dtype=torch.int32, device=dev)
        seq_len = torch.tensor(lens, dtype=torch.int32, device=dev)
        return self.forward(ids, pos_ids, seq_start, seq_len, max(lens), want_bf16)

    def forward(self, ids, pos_ids, seq_start, seq_len, max_len: int, want_bf16: bool = True):
        """Packed token rows -> pooled, L2-normalised embeddings.  Sequence b owns rows
        [seq_start[b], seq_start[b] + seq_len[b]); rows past that (the fixed-shape padding
        of a captured batch) are computed but never attended to or pooled."""
        cfg = self.cfg
        H, nh = cfg.hidden_size, cfg.num_heads
        eps = cfg.layer_norm_eps
        h = bert_embed_ln(ids, pos_ids, None, self.word, self.pos, self.typ, self.emb_g, self.emb_b, eps)
        for L in self.layers:
            qkv = linear(h, L.qkv_w, L.qkv_b)
            a = varlen_attention(qkv, seq_start, seq_len, max_len, nh, cfg.head_dim, self.scale, causal=False)
            h = layernorm(linear(a, L.o_w), L.ln1_g, L.ln1_b, eps, bias=L.o_b, residual=h)
            if _tile.supported(h, L.f1_w) and _tile.capture_ok(h.device, h.shape[0], L.f1_w.shape[0], H):
                f = _tile.gemm(h, L.f1_w, L.f1_b, act=_tile.ACT_GELU)  # bias + GELU in the GEMM epilogue
            else:
                f = bias_act(linear(h, L.f1_w), L.f1_b, ACT_GELU, inplace=True)
            h = layernorm(linear(f, L.f2_w), L.ln2_g, L.ln2_b, eps, bias=L.f2_b, residual=h)
        mode = POOL_CLS if cfg.pooling == "cls" else POOL_MEAN
        return pool_l2norm(h, seq_start[:-1], seq_len, mode, cfg.normalize, want_bf16=want_bf16)


class EncoderGraphs:
    """hipGraph-captured encoder passes for query-sized batches (VERDICT r1 weak
    item 4: the eager encoder is launch-bound, ~8 launches x 24 layers for a few
    short questions).  A batch of n sequences of at most l tokens runs in the
    (B >= n, L >= l) bucket: sequence b occupies rows [b*L, b*L + len_b), the
    padding rows ride along in the GEMMs but are masked out of attention and
    pooling by seq_len, and bucket rows past n are 1-token dummies.  Position ids
    and sequence starts are constants of the bucket; only token ids and lengths
    are copied in (one pinned H2D copy) before the replay."""

    B_BUCKETS = (1, 2, 4, 8, 16, 32, 64, 128)
    L_BUCKETS = (16, 32, 64, 128)

    def __init__(self, enc: "BertEncoder"):
        self.enc = enc
        self.graphs: dict = {}
        self.pool = None
        self._events: dict = {}
        self.stats = {"replays": 0, "captures": 0}

    def bucket(self, n: int, lmax: int):
        B = next((b for b in self.B_BUCKETS if b >= n), None)
        L = next((x for x in self.L_BUCKETS if x >= lmax and x <= self.enc.cfg.max_position), None)
        return None if B is None or L is None else (B, L)

    def bucket_for(self, batch: list[list[int]]):
        maxp = self.enc.cfg.max_position
        return self.bucket(len(batch), max(max(1, min(len(x), maxp)) for x in batch)) if batch else None

    def has(self, bk) -> bool:
        return bk in self.graphs

    def capture(self, B: int, L: int):
        """Capture bucket (B, L); the caller holds the capture guard (gpu_guard)."""
        return self.graphs.get((B, L)) or self._capture(B, L)

    def _capture(self, B: int, L: int):
        dev = self.enc.device
        n_in = 2 * B * L + 2 * B + 1
        host = torch.zeros(n_in, dtype=torch.int32).pin_memory()
        dbuf = torch.zeros(n_in, dtype=torch.int32, device=dev)
        ids, pos = dbuf[: B * L], dbuf[B * L: 2 * B * L]
        starts, lens = dbuf[2 * B * L: 2 * B * L + B + 1], dbuf[2 * B * L + B + 1:]
        pos.copy_(torch.arange(L, dtype=torch.int32, device=dev).repeat(B))
        starts.copy_(torch.arange(B + 1, dtype=torch.int32, device=dev) * L)
        lens.fill_(1)
        host.copy_(dbuf.cpu())
        # a private memory pool per bucket: with one pool shared by every bucket, a bucket captured later
        # may place its intermediates in memory an earlier bucket's graph also writes on replay -- safe only
        # while replays never overlap, which a pool of its own does not depend on
        pool = torch.cuda.graph_pool_handle()
        cur = torch.cuda.current_stream(dev)
        s = cur if cur != torch.cuda.default_stream(dev) else torch.cuda.Stream(device=dev)  # capture needs a side stream
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            self.enc.forward(ids, pos, starts, lens, L, want_bf16=True)  # eager warm-up sizes workspaces
            s.synchronize()
            g = torch.cuda.CUDAGraph()
            with no_gc(), torch.cuda.graph(g, pool=pool, stream=s, capture_error_mode="thread_local"):
                outf, outb = self.enc.forward(ids, pos, starts, lens, L, want_bf16=True)
        cur.wait_stream(s)
        self.stats["captures"] += 1
        ent = (g, host, dbuf, outf, outb)
        self.graphs[(B, L)] = ent
        return ent

    def run(self, batch: list[list[int]], allow_capture: bool = True):
        """-> (fp32 [n, H], bf16 [n, H]) views into the bucket's static outputs
        (valid until the next replay of that bucket on this stream); None when no
        bucket fits (the caller runs eagerly)."""
        n = len(batch)
        maxp = self.enc.cfg.max_position
        lens = [max(1, min(len(x), maxp)) for x in batch]
        bk = self.bucket(n, max(lens))
        if bk is None:
            return None
        B, L = bk
        ent = self.graphs.get(bk)
        if ent is None:
            if not allow_capture:
                return None
            ent = self._capture(B, L)
        g, host, dbuf, outf, outb = ent
        ev = self._events.get(bk)
        if ev is not None:
            ev.synchronize()  # the previous replay's H2D copy has read the pinned buffer
        h = host.numpy()
        h[: B * L] = 0
        for b, (x, ln) in enumerate(zip(batch, lens)):
            if x:
                h[b * L: b * L + ln] = x[:ln]
        lo = 2 * B * L + B + 1
        h[lo: lo + n] = lens
        h[lo + n: lo + B] = 1
        dbuf.copy_(host, non_blocking=True)
        ev = self._events[bk] = torch.cuda.Event()
        ev.record()
        g.replay()
        self.stats["replays"] += 1
        return outf[:n], outb[:n]
