"""Qwen2-family decoder (Qwen2 / Qwen2.5 / Qwen2.5-Coder) for the in-process
LLM engine — what the reference reached through the external vLLM container
(reference call sites rag_worker/src/worker/services/
qwen_llm.py:104-148, ingest/src/app/llm_init.py:68-143).

Layer dataflow per step (T tokens, kernels in brackets):
  embed gather [grag_embed_gather]
  per layer:
    residual += h ; x = RMSNorm(residual)            [grag_rmsnorm, fused]
    qkv = x W_qkv^T                                   [grag_gemm_tile at decode M, else library]
    q, K/V-cache <- bias + NeoX RoPE + paged store    [grag_qkv_rope_kvstore]
    a = paged flash attention (GQA-packed, MFMA)      [grag_paged_attention]
      (1-16 decode rows: the two lines above in one launch, [grag_paged_decode_mw_rope])
    h = a W_o^T        (+ TP all-reduce, RCCL)
    residual += h ; x = RMSNorm(residual)            [grag_rmsnorm]
    m = SiLU(x W_g^T) * (x W_u^T)                     [grag_gemm_tile EPI_SILU: one GEMM, the
                                                       SwiGLU product formed in registers; W_gu
                                                       stored gate/up-interleaved in 32-row blocks]
    h = m W_down^T     (+ TP all-reduce, RCCL)
  final RMSNorm ; LM head on last tokens (vocab-parallel under TP) ; fused
  sampler [grag_sample].

Tensor parallelism: q heads, kv heads (replicated when tp > num_kv_heads),
the FFN and the vocab are sharded per rank; two all-reduces per layer.
"""
from __future__ import annotations

import math
import os

import torch

from ..ops.attention import AttnMetadata, paged_attention, paged_decode_mw_rope
from ..ops.elementwise import qkv_rope_kvstore, rope_cos_sin, silu_mul
from ..ops.gemm import (EPI_PARTIAL, EPI_SILU, FoldedNorm, SplitKPartial, deinterleave_gate_up,
                        gemm_decode_norm, gemm_decode_red, gemm_decode_scaled, interleave_gate_up, mlp_gate_up,
                        norm_fuse_plan)
from ..ops.linear import linear, linear_deferred
from ..ops.norm import embed_gather, rmsnorm
from ..parallel.comm import Group
from .configs import DecoderConfig

FFN_PAD = int(os.environ.get("GRAG_FFN_PAD", "64"))  # per-rank FFN width granule (models/qwen2.py Qwen2Model)


class _Layer:
    __slots__ = ("in_norm", "qkv_w", "qkv_b", "o_w", "post_norm", "gu_w", "down_w", "w4")


class Qwen2Model:
    def __init__(self, cfg: DecoderConfig, device="cuda", dtype=torch.bfloat16, tp: Group | None = None,
                 seed: int = 0, state_dict: dict | None = None, init_std: float = 0.02):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.tp = tp or Group([0])
        ts, tr = self.tp.size, self.tp.rank
        assert cfg.num_heads % ts == 0, "num_heads must divide by tp"
        self.hq = cfg.num_heads // ts
        if cfg.num_kv_heads >= ts:
            assert cfg.num_kv_heads % ts == 0
            self.hkv = cfg.num_kv_heads // ts
            self.kv_head0 = tr * self.hkv
        else:  # replicate kv heads across ranks
            self.hkv = 1
            self.kv_head0 = tr // (ts // cfg.num_kv_heads)
        self.head_dim = cfg.head_dim
        assert cfg.intermediate_size % ts == 0
        # the per-rank FFN width, zero-padded up to a multiple of FFN_PAD (default 64) so every MLP GEMM
        # takes the owned kernels (K % 64): Qwen2-72B at TP=8 has 29568 / 8 = 3696 -> 3712.  The padded
        # gate/up rows and down_proj columns are zero, so silu(0) * 0 adds nothing: outputs are unchanged.
        self.inter_real = cfg.intermediate_size // ts
        pad = max(1, FFN_PAD)
        self.inter = -(-self.inter_real // pad) * pad
        # gate/up interleaved in 32-row blocks for the fused SwiGLU GEMM epilogue
        self.gu_interleaved = self.inter % 32 == 0
        self.vocab_shard = -(-cfg.vocab_size // ts)
        if ts > 1:  # shard starts on 8-token boundaries (the sampler reads seen bits 8 at a time)
            self.vocab_shard = -(-self.vocab_shard // 8) * 8
        self.vocab0 = tr * self.vocab_shard
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        self.cos_sin = rope_cos_sin(cfg.max_position, cfg.head_dim, cfg.rope_theta, self.device)
        self.w4_enabled = False
        if state_dict is not None:
            self._load(state_dict)
        else:
            self._init_random(seed, init_std)

    # ------------------------------------------------------------------ weights
    def _rand(self, g, *shape, std):
        t = torch.empty(*shape, dtype=self.dtype, device=self.device)
        if self.device.type == "cuda":
            t.normal_(0.0, std, generator=g)
        else:
            t.copy_(torch.randn(*shape, generator=g) * std)
        return t

    def _init_random(self, seed: int, std: float):
        cfg = self.cfg
        dev = self.device
        g = torch.Generator(device=dev if dev.type == "cuda" else "cpu")
        g.manual_seed(seed * 1000003 + 17)
        H, D = cfg.hidden_size, self.head_dim
        qkv_rows = (self.hq + 2 * self.hkv) * D
        self.embed = self._rand(g, cfg.vocab_size, H, std=std)
        self.layers = []
        for _ in range(cfg.num_layers):
            L = _Layer()
            L.in_norm = torch.ones(H, dtype=self.dtype, device=dev)
            L.qkv_w = self._rand(g, qkv_rows, H, std=std)
            L.qkv_b = self._rand(g, qkv_rows, std=std) if cfg.qkv_bias else None
            L.o_w = self._rand(g, H, self.hq * D, std=std)
            L.post_norm = torch.ones(H, dtype=self.dtype, device=dev)
            if self.inter == self.inter_real:
                L.gu_w = self._rand(g, 2 * self.inter, H, std=std)
                L.down_w = self._rand(g, H, self.inter, std=std)
            else:
                wg, wu = self._pad_ffn(self._rand(g, self.inter_real, H, std=std)), \
                    self._pad_ffn(self._rand(g, self.inter_real, H, std=std))
                L.gu_w = interleave_gate_up(wg, wu) if self.gu_interleaved else torch.cat([wg, wu], 0).contiguous()
                L.down_w = self._pad_ffn(self._rand(g, H, self.inter_real, std=std), dim=1)
            self.layers.append(L)
        self.norm = torch.ones(H, dtype=self.dtype, device=dev)
        if cfg.tie_word_embeddings:
            self.lm_head = self._pad_rows(self.embed[self.vocab0:self.vocab0 + self.vocab_shard])
        else:
            self.lm_head = self._pad_rows(self._rand(g, min(self.vocab_shard, cfg.vocab_size - self.vocab0), H,
                                                     std=std))

    def _pad_ffn(self, t: torch.Tensor, dim: int = 0) -> torch.Tensor:
        """Zero-pad an FFN weight from the real per-rank width to ``self.inter`` along ``dim``."""
        extra = self.inter - t.shape[dim]
        if extra <= 0:
            return t.contiguous()
        shape = list(t.shape)
        shape[dim] = extra
        return torch.cat([t, torch.zeros(shape, dtype=t.dtype, device=t.device)], dim).contiguous()

    def _pad_rows(self, t: torch.Tensor) -> torch.Tensor:
        # equal-sized vocab shards so the TP all-gather of logits is one collective
        if t.shape[0] == self.vocab_shard:
            return t
        pad = torch.zeros(self.vocab_shard - t.shape[0], t.shape[1], dtype=t.dtype, device=t.device)
        return torch.cat([t, pad], 0)

    def _load(self, sd: dict):
        """HF Qwen2 naming -> fused, TP-sharded tensors."""
        cfg = self.cfg
        D = self.head_dim
        dev, dt = self.device, self.dtype

        def get(name):
            return sd[name].to(device=dev, dtype=dt)

        q0, q1 = self.tp.rank * self.hq * D, (self.tp.rank + 1) * self.hq * D
        k0, k1 = self.kv_head0 * D, (self.kv_head0 + self.hkv) * D
        i0, i1 = self.tp.rank * self.inter_real, (self.tp.rank + 1) * self.inter_real
        self.embed = get("model.embed_tokens.weight")
        self.layers = []
        for i in range(cfg.num_layers):
            p = f"model.layers.{i}."
            L = _Layer()
            L.in_norm = get(p + "input_layernorm.weight")
            L.qkv_w = torch.cat([get(p + "self_attn.q_proj.weight")[q0:q1], get(p + "self_attn.k_proj.weight")[k0:k1],
                                 get(p + "self_attn.v_proj.weight")[k0:k1]], 0).contiguous()
            if cfg.qkv_bias:
                L.qkv_b = torch.cat([get(p + "self_attn.q_proj.bias")[q0:q1], get(p + "self_attn.k_proj.bias")[k0:k1],
                                     get(p + "self_attn.v_proj.bias")[k0:k1]], 0).contiguous()
            else:
                L.qkv_b = None
            L.o_w = get(p + "self_attn.o_proj.weight")[:, q0:q1].contiguous()
            L.post_norm = get(p + "post_attention_layernorm.weight")
            wg = self._pad_ffn(get(p + "mlp.gate_proj.weight")[i0:i1])
            wu = self._pad_ffn(get(p + "mlp.up_proj.weight")[i0:i1])
            L.gu_w = interleave_gate_up(wg, wu) if self.gu_interleaved else torch.cat([wg, wu], 0).contiguous()
            L.down_w = self._pad_ffn(get(p + "mlp.down_proj.weight")[:, i0:i1], dim=1)
            self.layers.append(L)
        self.norm = get("model.norm.weight")
        head = self.embed if cfg.tie_word_embeddings or "lm_head.weight" not in sd else get("lm_head.weight")
        self.lm_head = self._pad_rows(head[self.vocab0:self.vocab0 + self.vocab_shard].contiguous())

    # ------------------------------------------------------------------ W4A16 (AWQ precision)
    def quantize_w4(self) -> int:
        """4-bit weights (group-128 scales + zero points, AWQ's format) for the decode GEMMs
        (csrc/kernels/gemm_w4.hip); the bf16 weights are replaced by the values the 4-bit codes
        represent, so prefill (bf16 GEMMs) and decode compute with the same quantised model.
        Returns the bytes of packed 4-bit weights + scales."""
        from ..ops.w4 import W4Linear

        total = 0
        for L in self.layers:
            w4 = {}
            for name, silu in (("qkv_w", False), ("o_w", False), ("gu_w", self.gu_interleaved), ("down_w", False)):
                w = getattr(L, name)
                if w.shape[0] % 32 or w.shape[1] % 256:
                    continue
                q = W4Linear.quantize(w, silu=silu)
                setattr(L, name, q.dequant(w.dtype).contiguous())
                if w.is_cuda:  # the GPU kernel reads the packed copy; CPU keeps the codes for its reference
                    q.release_codes()
                w4[name] = q
                total += q.bytes()
            L.w4 = w4
        self.w4_enabled = True
        return total

    def _proj(self, x: torch.Tensor, L, name: str, bias=None, defer: bool = False):
        """A layer projection: the W4A16 decode GEMM at decode-sized batches when the model is
        quantised, else the bf16 path (ops/linear.py)."""
        w4 = getattr(L, "w4", None) if self.w4_enabled else None
        q = w4.get(name) if w4 else None
        if q is not None and x.is_cuda:
            from ..ops import w4 as W4

            if W4.plan(x.shape[0], q.N, q.K, q.silu) is not None and W4.capture_ok(x.device, x.shape[0], q):
                return W4.gemm_w4(x, q, bias)
        w = getattr(L, name)
        if defer and bias is None:  # o / down (residual add + RMSNorm) and qkv (RoPE pass) fold the split-K reduce
            return linear_deferred(x, w)
        if name == "gu_w":
            return mlp_gate_up(x, w) if self.gu_interleaved else silu_mul(linear(x, w))
        return linear(x, w, bias)

    def gate_up_weights(self, L) -> tuple[torch.Tensor, torch.Tensor]:
        """(gate [I, H], up [I, H]) of a layer in plain HF row order."""
        if self.gu_interleaved:
            return deinterleave_gate_up(L.gu_w)
        return L.gu_w[: self.inter], L.gu_w[self.inter:]

    def param_bytes(self) -> int:
        n = self.embed.numel() + self.norm.numel()
        for L in self.layers:
            for t in (L.in_norm, L.qkv_w, L.qkv_b, L.o_w, L.post_norm, L.gu_w, L.down_w):
                n += 0 if t is None else t.numel()
        if not self.cfg.tie_word_embeddings:
            n += self.lm_head.numel()
        return n * torch.finfo(self.dtype).bits // 8

    # ------------------------------------------------------------------ cache
    def kv_bytes_per_block(self, block_size: int) -> int:
        return 2 * self.cfg.num_layers * self.hkv * block_size * self.head_dim * torch.finfo(self.dtype).bits // 8

    def allocate_kv_cache(self, num_blocks: int, block_size: int):
        shape = (num_blocks, self.hkv, block_size, self.head_dim)
        return [(torch.zeros(shape, dtype=self.dtype, device=self.device),
                 torch.zeros(shape, dtype=self.dtype, device=self.device)) for _ in range(self.cfg.num_layers)]

    # ------------------------------------------------------------------ forward
    def forward(self, input_ids: torch.Tensor, positions: torch.Tensor, meta: AttnMetadata, kv_caches) -> torch.Tensor:
        cfg = self.cfg
        eps = cfg.rms_norm_eps
        h = embed_gather(input_ids, self.embed)
        residual = None
        defer = self.tp.trivial  # under TP the all-reduce sits between the projection and the norm
        # 1-4 rows: each split-K RMSNorm folded into the projections around it (ops/gemm.py FOLD_NORM)
        fold = (defer and self.gu_interleaved and not self.w4_enabled and input_ids.is_cuda
                and input_ids.shape[0] <= 4)  # (ops/gemm.py fold_plan: GRAG_FOLD_NORM=0 turns it off)
        nl = len(self.layers)
        for li, (L, (kc, vc)) in enumerate(zip(self.layers, kv_caches)):
            qkv = None
            if residual is None:
                residual = h
                x = rmsnorm(h, L.in_norm, eps)
            elif isinstance(h, FoldedNorm):  # the previous down_proj already added into the residual stream
                qkv = gemm_decode_scaled(h, L.in_norm, eps, L.qkv_w, EPI_PARTIAL)
                if qkv is None:
                    x = rmsnorm(residual, L.in_norm, eps)
            else:
                x = rmsnorm(h, L.in_norm, eps, residual=residual)
            if qkv is None:
                qkv = self._proj(x, L, "qkv_w", defer=True)  # a K-split's reduce folds into the RoPE pass
            # 1-16 decode rows: RoPE + K/V store inside the attention launch (ops/attention.py ROPE_FUSE)
            a = paged_decode_mw_rope(qkv, L.qkv_b, positions, self.cos_sin, kc, vc, meta, self.scale, self.hq,
                                     self.hkv, self.head_dim) if isinstance(qkv, SplitKPartial) else None
            if a is None:
                q = qkv_rope_kvstore(qkv, L.qkv_b, positions, self.cos_sin, meta.slot_mapping, kc, vc,
                                     self.hq, self.hkv, self.head_dim)
                a = paged_attention(q, kc, vc, meta, self.scale, causal=True)
            folded = gemm_decode_red(a, L.o_w, residual, 0) if fold else None
            m = None
            if folded is not None:
                m = gemm_decode_scaled(folded, L.post_norm, eps, L.gu_w, EPI_SILU)
                if m is None:
                    m = self._proj(rmsnorm(residual, L.post_norm, eps), L, "gu_w")
            else:
                h = self.tp.all_reduce(self._proj(a, L, "o_w", defer=defer))
                plan = None
                if isinstance(h, SplitKPartial) and self.gu_interleaved and not self.w4_enabled:
                    plan = norm_fuse_plan(h.M, L.gu_w.shape[0], h.N, True)
                if plan is not None:  # (A/B, off by default) the norm in the gate/up launch's prologue
                    r_new = torch.empty_like(residual)
                    m = gemm_decode_norm(h, residual, r_new, L.post_norm, eps, L.gu_w, EPI_SILU, plan)
                    residual = r_new
                else:
                    x = rmsnorm(h, L.post_norm, eps, residual=residual)
                    m = self._proj(x, L, "gu_w")
            h = gemm_decode_red(m, L.down_w, residual, 1) if fold and li + 1 < nl else None
            if h is None:
                h = self.tp.all_reduce(self._proj(m, L, "down_w", defer=defer))
        return rmsnorm(h, self.norm, eps, residual=residual)

    def local_logits(self, hidden: torch.Tensor) -> torch.Tensor:
        """hidden [B, H] -> this rank's vocab shard of the logits [B, vocab_shard] (tokens from
        ``vocab0``): what the vocab-parallel sampler (ops/sampling.sample_tp) consumes."""
        return linear(hidden, self.lm_head)

    def compute_logits(self, hidden: torch.Tensor) -> torch.Tensor:
        """hidden [B, H] -> logits [B, vocab] (bf16); vocab-parallel gather under TP (the engine
        samples from ``local_logits`` instead; this full gather serves tests and scoring)."""
        logits = linear(hidden, self.lm_head)
        if not self.tp.trivial:
            g = self.tp.all_gather(logits)  # [tp, B, Vs]
            logits = g.permute(1, 0, 2).reshape(hidden.shape[0], -1)[:, : self.cfg.vocab_size]
        return logits
