"""GPT-2-family decoder (gpt2 / -medium / -large / -xl) for the same paged-KV
engine as Qwen2 — BASELINE config 1's "GPT-2-small greedy answer" model.
The reference never runs a model in-process; its answer model is reached
over HTTP (rag_worker/src/worker/services/qwen_llm.py:104-148), so this is a
second model family behind the same ``complete()`` contract.

Pre-LN block, per layer (kernels in brackets):
  x  = LN1(residual)                                    (fused into the previous boundary)
  qkv = x W_attn^T                                      (hipBLASLt / skinny / stream-K GEMM)
  q, K/V-cache <- bias + paged store, no rotary         [grag_qkv_rope_kvstore, cos_sin = null]
  a  = causal paged flash attention (MHA, head_dim 64)  [grag_paged_attention]
  h  = a W_o^T        (+ TP all-reduce)
  residual += h + b_o ; x = LN2(residual)               [grag_add_layernorm: one pass]
  f  = GELU_tanh(x W_fc^T + b_fc)                       [grag_bias_act, act 3]
  h  = f W_proj^T     (+ TP all-reduce)
  residual += h + b_proj ; x = LN1'(residual)           [grag_add_layernorm]
The token + position embeddings enter through the same fused add+LN: the
position rows are gathered into the residual buffer and the token rows are
added to them by the first LN1.  Row-parallel biases are added once, after
the all-reduce, inside the LN kernel.  The LM head is the (tied) token
embedding, padded to a multiple of 128 rows so the vocab GEMM tiles evenly.
"""
from __future__ import annotations

import math

import torch

from ..ops.attention import AttnMetadata, paged_attention
from ..ops.elementwise import ACT_GELU_TANH, bias_act, qkv_rope_kvstore
from ..ops.linear import linear
from ..ops.norm import add_layernorm, embed_gather
from ..parallel.comm import Group
from .configs import DecoderConfig

_VOCAB_ALIGN = 128


class _GLayer:
    __slots__ = ("ln1_g", "ln1_b", "qkv_w", "qkv_b", "o_w", "o_b", "ln2_g", "ln2_b", "fc_w", "fc_b",
                 "proj_w", "proj_b")


class GPT2Model:
    def __init__(self, cfg: DecoderConfig, device="cuda", dtype=torch.bfloat16, tp: Group | None = None,
                 seed: int = 0, state_dict: dict | None = None, init_std: float = 0.02):
        assert cfg.arch == "gpt2", cfg.arch
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.tp = tp or Group([0])
        ts, tr = self.tp.size, self.tp.rank
        assert cfg.num_heads % ts == 0 and cfg.intermediate_size % ts == 0, "heads / ffn must divide by tp"
        self.hq = self.hkv = cfg.num_heads // ts
        self.head_dim = cfg.head_dim
        self.inter = cfg.intermediate_size // ts
        per = -(-cfg.vocab_size // ts)
        self.vocab_shard = -(-per // _VOCAB_ALIGN) * _VOCAB_ALIGN
        self.vocab0 = tr * per
        self.vocab_rows = max(0, min(per, cfg.vocab_size - self.vocab0))
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
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

    def _ones(self, n):
        return torch.ones(n, dtype=self.dtype, device=self.device)

    def _zeros(self, *shape):
        return torch.zeros(*shape, dtype=self.dtype, device=self.device)

    def _init_random(self, seed: int, std: float):
        cfg = self.cfg
        g = torch.Generator(device=self.device if self.device.type == "cuda" else "cpu")
        g.manual_seed(seed * 1000003 + 29)
        H, D = cfg.hidden_size, self.head_dim
        q = self.hq * D
        self.wte = self._rand(g, cfg.vocab_size, H, std=std)
        self.wpe = self._rand(g, cfg.max_position, H, std=std / 2)
        # GPT-2 scales the residual projections by 1/sqrt(2L) at init
        proj_std = std / math.sqrt(2 * cfg.num_layers)
        self.layers = []
        for _ in range(cfg.num_layers):
            L = _GLayer()
            L.ln1_g, L.ln1_b = self._ones(H), self._zeros(H)
            L.qkv_w = self._rand(g, 3 * q, H, std=std)
            L.qkv_b = self._rand(g, 3 * q, std=std)
            L.o_w = self._rand(g, H, q, std=proj_std)
            L.o_b = self._rand(g, H, std=std)
            L.ln2_g, L.ln2_b = self._ones(H), self._zeros(H)
            L.fc_w = self._rand(g, self.inter, H, std=std)
            L.fc_b = self._rand(g, self.inter, std=std)
            L.proj_w = self._rand(g, H, self.inter, std=proj_std)
            L.proj_b = self._rand(g, H, std=std)
            self.layers.append(L)
        self.lnf_g, self.lnf_b = self._ones(H), self._zeros(H)
        self._make_head()

    def _make_head(self):
        rows = self.wte[self.vocab0:self.vocab0 + self.vocab_rows]
        head = self._zeros(self.vocab_shard, self.cfg.hidden_size)
        head[: rows.shape[0]].copy_(rows)
        self.lm_head = head

    def _load(self, sd: dict):
        """HF GPT2LMHeadModel naming (Conv1D weights are [in, out])."""
        cfg = self.cfg
        pre = "transformer." if any(k.startswith("transformer.") for k in sd) else ""
        dev, dt = self.device, self.dtype
        D, H = self.head_dim, cfg.hidden_size
        tr = self.tp.rank
        q0, q1 = tr * self.hq * D, (tr + 1) * self.hq * D
        i0, i1 = tr * self.inter, (tr + 1) * self.inter

        def get(name):
            return sd[pre + name].to(device=dev, dtype=dt)

        self.wte = get("wte.weight")
        self.wpe = get("wpe.weight")
        self.layers = []
        for i in range(cfg.num_layers):
            p = f"h.{i}."
            L = _GLayer()
            L.ln1_g, L.ln1_b = get(p + "ln_1.weight"), get(p + "ln_1.bias")
            w = get(p + "attn.c_attn.weight").t()  # [3H, H]
            b = get(p + "attn.c_attn.bias")
            L.qkv_w = torch.cat([w[j * H + q0:j * H + q1] for j in range(3)], 0).contiguous()
            L.qkv_b = torch.cat([b[j * H + q0:j * H + q1] for j in range(3)], 0).contiguous()
            L.o_w = get(p + "attn.c_proj.weight").t()[:, q0:q1].contiguous()
            L.o_b = get(p + "attn.c_proj.bias")
            L.ln2_g, L.ln2_b = get(p + "ln_2.weight"), get(p + "ln_2.bias")
            L.fc_w = get(p + "mlp.c_fc.weight").t()[i0:i1].contiguous()
            L.fc_b = get(p + "mlp.c_fc.bias")[i0:i1].contiguous()
            L.proj_w = get(p + "mlp.c_proj.weight").t()[:, i0:i1].contiguous()
            L.proj_b = get(p + "mlp.c_proj.bias")
            self.layers.append(L)
        self.lnf_g, self.lnf_b = get("ln_f.weight"), get("ln_f.bias")
        self._make_head()

    def hf_state_dict(self) -> dict:
        """Export (TP=1) back to HF GPT-2 names (round-trip tests)."""
        sd = {"transformer.wte.weight": self.wte, "transformer.wpe.weight": self.wpe,
              "transformer.ln_f.weight": self.lnf_g, "transformer.ln_f.bias": self.lnf_b}
        for i, L in enumerate(self.layers):
            p = f"transformer.h.{i}."
            sd.update({p + "ln_1.weight": L.ln1_g, p + "ln_1.bias": L.ln1_b,
                       p + "attn.c_attn.weight": L.qkv_w.t(), p + "attn.c_attn.bias": L.qkv_b,
                       p + "attn.c_proj.weight": L.o_w.t(), p + "attn.c_proj.bias": L.o_b,
                       p + "ln_2.weight": L.ln2_g, p + "ln_2.bias": L.ln2_b,
                       p + "mlp.c_fc.weight": L.fc_w.t(), p + "mlp.c_fc.bias": L.fc_b,
                       p + "mlp.c_proj.weight": L.proj_w.t(), p + "mlp.c_proj.bias": L.proj_b})
        return {k: v.detach().contiguous().clone() for k, v in sd.items()}

    def param_bytes(self) -> int:
        n = self.wte.numel() + self.wpe.numel() + 2 * self.lnf_g.numel()
        for L in self.layers:
            n += sum(getattr(L, s).numel() for s in _GLayer.__slots__)
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
        eps = self.cfg.norm_eps
        residual = embed_gather(positions, self.wpe)  # becomes the residual stream
        h, b = embed_gather(input_ids, self.wte), None
        for L, (kc, vc) in zip(self.layers, kv_caches):
            x = add_layernorm(h, L.ln1_g, L.ln1_b, eps, residual, bias=b)
            qkv = linear(x, L.qkv_w)
            q = qkv_rope_kvstore(qkv, L.qkv_b, positions, None, meta.slot_mapping, kc, vc,
                                 self.hq, self.hkv, self.head_dim)
            a = paged_attention(q, kc, vc, meta, self.scale, causal=True)
            h = self.tp.all_reduce(linear(a, L.o_w))
            x = add_layernorm(h, L.ln2_g, L.ln2_b, eps, residual, bias=L.o_b)
            f = bias_act(linear(x, L.fc_w), L.fc_b, ACT_GELU_TANH, inplace=True)
            h, b = self.tp.all_reduce(linear(f, L.proj_w)), L.proj_b
        return add_layernorm(h, self.lnf_g, self.lnf_b, eps, residual, bias=b)

    def compute_logits(self, hidden: torch.Tensor) -> torch.Tensor:
        """hidden [B, H] -> logits [B, vocab] (a strided view of the padded GEMM output)."""
        logits = linear(hidden, self.lm_head)
        if not self.tp.trivial:
            g = self.tp.all_gather(logits)  # [tp, B, Vs]
            return g.permute(1, 0, 2)[..., : -(-self.cfg.vocab_size // self.tp.size)].reshape(
                hidden.shape[0], -1)[:, : self.cfg.vocab_size]
        return logits[:, : self.cfg.vocab_size]
