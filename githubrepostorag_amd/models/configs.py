"""Model configurations.

Architectural dimensions of the public checkpoints named in SURVEY §2.7
(re-verified against the public HF configs at build time is impossible
offline; these are the standard published values).  Weights are random-init
unless a local HF-format directory is given (see models/weights.py).
"""
from __future__ import annotations

from dataclasses import asdict, dataclass, replace


@dataclass(frozen=True)
class DecoderConfig:
    name: str
    vocab_size: int
    hidden_size: int
    intermediate_size: int
    num_layers: int
    num_heads: int
    num_kv_heads: int
    head_dim: int = 128
    rms_norm_eps: float = 1e-6
    rope_theta: float = 1_000_000.0
    max_position: int = 32768
    tie_word_embeddings: bool = False
    qkv_bias: bool = True
    arch: str = "qwen2"

    def to_dict(self):
        return asdict(self)

    @property
    def norm_eps(self) -> float:
        return self.rms_norm_eps

    def param_count(self) -> int:
        H, I, L = self.hidden_size, self.intermediate_size, self.num_layers
        q = self.num_heads * self.head_dim
        kv = self.num_kv_heads * self.head_dim
        emb = self.vocab_size * H * (1 if self.tie_word_embeddings else 2)
        if self.arch == "gpt2":  # LN(w,b) x2, qkv+bias, o+bias, fc+bias, proj+bias; learned positions
            per_layer = 4 * H + H * 3 * q + 3 * q + q * H + H + 2 * H * I + I + H
            return L * per_layer + emb + self.max_position * H + 2 * H
        per_layer = H * (q + 2 * kv) + (q + 2 * kv) + q * H + 3 * H * I + 2 * H
        return L * per_layer + emb + H


@dataclass(frozen=True)
class EncoderConfig:
    name: str
    vocab_size: int = 30522
    hidden_size: int = 384
    num_layers: int = 6
    num_heads: int = 12
    intermediate_size: int = 1536
    max_position: int = 512
    type_vocab_size: int = 2
    layer_norm_eps: float = 1e-12
    pooling: str = "mean"  # "mean" | "cls"
    normalize: bool = True
    max_seq_length: int = 256  # sentence-transformers truncation
    query_prefix: str = ""

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_heads

    def to_dict(self):
        return asdict(self)


DECODERS = {
    # reference deployment (helm/values.yaml:67) — served unquantised here
    "qwen2.5-coder-7b": DecoderConfig("qwen2.5-coder-7b", 152064, 3584, 18944, 28, 28, 4),
    # code default (rag_shared/config.py:29)
    "qwen2.5-3b": DecoderConfig("qwen2.5-3b", 151936, 2048, 11008, 36, 16, 2, tie_word_embeddings=True),
    "qwen2-0.5b": DecoderConfig("qwen2-0.5b", 151936, 896, 4864, 24, 14, 2, 64, tie_word_embeddings=True),
    "qwen2-1.5b": DecoderConfig("qwen2-1.5b", 151936, 1536, 8960, 28, 12, 2, tie_word_embeddings=True),
    "qwen2-7b": DecoderConfig("qwen2-7b", 152064, 3584, 18944, 28, 28, 4),
    "qwen2-72b": DecoderConfig("qwen2-72b", 152064, 8192, 29568, 80, 64, 8),
    # tiny configs for tests / CPU plumbing
    "qwen2-tiny": DecoderConfig("qwen2-tiny", 512, 256, 512, 2, 4, 2, 64, max_position=4096),
    "qwen2-small": DecoderConfig("qwen2-small", 4096, 512, 1408, 4, 8, 2, 64, max_position=8192),
    # Qwen2-72B's head layout scaled down (GQA 8:1 -> 16 q / 8 kv heads): TP = 8 leaves each rank 2 q heads and
    # one kv head, as the 72B's 8 / 1 at TP = 8 (BASELINE config 4's command form, rehearsed on the host)
    "qwen2-tiny-tp8": DecoderConfig("qwen2-tiny-tp8", 512, 512, 1024, 2, 16, 8, 32, max_position=4096),
    # GPT-2 family (BASELINE config 1: "GPT-2-small greedy answer"): pre-LN,
    # learned absolute positions, GELU(tanh) MLP, MHA, tied LM head
    "gpt2": DecoderConfig("gpt2", 50257, 768, 3072, 12, 12, 12, 64, 1e-5, 0.0, 1024, True, True, "gpt2"),
    "gpt2-medium": DecoderConfig("gpt2-medium", 50257, 1024, 4096, 24, 16, 16, 64, 1e-5, 0.0, 1024, True, True,
                                 "gpt2"),
    "gpt2-large": DecoderConfig("gpt2-large", 50257, 1280, 5120, 36, 20, 20, 64, 1e-5, 0.0, 1024, True, True,
                                "gpt2"),
    "gpt2-xl": DecoderConfig("gpt2-xl", 50257, 1600, 6400, 48, 25, 25, 64, 1e-5, 0.0, 1024, True, True, "gpt2"),
    "gpt2-tiny": DecoderConfig("gpt2-tiny", 512, 256, 1024, 2, 4, 4, 64, 1e-5, 0.0, 512, True, True, "gpt2"),
}

ENCODERS = {
    # reference default (rag_shared/config.py:24)
    "all-minilm-l6-v2": EncoderConfig("all-minilm-l6-v2", hidden_size=384, num_layers=6, num_heads=12,
                                      intermediate_size=1536, pooling="mean", max_seq_length=256),
    # README claim (README.md:139)
    "e5-small-v2": EncoderConfig("e5-small-v2", hidden_size=384, num_layers=12, num_heads=12,
                                 intermediate_size=1536, pooling="mean", max_seq_length=512,
                                 query_prefix="query: "),
    "bge-small-en-v1.5": EncoderConfig("bge-small-en-v1.5", hidden_size=384, num_layers=12, num_heads=12,
                                       intermediate_size=1536, pooling="cls", max_seq_length=512),
    "bge-base-en-v1.5": EncoderConfig("bge-base-en-v1.5", hidden_size=768, num_layers=12, num_heads=12,
                                      intermediate_size=3072, pooling="cls", max_seq_length=512),
    "bge-large-en-v1.5": EncoderConfig("bge-large-en-v1.5", hidden_size=1024, num_layers=24, num_heads=16,
                                       intermediate_size=4096, pooling="cls", max_seq_length=512),
    "encoder-tiny": EncoderConfig("encoder-tiny", vocab_size=2048, hidden_size=128, num_layers=2, num_heads=4,
                                  intermediate_size=256, max_position=256, max_seq_length=128),
}

ALIASES = {
    "qwen/qwen2.5-coder-7b-instruct-awq": "qwen2.5-coder-7b",
    "qwen/qwen2.5-coder-7b-instruct": "qwen2.5-coder-7b",
    "qwen/qwen2.5-3b-instruct": "qwen2.5-3b",
    "qwen/qwen2-7b": "qwen2-7b",
    "qwen/qwen2-7b-instruct": "qwen2-7b",
    "qwen/qwen2-1.5b": "qwen2-1.5b",
    "qwen/qwen2-72b": "qwen2-72b",
    "openai-community/gpt2": "gpt2",
    "openai-community/gpt2-medium": "gpt2-medium",
    "gpt2-small": "gpt2",
    "sentence-transformers/all-minilm-l6-v2": "all-minilm-l6-v2",
    "intfloat/e5-small-v2": "e5-small-v2",
    "baai/bge-base-en-v1.5": "bge-base-en-v1.5",
    "baai/bge-large-en-v1.5": "bge-large-en-v1.5",
    "baai/bge-small-en-v1.5": "bge-small-en-v1.5",
}


def _key(name: str) -> str:
    k = name.strip().lower()
    return ALIASES.get(k, k.split("/")[-1])


def decoder_config(name: str, **overrides) -> DecoderConfig:
    cfg = DECODERS[_key(name)]
    return replace(cfg, **overrides) if overrides else cfg


def encoder_config(name: str, **overrides) -> EncoderConfig:
    cfg = ENCODERS[_key(name)]
    return replace(cfg, **overrides) if overrides else cfg
