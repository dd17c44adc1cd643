"""Model families: Qwen2 and GPT-2 decoders (paged-KV engine), BERT-family encoders."""
from __future__ import annotations


def build_decoder(cfg, **kw):
    """Instantiate the decoder class for ``cfg.arch`` (same engine interface:
    forward / compute_logits / allocate_kv_cache / kv_bytes_per_block)."""
    if cfg.arch == "gpt2":
        from .gpt2 import GPT2Model

        return GPT2Model(cfg, **kw)
    from .qwen2 import Qwen2Model

    return Qwen2Model(cfg, **kw)
