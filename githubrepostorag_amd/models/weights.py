"""Checkpoint loading (safetensors only — executes nothing from the file) and
saving in HF layout (used by the round-trip tests and offline exports)."""
from __future__ import annotations

import json
from pathlib import Path

import torch


def load_state_dict(path: str | Path | None, device=None) -> dict | None:
    """All tensors of a safetensors checkpoint (file, directory or sharded
    index).  AutoAWQ W4A16 checkpoints (the reference's deployed
    Qwen2.5-Coder-7B-Instruct-AWQ, helm/values.yaml:67) are dequantised to
    bf16 HF-layout ``.weight`` tensors — on ``device`` with the HIP kernel
    when it is a GPU (ops/quant.py)."""
    if not path:
        return None
    from safetensors.torch import load_file

    p = Path(path)
    files = [p] if p.is_file() else sorted(p.glob("*.safetensors"))
    if not files:
        idx = p / "model.safetensors.index.json"
        if idx.exists():
            files = sorted({p / f for f in json.loads(idx.read_text())["weight_map"].values()})
    if not files:
        raise FileNotFoundError(f"no safetensors under {path}")
    sd: dict = {}
    for f in files:
        sd.update(load_file(str(f)))
    if any(k.endswith(".qweight") for k in sd):
        from ..ops.quant import dequantize_awq_state_dict

        sd = dequantize_awq_state_dict(sd, device=device)
    return sd


def save_state_dict(sd: dict, path: str | Path) -> None:
    from safetensors.torch import save_file

    Path(path).parent.mkdir(parents=True, exist_ok=True)
    save_file({k: v.contiguous().cpu() for k, v in sd.items()}, str(path))


def qwen2_hf_state_dict(model) -> dict:
    """Export a (TP=1) Qwen2Model back to HF tensor names."""
    cfg = model.cfg
    D = model.head_dim
    q, kv = model.hq * D, model.hkv * D
    sd = {"model.embed_tokens.weight": model.embed, "model.norm.weight": model.norm}
    for i, L in enumerate(model.layers):
        p = f"model.layers.{i}."
        sd[p + "input_layernorm.weight"] = L.in_norm
        sd[p + "post_attention_layernorm.weight"] = L.post_norm
        sd[p + "self_attn.q_proj.weight"] = L.qkv_w[:q]
        sd[p + "self_attn.k_proj.weight"] = L.qkv_w[q:q + kv]
        sd[p + "self_attn.v_proj.weight"] = L.qkv_w[q + kv:]
        if L.qkv_b is not None:
            sd[p + "self_attn.q_proj.bias"] = L.qkv_b[:q]
            sd[p + "self_attn.k_proj.bias"] = L.qkv_b[q:q + kv]
            sd[p + "self_attn.v_proj.bias"] = L.qkv_b[q + kv:]
        sd[p + "self_attn.o_proj.weight"] = L.o_w
        sd[p + "mlp.gate_proj.weight"], sd[p + "mlp.up_proj.weight"] = model.gate_up_weights(L)
        sd[p + "mlp.down_proj.weight"] = L.down_w
    if not cfg.tie_word_embeddings:
        sd["lm_head.weight"] = model.lm_head[: cfg.vocab_size]
    return {k: v.detach().clone() for k, v in sd.items()}


def bert_hf_state_dict(enc) -> dict:
    H = enc.cfg.hidden_size
    sd = {"embeddings.word_embeddings.weight": enc.word, "embeddings.position_embeddings.weight": enc.pos,
          "embeddings.token_type_embeddings.weight": enc.typ, "embeddings.LayerNorm.weight": enc.emb_g,
          "embeddings.LayerNorm.bias": enc.emb_b}
    for i, L in enumerate(enc.layers):
        p = f"encoder.layer.{i}."
        for j, n in enumerate(("query", "key", "value")):
            sd[p + f"attention.self.{n}.weight"] = L.qkv_w[j * H:(j + 1) * H]
            sd[p + f"attention.self.{n}.bias"] = L.qkv_b[j * H:(j + 1) * H]
        sd[p + "attention.output.dense.weight"] = L.o_w
        sd[p + "attention.output.dense.bias"] = L.o_b
        sd[p + "attention.output.LayerNorm.weight"] = L.ln1_g
        sd[p + "attention.output.LayerNorm.bias"] = L.ln1_b
        sd[p + "intermediate.dense.weight"] = L.f1_w
        sd[p + "intermediate.dense.bias"] = L.f1_b
        sd[p + "output.dense.weight"] = L.f2_w
        sd[p + "output.dense.bias"] = L.f2_b
        sd[p + "output.LayerNorm.weight"] = L.ln2_g
        sd[p + "output.LayerNorm.bias"] = L.ln2_b
    return {k: v.detach().clone() for k, v in sd.items()}
