"""BASELINE config 4's tensor-parallel layout on the HIP kernels: a Qwen2-72B-shaped decoder (the real 72B
dims -- hidden 8192, 64 query / 8 KV heads, FFN 29568 -> 3696 per rank zero-padded to 3712 -- at 2 layers)
sharded TP=8 over 8 processes that share the box's one GPU (gloo control plane; with 8 ranks on one
device the one-shot IPC all-reduce stays off -- parallel/custom_ar.enable_for_group -- and decode runs
eagerly, since gloo-staged collectives cannot live in a hipGraph).  Greedy tokens of the TP=8 engine must
be the TP=1 model's best tokens up to bf16 noise (tests/_logits.py), identical on every rank."""
import dataclasses
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from dist_utils import run_ranks  # noqa: E402

pytestmark = pytest.mark.gpu

PROMPTS = [[5, 17, 99, 3, 250, 7, 7, 1024], list(range(1, 40))]
NLAYERS = 2


def _cfg():
    from githubrepostorag_amd.models.configs import decoder_config

    return dataclasses.replace(decoder_config("qwen2-72b"), num_layers=NLAYERS, max_position=2048)


def _state_dict(cfg, dev):
    """HF-layout weights generated on the GPU from one seed: identical in every process."""
    g = torch.Generator(device=dev).manual_seed(72)
    H, D = cfg.hidden_size, cfg.head_dim

    def rnd(*shape, std=0.02):
        return (torch.randn(*shape, generator=g, device=dev, dtype=torch.float32) * std).to(torch.bfloat16)

    sd = {"model.embed_tokens.weight": rnd(cfg.vocab_size, H), "model.norm.weight": 1 + rnd(H, std=0.1),
          "lm_head.weight": rnd(cfg.vocab_size, H)}
    for i in range(cfg.num_layers):
        p = f"model.layers.{i}."
        for name, shape in (("self_attn.q_proj.weight", (cfg.num_heads * D, H)),
                            ("self_attn.k_proj.weight", (cfg.num_kv_heads * D, H)),
                            ("self_attn.v_proj.weight", (cfg.num_kv_heads * D, H)),
                            ("self_attn.o_proj.weight", (H, cfg.num_heads * D)),
                            ("mlp.gate_proj.weight", (cfg.intermediate_size, H)),
                            ("mlp.up_proj.weight", (cfg.intermediate_size, H)),
                            ("mlp.down_proj.weight", (H, cfg.intermediate_size))):
            sd[p + name] = rnd(*shape)
        for name, n in (("self_attn.q_proj.bias", cfg.num_heads * D), ("self_attn.k_proj.bias", cfg.num_kv_heads * D),
                        ("self_attn.v_proj.bias", cfg.num_kv_heads * D)):
            sd[p + name] = rnd(n)
        sd[p + "input_layernorm.weight"] = 1 + rnd(H, std=0.1)
        sd[p + "post_attention_layernorm.weight"] = 1 + rnd(H, std=0.1)
    return sd


def _tp_rank(rank, world):
    from githubrepostorag_amd.engine.llm_engine import EngineConfig, LLMEngine
    from githubrepostorag_amd.engine.sequence import SamplingParams
    from githubrepostorag_amd.engine.tokenizer import ByteBPETokenizer
    from githubrepostorag_amd.models.qwen2 import Qwen2Model
    from githubrepostorag_amd.parallel.comm import make_tp_dp_groups
    from githubrepostorag_amd.parallel.custom_ar import enable_for_group

    dev = torch.device("cuda", 0)
    cfg = _cfg()
    tp, _ = make_tp_dp_groups(world)
    ar = enable_for_group(tp, dev)
    sd = _state_dict(cfg, dev)
    model = Qwen2Model(cfg, device=dev, dtype=torch.bfloat16, tp=tp, state_dict=sd)
    del sd
    torch.cuda.empty_cache()
    eng = LLMEngine(model, ByteBPETokenizer(cfg.vocab_size),
                    EngineConfig(max_num_seqs=4, max_model_len=256, num_blocks=64, use_cuda_graph=True,
                                 graph_batch_sizes=(1, 2, 4), seed=3))
    out = [o.token_ids for o in eng.generate(PROMPTS, SamplingParams(max_tokens=8, temperature=0.0,
                                                                      ignore_eos=True))]
    torch.cuda.synchronize()
    return {"greedy": out, "hq": model.hq, "hkv": model.hkv, "inter": model.inter, "inter_real": model.inter_real,
            "custom_ar": ar is not None, "graph_captures": eng.stats["graph_captures"]}


def test_tp8_qwen2_72b_dims_matches_tp1(dev):
    from _logits import greedy_within_tolerance

    from githubrepostorag_amd.models.qwen2 import Qwen2Model

    res = run_ranks(_tp_rank, 8, timeout=900)
    cfg = _cfg()
    for r in res:
        assert r["hq"] == 8 and r["hkv"] == 1 and r["inter_real"] == 3696 and r["inter"] == 3712
        assert not r["custom_ar"] and r["graph_captures"] == 0  # 8 ranks on one device: gloo, eager decode
    assert all(r["greedy"] == res[0]["greedy"] for r in res)  # lockstep ranks sample the same ids
    ref = Qwen2Model(cfg, device=dev, dtype=torch.bfloat16, state_dict=_state_dict(cfg, dev))
    for prompt, toks in zip(PROMPTS, res[0]["greedy"]):
        assert len(toks) == 8
        greedy_within_tolerance(ref, dev, prompt, toks)
