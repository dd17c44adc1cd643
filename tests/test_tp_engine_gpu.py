"""Tensor-parallel Qwen2 engine on the HIP kernels, two processes on one GPU.

The gpurun box has one MI355X, so the two TP ranks share cuda:0 and talk over
gloo for the host control plane (RCCL refuses two ranks on one device).  Every
device collective of a decode step goes through the one-shot IPC communicator
(parallel/custom_ar.py): the o_proj / down_proj all-reduces (bf16), the
vocab-parallel sampler's histograms (fp32 sum) and its (max, id) / winner
exchanges (all-gather).  The decode steps run as captured hipGraphs, which
could not hold a gloo call: a passing run means each graph held only HIP
kernels, the configuration the 8-GPU node runs over xGMI.

Checks: greedy tokens of the TP=2 engine are the TP=1 model's best tokens up
to bf16 noise (tests/_logits.py rule), both ranks produce identical tokens,
and sampled decoding (temperature / top-p / repetition penalty, the
reference worker's knobs: rag_worker/src/worker/services/qwen_llm.py:107-113)
agrees across the ranks."""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from dist_utils import run_ranks  # noqa: E402

pytestmark = pytest.mark.gpu

CFG = "qwen2-small"
PROMPTS = [[5, 17, 99, 3, 250, 7, 7, 1024], list(range(1, 40)), [300 + i for i in range(77)]]


def _state_dict(cfg):
    from test_parallel_cpu import _hf_state_dict

    return _hf_state_dict(cfg)


def _engine(model, graphs=True):
    from githubrepostorag_amd.engine.llm_engine import EngineConfig, LLMEngine
    from githubrepostorag_amd.engine.tokenizer import ByteBPETokenizer

    return LLMEngine(model, ByteBPETokenizer(model.cfg.vocab_size),
                     EngineConfig(max_num_seqs=8, max_model_len=512, num_blocks=256, use_cuda_graph=graphs,
                                  graph_batch_sizes=(1, 2, 4, 8), seed=3))


def _tp_rank(rank, world):
    from githubrepostorag_amd.engine.sequence import SamplingParams
    from githubrepostorag_amd.models.configs import decoder_config
    from githubrepostorag_amd.models.qwen2 import Qwen2Model
    from githubrepostorag_amd.parallel.comm import make_tp_dp_groups
    from githubrepostorag_amd.parallel.custom_ar import enable_for_group

    dev = torch.device("cuda", 0)
    cfg = decoder_config(CFG)
    tp, _ = make_tp_dp_groups(world)
    ar = enable_for_group(tp, dev)
    assert ar is not None, "one-shot IPC communicator unavailable"
    model = Qwen2Model(cfg, device=dev, dtype=torch.bfloat16, tp=tp, state_dict=_state_dict(cfg))
    eng = _engine(model)
    greedy = [o.token_ids for o in eng.generate(PROMPTS, SamplingParams(max_tokens=12, temperature=0.0,
                                                                         ignore_eos=True))]
    sampled = [o.token_ids for o in eng.generate(PROMPTS, SamplingParams(max_tokens=12, temperature=0.4, top_p=0.8,
                                                                          repetition_penalty=1.2, ignore_eos=True))]
    torch.cuda.synchronize()
    assert not ar.failed()
    return {"greedy": greedy, "sampled": sampled, "graph_replays": eng.stats["graph_replays"],
            "graph_captures": eng.stats["graph_captures"], "hq": model.hq, "inter": model.inter}


def test_tp2_engine_two_processes_matches_tp1(dev):
    from githubrepostorag_amd.models.configs import decoder_config
    from githubrepostorag_amd.models.qwen2 import Qwen2Model

    from _logits import greedy_within_tolerance

    res = run_ranks(_tp_rank, 2, timeout=300)
    cfg = decoder_config(CFG)
    for r in res:
        assert r["hq"] == cfg.num_heads // 2 and r["inter"] == cfg.intermediate_size // 2
        assert r["graph_captures"] > 0 and r["graph_replays"] > 0  # decode ran as hipGraphs
    assert res[0]["greedy"] == res[1]["greedy"]  # lockstep ranks sample the same ids
    assert res[0]["sampled"] == res[1]["sampled"]
    ref = Qwen2Model(cfg, device=dev, dtype=torch.bfloat16, state_dict=_state_dict(cfg))
    for prompt, toks in zip(PROMPTS, res[0]["greedy"]):
        assert len(toks) == 12
        greedy_within_tolerance(ref, dev, prompt, toks)
