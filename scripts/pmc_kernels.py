"""Workload for rocprofv3 --pmc passes over the framework's own HIP kernels
(no hipGraphs, so every dispatch is counted):
  1. bge-large encoder over 256 ingest-sized chunks (attn_fwd, layernorm,
     bias_act, pool_l2norm kernels + library GEMMs);
  2. fused cosine score + top-k over a 2M x 1024 bf16 flat shard (score_topk);
  3. Qwen2-7B (random init) prefill of 32 x 1024-token prompts + 8 eager
     decode steps (attn_prefill, paged_decode, combine, rmsnorm, qkv_rope,
     silu_mul, sampling kernels).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from githubrepostorag_amd.embed.service import Embedder  # noqa: E402
from githubrepostorag_amd.engine.llm_engine import EngineConfig, LLMEngine  # noqa: E402
from githubrepostorag_amd.engine.sequence import SamplingParams  # noqa: E402
from githubrepostorag_amd.engine.tokenizer import ByteBPETokenizer  # noqa: E402
from githubrepostorag_amd.models.configs import decoder_config  # noqa: E402
from githubrepostorag_amd.models.qwen2 import Qwen2Model  # noqa: E402
from githubrepostorag_amd.ops.topk import score_topk  # noqa: E402
from githubrepostorag_amd.utils import synthetic  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    emb = Embedder.from_name("bge-large-en-v1.5", device="cuda", seed=2)
    v = emb.embed_documents([synthetic.chunk_text(i, 1600) for i in range(256)])
    torch.cuda.synchronize()
    print("encoder", tuple(v.shape), flush=True)

    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.nn.functional.normalize(torch.randn(2_000_000, 1024, device=dev, generator=g), dim=1).bfloat16()
    Q = torch.nn.functional.normalize(torch.randn(64, 1024, device=dev, generator=g), dim=1).bfloat16()
    s, i = score_topk(X, Q, 10)
    torch.cuda.synchronize()
    print("topk", tuple(s.shape), flush=True)
    del X

    cfg = decoder_config("qwen2-7b")
    model = Qwen2Model(cfg, device=dev, seed=1)
    tok = ByteBPETokenizer(cfg.vocab_size)
    eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=32, max_model_len=2048, num_blocks=4096,
                                             use_cuda_graph=False))
    gen = torch.Generator().manual_seed(3)
    prompts = [torch.randint(10, 150000, (1024,), generator=gen).tolist() for _ in range(32)]
    outs = eng.generate(prompts, SamplingParams(max_tokens=8, temperature=0.4, top_p=0.8, repetition_penalty=1.2,
                                                ignore_eos=True))
    torch.cuda.synchronize()
    print("decoder", sum(len(o.token_ids) for o in outs), "tokens", flush=True)


if __name__ == "__main__":
    main()
