"""Workloads for rocprofv3 --pmc passes at the serving bench's operating points
(scripts/pmc_serving.sh runs each mode under every counter pass):

  --mode gemm --M 4096|7104   owned tile GEMM on the Qwen2-7B prefill shapes: fused gate/up + SiLU*mul
                              (4096 x 37888 x 3584) and down_proj (4096 x 3584 x 18944), 10 calls each,
                              with the schedule ops/gemm.py picks (random operands: DVFS-honest);
  --mode decode               Qwen2-7B (random init) engine with 192 sequences of 1024-token prompts and
                              8 eager decode steps: paged decode attention and the decode GEMMs at the
                              bench's ~190-row decode batch (the round-1 PMC point was batch 32).
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from githubrepostorag_amd.ops import gemm as G  # noqa: E402
from githubrepostorag_amd.ops.linear import enable_tuned_gemms  # noqa: E402


def gemm_mode(M: int, reps: int) -> None:
    dev = torch.device("cuda", 0)
    enable_tuned_gemms()
    g = torch.Generator(device=dev).manual_seed(0)
    for name, (N, K, silu) in {"gate_up": (37888, 3584, True), "down": (3584, 18944, False)}.items():
        w = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) * 0.05).bfloat16()
        x = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).bfloat16()
        ks, sk = G.schedule(M, N, K, silu)
        G.WS.reserve(dev, G._ws_floats(M, N, ks, sk))
        for _ in range(reps):
            G.gemm_silu(x, w, ksplit=ks, sk=sk) if silu else G.gemm(x, w, ksplit=ks, sk=sk)
        torch.cuda.synchronize()
        print(name, M, N, K, "schedule", (ks, sk), flush=True)


def decode_mode(nseq: int, steps: int) -> None:
    from githubrepostorag_amd.engine.llm_engine import EngineConfig, LLMEngine
    from githubrepostorag_amd.engine.sequence import SamplingParams
    from githubrepostorag_amd.engine.tokenizer import ByteBPETokenizer
    from githubrepostorag_amd.models.configs import decoder_config
    from githubrepostorag_amd.models.qwen2 import Qwen2Model

    dev = torch.device("cuda", 0)
    cfg = decoder_config("qwen2-7b")
    model = Qwen2Model(cfg, device=dev, seed=1)
    tok = ByteBPETokenizer(cfg.vocab_size)
    eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=nseq, max_model_len=2048,
                                             num_blocks=nseq * (1024 + steps + 16) // 16 + 64,
                                             max_num_batched_tokens=16384, use_cuda_graph=False))
    gen = torch.Generator().manual_seed(3)
    prompts = [torch.randint(10, 150000, (1024,), generator=gen).tolist() for _ in range(nseq)]
    outs = eng.generate(prompts, SamplingParams(max_tokens=steps, temperature=0.4, top_p=0.8,
                                                repetition_penalty=1.2, ignore_eos=True))
    torch.cuda.synchronize()
    print("decoder", sum(len(o.token_ids) for o in outs), "tokens", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="gemm", choices=["gemm", "decode"])
    ap.add_argument("--M", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--nseq", type=int, default=192)
    ap.add_argument("--steps", type=int, default=8)
    a = ap.parse_args()
    if a.mode == "gemm":
        gemm_mode(a.M, a.reps)
    else:
        decode_mode(a.nseq, a.steps)


if __name__ == "__main__":
    main()
