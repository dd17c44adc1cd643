"""Low-load engine probes: the reference's own operating regime.

The reference serves one user with vLLM at ``--max-num-seqs 4 --max-model-len 11712``
(/root/reference/helm/templates/qwen-deployment.yaml:30-33), so its latency is set by
  * single-prompt TTFT at up to 11.7K context (one prefill on an idle engine), and
  * decode TPOT at 1-4 live sequences (a weight-streaming step: every weight byte per token).
``run_low_load`` measures both on an engine of its own (max_model_len 11712, at most 16 live
sequences), through the production path: ``LLMEngine.step`` with hipGraph decode windows, the
reference worker's sampling parameters (temperature 0.4, top_p 0.8, repetition_penalty 1.2:
rag_worker/src/worker/services/qwen_llm.py:107-113), random prompt ids (no prefix-cache hits).

  ttft_ms[L]           add_request -> first token, one L-token prompt, idle engine (median of reps)
  tpot[(B, ctx)]       decode wall time per token once all B prompts are prefilled (host work included:
                       scheduling, replay, token read-back), and the bytes one step must read (weights +
                       the live KV) over that time
"""
from __future__ import annotations

import statistics
import time

import torch

from .llm_engine import EngineConfig, LLMEngine
from .sequence import SamplingParams

REF_MAX_MODEL_LEN = 11712  # helm/values.yaml:74


def _rand_prompt(g: torch.Generator, n: int, vocab: int) -> list[int]:
    return torch.randint(100, vocab - 1000, (n,), generator=g).tolist()


def run_low_load(model, tok, batches=(1, 4, 16), ctxs=(1024, 4096, 11600), ttft_lens=(1024, 4096, 11600),
                 gen: int = 49, ttft_reps: int = 3, kv_cache_gb: float | None = None, use_graph: bool = True,
                 log=None) -> dict:
    vocab = model.cfg.vocab_size
    mml = min(REF_MAX_MODEL_LEN, model.cfg.max_position)
    ctxs = [c for c in ctxs if c + gen < mml]
    ttft_lens = [n for n in ttft_lens if n + 1 < mml]
    bmax = max(batches)
    eng = LLMEngine(model, tok, EngineConfig(
        max_num_seqs=bmax, max_model_len=mml, kv_cache_gb=kv_cache_gb, use_cuda_graph=use_graph, seed=5,
        max_num_batched_tokens=16384, graph_batch_sizes=tuple(b for b in (1, 2, 4, 8, 16) if b <= bmax) or (bmax,)))
    sp = SamplingParams(max_tokens=gen, temperature=0.4, top_p=0.8, repetition_penalty=1.2, ignore_eos=True)
    g = torch.Generator().manual_seed(99)
    wbytes = model.param_bytes()
    kv_tok = model.kv_bytes_per_block(1)
    out = {"engine": {"max_model_len": mml, "max_num_seqs": bmax}, "ttft_ms": {}, "tpot": []}
    try:
        # warm the sampler chain and capture every decode graph the probes replay, outside the timings
        eng.generate([_rand_prompt(g, 64, vocab)], sp)
        if use_graph and eng.on_gpu:
            # gen = 8 k + 1: the prefill samples token 1, then k full 8-step windows (one graph per batch x plan)
            eng.warmup_graphs(list(batches), max_ctx=sorted({c + d for c in ctxs for d in (1, gen)}),
                              windows=(8,) if (gen - 1) % 8 == 0 else (1, 2, 4, 8))
        for L in ttft_lens:
            ts = []
            for _ in range(ttft_reps + 1):
                rid = eng.add_request(_rand_prompt(g, L, vocab), SamplingParams(max_tokens=1, temperature=0.4,
                                                                                top_p=0.8, ignore_eos=True))
                if eng.on_gpu:
                    torch.cuda.synchronize()
                t0 = time.perf_counter()
                while eng.get(rid).first_token_time is None:
                    eng.step()
                ts.append((eng.get(rid).first_token_time - t0) * 1000.0)
                while eng.has_unfinished():
                    eng.step()
                eng.pop(rid)
            out["ttft_ms"][str(L)] = round(statistics.median(ts[1:]), 2)  # the first rep warms this length
            if log:
                log(f"low-load TTFT {L} tokens: {out['ttft_ms'][str(L)]} ms")
        for B in batches:
            for ctx in ctxs:
                rids = [eng.add_request(_rand_prompt(g, ctx, vocab), sp) for _ in range(B)]
                while any(eng.get(r).first_token_time is None for r in rids):
                    eng.step()
                have = [len(eng.get(r).output_ids) for r in rids]
                d0 = eng.stats["decode_steps"]
                t0 = time.perf_counter()
                while eng.has_unfinished():
                    eng.step()
                dt = time.perf_counter() - t0
                toks = min(gen - h for h in have)
                steps = eng.stats["decode_steps"] - d0
                for r in rids:
                    eng.pop(r)
                tpot = dt / max(1, toks) * 1000.0
                step_bytes = wbytes + B * (ctx + gen // 2) * kv_tok
                rec = {"B": B, "ctx": ctx, "tpot_ms": round(tpot, 3), "decode_steps": steps,
                       "step_bytes_gb": round(step_bytes / 1e9, 2),
                       "effective_TB_s": round(step_bytes / (tpot * 1e-3) / 1e12, 2)}
                out["tpot"].append(rec)
                if log:
                    log(f"low-load decode B={B} ctx={ctx}: TPOT {rec['tpot_ms']} ms ({rec['effective_TB_s']} TB/s)")
    finally:
        del eng
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
    return out
