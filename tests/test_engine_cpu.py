"""LLM engine on CPU (fp32 reference ops): continuous batching, chunked
prefill, prefix cache, preemption, abort, stop handling, the native block
allocator and the tokenizers.  The GPU tier (test_engine_gpu.py) repeats the
numerics on the HIP kernels with hipGraph decode windows."""
import time

import numpy as np
import pytest
import torch

from githubrepostorag_amd.engine.llm_engine import EngineConfig, LLMEngine
from githubrepostorag_amd.engine.scheduler import KVCacheManager
from githubrepostorag_amd.engine.sequence import SamplingParams, Sequence
from githubrepostorag_amd.engine.tokenizer import (IM_END, IM_START, ByteBPETokenizer, IncrementalDetokenizer,
                                                   WordPieceTokenizer, chatml)
from githubrepostorag_amd.models.configs import decoder_config
from githubrepostorag_amd.models.qwen2 import Qwen2Model


@pytest.fixture(scope="module")
def model():
    return Qwen2Model(decoder_config("qwen2-tiny"), device="cpu", dtype=torch.float32, seed=0, init_std=0.05)


@pytest.fixture(scope="module")
def tok():
    return ByteBPETokenizer(512)


PROMPTS = [[5, 17, 99, 3, 250], list(range(1, 40)), [7] * 70, [300, 301, 302]]
GREEDY = SamplingParams(max_tokens=7, temperature=0.0, ignore_eos=True)


def _gen(model, tok, prompts=PROMPTS, sp=GREEDY, **cfg):
    kw = dict(max_num_seqs=4, max_model_len=512, num_blocks=256, use_cuda_graph=False)
    kw.update(cfg)
    eng = LLMEngine(model, tok, EngineConfig(**kw))
    return eng, eng.generate(prompts, sp)


def test_decode_matches_full_recompute(model, tok):
    _, outs = _gen(model, tok)
    _, ref_eng = None, LLMEngine(model, tok, EngineConfig(max_num_seqs=1, max_model_len=512, num_blocks=256,
                                                          use_cuda_graph=False, enable_prefix_caching=False))
    for p, o in zip(PROMPTS, outs):
        assert len(o.token_ids) == 7 and o.finish_reason == "length"
        for j in range(len(o.token_ids)):
            r = ref_eng.generate([p + o.token_ids[:j]], SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True))
            assert r[0].token_ids[0] == o.token_ids[j]


def test_chunked_prefill_and_small_batches_identical(model, tok):
    _, a = _gen(model, tok)
    eng, b = _gen(model, tok, max_num_batched_tokens=16, max_num_seqs=2)
    assert [x.token_ids for x in a] == [x.token_ids for x in b]
    assert eng.stats["steps"] > 10


def test_preemption_recomputes_identically(model, tok):
    prompts = [[(7 * i + j) % 500 + 1 for j in range(31)] for i in range(4)]
    # 16 usable blocks of 8 tokens: the admission watermark (a free block per running sequence) admits
    # three 31-token prompts (4 blocks each); their growth to 51 tokens (7 blocks each) does not fit:
    # decode must preempt the youngest and recompute it later
    sp = SamplingParams(max_tokens=20, temperature=0.0, ignore_eos=True)
    _, a = _gen(model, tok, prompts=prompts, sp=sp)
    eng, b = _gen(model, tok, prompts=prompts, sp=sp, num_blocks=17, block_size=8, enable_prefix_caching=False)
    assert [x.token_ids for x in a] == [x.token_ids for x in b]
    assert eng.sched.num_preemptions > 0


def test_admission_watermark_avoids_preemption(model, tok):
    """Round 3 admitted the fourth 31-token prompt into the last free blocks and preempted at the next
    block crossing; the watermark keeps one free block per running sequence, so growth to 38 tokens
    (5 blocks each) finishes without a preemption."""
    prompts = [[(7 * i + j) % 500 + 1 for j in range(31)] for i in range(4)]
    eng, b = _gen(model, tok, prompts=prompts, num_blocks=17, block_size=8, enable_prefix_caching=False)
    _, a = _gen(model, tok, prompts=prompts)
    assert [x.token_ids for x in a] == [x.token_ids for x in b]
    assert eng.sched.num_preemptions == 0


def test_prefix_cache_hit(model, tok):
    base = list(range(10, 90))
    eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=4, max_model_len=512, num_blocks=256,
                                             use_cuda_graph=False))
    eng.generate([base + [1]], GREEDY)
    outs = eng.generate([base + [2], base + [3]], GREEDY)
    assert all(o.cached_tokens >= 64 for o in outs)
    assert eng.kv.stats()["prefix_hits"] > 0
    _, ref = _gen(model, tok, prompts=[base + [2], base + [3]], enable_prefix_caching=False)
    assert [o.token_ids for o in outs] == [o.token_ids for o in ref]


def test_abort_and_stop_tokens(model, tok):
    eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=4, max_model_len=512, num_blocks=256,
                                             use_cuda_graph=False))
    rid = eng.add_request(PROMPTS[0], SamplingParams(max_tokens=50, temperature=0.0, ignore_eos=True))
    eng.step()
    eng.abort(rid)
    while eng.has_unfinished():
        eng.step()
    assert eng.get(rid).finish_reason == "abort"
    _, full = _gen(model, tok, prompts=[PROMPTS[1]])
    stop = full[0].token_ids[3]
    _, cut = _gen(model, tok, prompts=[PROMPTS[1]],
                  sp=SamplingParams(max_tokens=7, temperature=0.0, ignore_eos=True, stop_token_ids=[stop]))
    k = full[0].token_ids.index(stop)
    assert cut[0].token_ids == full[0].token_ids[: k + 1] and cut[0].finish_reason == "stop"


def test_sampling_seeded_and_penalty(model, tok):
    sp = SamplingParams(max_tokens=12, temperature=0.9, top_p=0.9, repetition_penalty=1.3, ignore_eos=True, seed=7)
    _, a = _gen(model, tok, sp=sp)
    _, b = _gen(model, tok, sp=sp)
    assert [x.token_ids for x in a] == [x.token_ids for x in b]


def test_streaming_callback(model, tok):
    eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=2, max_model_len=512, num_blocks=64, use_cuda_graph=False))
    seen = []
    eng.add_request("def retry(policy):", SamplingParams(max_tokens=5, temperature=0.0, ignore_eos=True),
                    on_token=lambda s, d, fin: seen.append((d, fin)))
    while eng.has_unfinished():
        eng.step()
    assert len(seen) == 5 and seen[-1][1] is True


def test_block_allocator_prefix_and_free():
    kv = KVCacheManager(num_blocks=32, block_size=4)
    free0 = kv.num_free
    s = Sequence("a", list(range(40)), SamplingParams())
    assert kv.ensure(s, 40) and len(s.blocks) == 10 and kv.num_free == free0 - 10
    assert KVCacheManager.SCRATCH_BLOCK not in s.blocks
    s.num_computed = 40
    kv.register_full_blocks(s)
    t = Sequence("b", list(range(40)) + [99], SamplingParams())
    got = kv.match_prefix(t)
    assert got == 40 and t.blocks == s.blocks
    kv.free(s)
    kv.free(t)
    assert kv.num_free == free0
    big = Sequence("c", list(range(1000)), SamplingParams())
    assert not kv.ensure(big, 1000)  # more blocks than exist: refused, nothing leaked
    assert kv.num_free == free0


def test_byte_bpe_roundtrip_and_chatml(tok):
    for text in ["def f(x):\n    return x * 2  # ünïcode ✓", "", "   spaces\t\ttabs\n\n"]:
        assert tok.decode(tok.encode(text)) == text
    msg = chatml([{"role": "system", "content": "be brief"}, {"role": "user", "content": "hi"}])
    assert msg.startswith(IM_START + "system\nbe brief" + IM_END) and msg.endswith(IM_START + "assistant\n")
    ids = tok.encode(msg)
    assert max(ids) < 512


def test_streaming_detokenizer_multibyte(tok):
    """Per-token deltas concatenate to the full decode even when a UTF-8 character
    spans tokens; the id->bytes table matches the native decoder."""
    text = "naïve café ✓ 日本語 — déjà vu; def f(): return 'ö'"
    ids = tok.encode(text)
    d = IncrementalDetokenizer(tok)
    deltas = [d.push(i) for i in ids] + [d.flush()]
    assert "".join(deltas) == text and all("\ufffd" not in x for x in deltas)
    for i in list(range(0, 600)) + [tok.special[IM_END]]:
        assert tok.token_bytes(i) == tok.decode_bytes([i])


def test_wordpiece_basic():
    wp = WordPieceTokenizer(2048)
    ids = wp.encode("Hello, World! retry_policy", max_len=16)
    assert ids[0] != ids[-1] and 2 < len(ids) <= 16
    assert all(0 <= i < 2048 for i in ids)
    assert wp.encode("hello world", 64) == wp.encode("HELLO world", 64)  # lowercasing
    assert np.asarray(wp.encode("x " * 500, 32)).shape == (32,)


def test_in_step_prefix_sharing(model, tok):
    """Prompts admitted in the SAME prefill step share their common full blocks: the first registers its
    prompt blocks when scheduled, the later ones match them (scheduler.py docstring) -- long (300-token)
    and short (40-token) shared prefixes alike, and a prefix split over chunked-prefill steps; outputs
    identical to an engine without prefix caching, and the prefill computes each shared block once."""
    for n_shared, chunk in ((300, 16384), (40, 16384), (300, 128)):
        base = [(7 * i) % 480 + 10 for i in range(n_shared)]
        prompts = [base + [1], base + [2], base + [3, 4]]
        eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=4, max_model_len=512, num_blocks=256,
                                                 use_cuda_graph=False, max_num_batched_tokens=chunk))
        outs = eng.generate(prompts, GREEDY)
        shared = n_shared // 16 * 16
        assert [o.cached_tokens for o in outs][1:] == [shared, shared], (n_shared, chunk)
        assert eng.stats["prefill_tokens"] == sum(len(p) for p in prompts) - 2 * shared
        _, ref = _gen(model, tok, prompts=prompts, enable_prefix_caching=False)
        assert [o.token_ids for o in outs] == [o.token_ids for o in ref]


def test_failed_prefill_step_unregisters_its_blocks(model, tok):
    """A prefill step that raises must not leave its (never written) prompt blocks in the prefix cache."""
    eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=4, max_model_len=512, num_blocks=256,
                                             use_cuda_graph=False))
    prompt = [(5 * i) % 400 + 3 for i in range(100)]
    eng.add_request(prompt, GREEDY)
    real = eng._run_prefill

    def boom(items):
        raise RuntimeError("injected fault")

    eng._run_prefill = boom
    with pytest.raises(RuntimeError):
        eng.step()
    eng._run_prefill = real
    assert eng.kv.stats()["cached_blocks"] == 0
    from githubrepostorag_amd.engine.sequence import Sequence

    probe = Sequence("p", prompt + [9], GREEDY)
    assert eng.kv.match_prefix(probe) == 0


def test_failed_prefill_step_rolls_back_sharers(model, tok):
    """Two prompts sharing a prefix are admitted in one step (the second matches blocks the first registered
    when scheduled); the step fails.  A caller that keeps stepping must get the outputs of a clean run: the
    sharer restarts its prefill, the owner re-registers its blocks once they are really computed."""
    cfg = EngineConfig(max_num_seqs=4, max_model_len=512, num_blocks=256, use_cuda_graph=False)
    shared = [(7 * i) % 300 + 5 for i in range(64)]
    p1, p2 = shared + [11, 12, 13], shared + [21, 22]

    def clean():
        e = LLMEngine(model, tok, cfg)
        return [c.token_ids for c in e.generate([p1, p2], GREEDY)]

    want = clean()
    eng = LLMEngine(model, tok, cfg)
    r1, r2 = eng.add_request(p1, GREEDY), eng.add_request(p2, GREEDY)
    real = eng._run_prefill
    seen = {}

    def boom(items):
        seen["items"] = [(s.req_id, a, b) for s, a, b in items]
        raise RuntimeError("injected fault")

    eng._run_prefill = boom
    with pytest.raises(RuntimeError):
        eng.step()
    eng._run_prefill = real
    assert [r for r, _, _ in seen["items"]] == [r1, r2]
    assert seen["items"][1][1] > 0  # the sharer had matched the owner's (unwritten) blocks
    s1, s2 = eng.get(r1), eng.get(r2)
    assert s1.num_computed == 0 and s2.num_computed == 0 and s1.block_hashes == [] and s2.blocks == []
    while eng.has_unfinished():
        eng.step()
    assert [eng.get(r).output_ids for r in (r1, r2)] == want
    probe = Sequence("p", shared + [9], GREEDY)
    assert eng.kv.match_prefix(probe) == 64  # the owner's blocks are registered again, now computed


def test_priority_admission_order(model, tok):
    """A high-priority request jumps the waiting queue (FCFS within a priority)."""
    eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=1, max_model_len=512, num_blocks=256,
                                             use_cuda_graph=False))
    lo = SamplingParams(max_tokens=3, temperature=0.0, ignore_eos=True)
    hi = SamplingParams(max_tokens=3, temperature=0.0, ignore_eos=True, priority=1)
    ids = [eng.add_request([5, 6, 7], lo)]
    eng.step()  # the first request is running; the next ones queue behind it
    ids += [eng.add_request([8, 9], lo), eng.add_request([3, 4], hi), eng.add_request([1, 2], hi)]
    while eng.has_unfinished():
        eng.step()
    order = sorted(ids, key=lambda r: eng.get(r).first_token_time)
    assert order == [ids[0], ids[2], ids[3], ids[1]]


def test_interactive_prefill_ahead_of_bulk_chunks(model, tok):
    """A higher-priority arrival takes the next step's prefill budget ahead of the remaining chunks of a bulk
    prompt already in chunked prefill (ingest running beside the serving loop); greedy outputs unchanged."""
    cfg = EngineConfig(max_num_seqs=4, max_model_len=512, num_blocks=256, max_num_batched_tokens=32,
                       use_cuda_graph=False)
    bulk = SamplingParams(max_tokens=3, temperature=0.0, ignore_eos=True)
    hi = SamplingParams(max_tokens=3, temperature=0.0, ignore_eos=True, priority=2)
    long_prompt = [(7 * i) % 200 + 3 for i in range(160)]  # 5 chunks of 32
    eng = LLMEngine(model, tok, cfg)
    rb = eng.add_request(long_prompt, bulk)
    eng.step()  # first chunk of the bulk prompt
    rh = eng.add_request([11, 12, 13, 14], hi)
    eng.step()
    h, b = eng.get(rh), eng.get(rb)
    assert h.num_computed == 4, h.num_computed  # the arrival was prefilled in this step ...
    assert b.num_computed == 32 + 28, b.num_computed  # ... and the bulk prompt took the rest of the budget
    while eng.has_unfinished():
        eng.step()
    ref = LLMEngine(model, tok, cfg)
    r1, r2 = ref.add_request(long_prompt, bulk), ref.add_request([11, 12, 13, 14], hi)
    while ref.has_unfinished():
        ref.step()
    assert eng.get(rb).output_ids == ref.get(r1).output_ids and eng.get(rh).output_ids == ref.get(r2).output_ids


def test_bulk_budget_caps_low_priority_prefill(model, tok):
    """``bulk_budget``: requests below INTERACTIVE_PRIORITY take at most that many of a step's prefill tokens;
    interactive ones are not capped (EngineRunner passes it while arrivals keep coming)."""
    from githubrepostorag_amd.engine.scheduler import INTERACTIVE_PRIORITY

    eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=4, max_model_len=512, num_blocks=256,
                                             max_num_batched_tokens=64, use_cuda_graph=False))
    bulk = SamplingParams(max_tokens=2, temperature=0.0, ignore_eos=True)
    hi = SamplingParams(max_tokens=2, temperature=0.0, ignore_eos=True, priority=INTERACTIVE_PRIORITY)
    rb = eng.add_request([(5 * i) % 200 + 3 for i in range(100)], bulk)
    eng.step(prefill_budget=64, bulk_budget=8)  # bulk alone: its 8-token share
    assert eng.get(rb).num_computed == 8
    rh = eng.add_request([(3 * i) % 200 + 3 for i in range(40)], hi)
    eng.step(prefill_budget=64, bulk_budget=8)  # a step carrying an interactive prompt carries no bulk
    assert eng.get(rh).num_computed == 40 and eng.get(rb).num_computed == 8
    eng.step(prefill_budget=64, bulk_budget=8)  # the interactive prompt decodes; bulk gets 8 more
    assert eng.get(rb).num_computed <= 16
    while eng.has_unfinished():
        eng.step()
    assert eng.get(rb).finish_reason and eng.get(rh).finish_reason


def test_mixed_prefill_decode_steps_identical(model, tok):
    """Decode tokens riding along in prefill steps (one weight pass for both)
    give the same greedy outputs as separate prefill / decode steps."""
    def run(mixed):
        eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=4, max_model_len=512, num_blocks=256,
                                                 max_num_batched_tokens=24, use_cuda_graph=False,
                                                 mixed_batches=mixed))
        ids = [eng.add_request(PROMPTS[0], GREEDY)]
        for p in PROMPTS[1:]:  # later arrivals prefill (in 24-token chunks) while the first decodes
            eng.step()
            ids.append(eng.add_request(p, GREEDY))
        while eng.has_unfinished():
            eng.step()
        return [eng.get(r).output_ids for r in ids], eng.stats["mixed_steps"]

    a, n_mixed = run(True)
    b, n_sep = run(False)
    assert a == b and n_mixed > 0 and n_sep == 0


def test_complete_many_wave_matches_single_calls(model, tok):
    """EngineLLM.complete_many (ingest waves: tokenised in the caller, submitted together) returns the
    same greedy completions as one complete() call per prompt."""
    from githubrepostorag_amd.agent.llm import EngineLLM
    from githubrepostorag_amd.engine.runner import EngineRunner

    eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=4, max_num_batched_tokens=64, use_cuda_graph=False))
    runner = EngineRunner(eng)
    try:
        llm = EngineLLM(runner, tok, max_tokens=5, mode="worker", timeout_s=60.0)
        ps = ["def retry(policy):", "explain the cache", "widgets", "billing module", "x = 1"]
        many = llm.complete_many(ps, temperature=0.0, repetition_penalty=1.0)
        single = [llm.complete(p, temperature=0.0, repetition_penalty=1.0) for p in ps]
        assert [m.text for m in many] == [s.text for s in single]
        assert all(not m.error for m in many)
    finally:
        runner.shutdown()


def test_lazy_detokenization_matches_streaming_text():
    """Requests without a token callback or stop strings are detokenized once at finish (host time per
    decode step); the text must equal what the per-token incremental decoder produces for the same ids."""
    from githubrepostorag_amd.engine.llm_engine import EngineConfig, LLMEngine
    from githubrepostorag_amd.engine.sequence import SamplingParams
    from githubrepostorag_amd.engine.tokenizer import ByteBPETokenizer
    from githubrepostorag_amd.models.configs import decoder_config
    from githubrepostorag_amd.models.qwen2 import Qwen2Model

    cfg = decoder_config("qwen2-tiny")
    model = Qwen2Model(cfg, device="cpu", seed=0)
    tok = ByteBPETokenizer(cfg.vocab_size)
    eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=4, max_model_len=256, num_blocks=64))
    prompts = [tok.encode("def retry(policy): " * n) for n in (1, 3)]
    sp = SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True)
    lazy = eng.generate(prompts, sp)
    seen = []
    streamed = [eng.add_request(p, sp, on_token=lambda s, d, f: seen.append(d)) for p in prompts]
    while eng.has_unfinished():
        eng.step()
    for rid, a in zip(streamed, lazy):
        b = eng.completion(eng.pop(rid))
        assert b.token_ids == a.token_ids and b.text == a.text and b.text
        assert a.text == eng._detok_all(a.token_ids)
    assert seen  # the streamed requests went through the per-token path


def test_over_long_prompt_rejected_by_engine_and_fitted_by_agent_llm(model, tok):
    """The prompt-length contract (vLLM --max-model-len, helm/templates/qwen-deployment.yaml:30-31): the
    engine rejects a prompt that leaves no room to generate instead of silently keeping its tail; the
    agent / ingest client cuts the MIDDLE (retrieved context) and keeps the head (system prompt +
    question) and the answer cue; the OpenAI endpoint answers 400."""
    from fastapi.testclient import TestClient

    from githubrepostorag_amd.agent.llm import EngineLLM
    from githubrepostorag_amd.config import Settings
    from githubrepostorag_amd.engine.llm_engine import PromptTooLongError
    from githubrepostorag_amd.engine.runner import EngineRunner
    from githubrepostorag_amd.service.api import APIState, create_app

    eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=4, max_model_len=128, num_blocks=64, use_cuda_graph=False))
    with pytest.raises(PromptTooLongError):
        eng.add_request(list(range(1, 200)), GREEDY)
    runner = EngineRunner(eng)
    try:
        llm = EngineLLM(runner, tok, max_tokens=8, mode="worker", timeout_s=60.0)
        ids = list(range(1, 300))
        fitted = llm.fit(ids, 8)
        assert len(fitted) <= 120 and fitted[:40] == ids[:40] and fitted[-20:] == ids[-20:]
        assert llm.fit(ids[:50], 8) == ids[:50]
        prompt = "SYSTEM RULES. Question: where are widgets?\n\nContext:\n" + "block text " * 400 + "\n\nAnswer:"
        r = llm.complete(prompt, temperature=0.0)
        assert not r.error and isinstance(r.text, str)

        class RT:  # the OpenAI endpoint over this runner
            settings = Settings(index_dir=None, data_dir=None, job_timeout_s=30.0)
            tokenizer = tok

        RT.runner = runner
        with TestClient(create_app(APIState(runtime=RT()))) as client:
            bad = client.post("/v1/completions", json={"prompt": "x " * 400, "max_tokens": 4})
            assert bad.status_code == 400 and "maximum context length is 128" in bad.json()["detail"]
            ok = client.post("/v1/completions", json={"prompt": "hello", "max_tokens": 4, "temperature": 0})
            assert ok.status_code == 200 and ok.json()["choices"][0]["finish_reason"] in ("length", "stop")
            # vLLM: prompt + max_tokens beyond max_model_len is a 400, not a completion cut short at the limit
            n = len(tok.encode("hello"))
            over = client.post("/v1/completions", json={"prompt": "hello", "max_tokens": 129 - n})
            assert over.status_code == 400 and "in the completion" in over.json()["detail"]
            fits = client.post("/v1/completions", json={"prompt": "hello", "max_tokens": 128 - n, "temperature": 0})
            assert fits.status_code == 200
            # chat with max_tokens unset: up to max_model_len (vLLM's default), not a 400
            unset = client.post("/v1/chat/completions", json={"messages": [{"role": "user", "content": "hello"}],
                                                               "temperature": 0})
            assert unset.status_code == 200, unset.text
    finally:
        runner.shutdown()


def test_engine_llm_acomplete_many_coroutines_and_cancel(model, tok):
    """EngineLLM.acomplete: 48 concurrent coroutines share the engine through awaited futures (no thread per
    call) and get the same text as the blocking complete(); a cancel check aborts an in-flight call."""
    import asyncio

    from githubrepostorag_amd.agent.graph_agent import Cancelled
    from githubrepostorag_amd.agent.llm import EngineLLM
    from githubrepostorag_amd.engine.runner import EngineRunner

    eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=16, max_model_len=512, num_blocks=512,
                                             use_cuda_graph=False))
    runner = EngineRunner(eng)
    try:
        llm = EngineLLM(runner, tok, max_tokens=6, mode="worker", timeout_s=120.0)
        prompts = [f"question number {i} about widgets" for i in range(48)]
        want = [llm.complete(p, temperature=0.0).text for p in prompts[:4]]

        async def many():
            return await asyncio.gather(*[llm.acomplete(p, temperature=0.0) for p in prompts])

        got = asyncio.run(many())
        assert [r.text for r in got[:4]] == want and not any(r.error for r in got)
        llm.CANCEL_POLL_S = 0.01
        flag = {"c": False}

        async def cancelled():
            async def flip():
                await asyncio.sleep(0.02)
                flag["c"] = True
            asyncio.ensure_future(flip())
            return await llm.acomplete("a long answer please", max_tokens=400, ignore_eos=True,
                                       cancel_check=lambda: flag["c"])

        with pytest.raises(Cancelled):
            asyncio.run(cancelled())
    finally:
        runner.shutdown()


def test_interactive_reserve_beside_bulk_admissions():
    """While interactive traffic is on (a bulk budget is passed), bulk admissions leave the reserve of slots
    and KV blocks free, so an interactive arrival is admitted at the next step instead of waiting for bulk
    sequences to finish; without interactive traffic bulk work may use every slot.  Preemption takes a bulk
    sequence before an interactive one."""
    from githubrepostorag_amd.engine.scheduler import KVCacheManager, Scheduler
    from githubrepostorag_amd.engine.sequence import SamplingParams, Sequence

    def mk(n_slots, reserve):
        kv = KVCacheManager(num_blocks=400, block_size=16)
        return Scheduler(kv, n_slots, 16384, 4096, mixed_batches=False, reserve_seqs=reserve,
                         reserve_tokens=16 * 16 if reserve else 0)

    bulk = [Sequence(f"b{i}", list(range(100 + i, 164 + i)), SamplingParams(priority=0)) for i in range(12)]
    sch = mk(8, 2)
    for s in bulk:
        sch.add(s)
    kind, items = sch.schedule(4096, bulk_budget=4096)
    assert kind == "prefill" and len(items) == 6  # 8 slots - 2 reserved
    q = Sequence("q", list(range(7, 71)), SamplingParams(priority=2))
    sch.add(q)
    kind, items = sch.schedule(4096, bulk_budget=512)
    assert [it[0].req_id for it in items] == ["q"]  # admitted at once, and the step carries no bulk prefill
    # no interactive traffic: bulk work takes every slot
    sch2 = mk(8, 2)
    for s in [Sequence(f"c{i}", list(range(64)), SamplingParams(priority=0)) for i in range(12)]:
        sch2.add(s)
    kind, items = sch2.schedule(4096)
    assert len(items) == 8
    # preemption victim: lowest priority first
    sch.running.sort(key=lambda s: s.arrival)
    assert sch._preempt_one(keep=sch.running[0]) and q in sch.running


def test_queue_order_key_puts_older_jobs_first():
    """SamplingParams.order (an agent job's start time on each of its calls): within a priority the waiting
    queue and the chunked-prefill pass go by the key, so an older job's next call is admitted / prefilled
    before newer jobs' calls; requests without a key keep FCFS by arrival; priority still comes first."""
    from githubrepostorag_amd.engine.scheduler import KVCacheManager, Scheduler

    sch = Scheduler(KVCacheManager(num_blocks=400, block_size=16), 2, 4096, 4096, mixed_batches=False)
    mk = lambda name, **kw: Sequence(name, list(range(3, 200)), SamplingParams(**kw))  # noqa: E731
    for s in (mk("new1", order=30.0), mk("new2", order=31.0), mk("old", order=10.0), mk("mid", order=20.0),
              mk("synth", priority=3, order=40.0), mk("plain")):
        sch.add(s)
    # "plain" has no key: its arrival (perf_counter, far above these keys) queues it last
    assert [s.req_id for s in sch.waiting] == ["synth", "old", "mid", "new1", "new2", "plain"]
    kind, items = sch.schedule(4096)  # two slots: the synthesize call and the oldest job's call
    assert kind == "prefill" and [it[0].req_id for it in items] == ["synth", "old"]
    # the newest job (by key) is the preemption victim among equal priorities
    sch.running.append(sch.waiting.popleft())  # "mid" as if admitted too
    assert sch._preempt_one(keep=sch.running[0]) and [s.req_id for s in sch.running] == ["synth", "old"]


def test_pacing_hold_lasts_while_bulk_work_is_in_flight(model, tok):
    """The arrival-pacing hold applies while bulk (ingest) requests are in flight -- not only for a few seconds
    after their submit, which dropped it in the middle of an ingest wave's long decode -- and ends once they
    finish and the recent-submit window has passed."""
    from githubrepostorag_amd.engine.runner import EngineRunner

    eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=4, max_num_batched_tokens=64, use_cuda_graph=False))
    runner = EngineRunner(eng)
    try:
        hs = [runner.submit([5, 6, 7, 8 + i], SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True),
                            interactive=False) for i in range(3)]
        assert runner._bulk_live == 3
        runner._last_bulk = -1e9  # the recent-submit window is long gone: in-flight bulk work alone holds
        assert runner._hold(time.monotonic()) == runner.PACE_HOLD_S or all(h.done.is_set() for h in hs)
        for h in hs:
            h.wait(60)
        assert runner._bulk_live == 0
        assert runner._hold(time.monotonic()) == 0.0
        h = runner.submit([9, 9, 9], SamplingParams(max_tokens=2, temperature=0.0, ignore_eos=True))
        h.wait(60)
        assert runner._bulk_live == 0  # interactive requests are not counted
    finally:
        runner.shutdown()


def test_bulk_reserve_grows_with_live_interactive_sequences():
    """While interactive traffic is on, bulk admissions leave free the fixed reserve PLUS half the live
    interactive sequences (slots and their prompt blocks): bulk work cannot fill the slots the next queries
    need.  The interactive count follows admissions, finishes and preemptions."""
    from githubrepostorag_amd.engine.scheduler import KVCacheManager, Scheduler

    sch = Scheduler(KVCacheManager(num_blocks=2000, block_size=16), 40, 1 << 20, 4096, mixed_batches=False,
                    reserve_seqs=2, reserve_tokens=0)
    inter = [Sequence(f"q{i}", list(range(1, 65)), SamplingParams(priority=2)) for i in range(12)]
    for s in inter:
        sch.add(s)
    sch.schedule(1 << 20, bulk_budget=1 << 20)
    assert sch.n_interactive == 12
    for q in inter:  # their prompts ran (the engine would advance this)
        q.num_computed = len(q.prompt_ids)
    bulk = [Sequence(f"b{i}", list(range(100 + i, 164 + i)), SamplingParams(priority=0)) for i in range(40)]
    for s in bulk:
        sch.add(s)
    sch.schedule(1 << 20, bulk_budget=1 << 20)
    # 40 slots - (2 fixed + 12 // 2) reserved = 32 running at most with bulk admissions
    assert len(sch.running) == 40 - 2 - 6
    sch.finish(inter[0])
    assert sch.n_interactive == 11
    sch._preempt_one(keep=bulk[0])  # a bulk victim first: the interactive count is unchanged
    assert sch.n_interactive == 11
