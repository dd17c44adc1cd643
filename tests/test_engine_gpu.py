"""End-to-end decoder engine on cuda:0: continuous batching, paged KV,
prefix cache, hipGraph decode vs eager decode, decode vs full recompute."""
import pytest
import torch

from githubrepostorag_amd.engine.llm_engine import EngineConfig, LLMEngine
from githubrepostorag_amd.engine.sequence import SamplingParams
from githubrepostorag_amd.engine.tokenizer import ByteBPETokenizer
from githubrepostorag_amd.models.configs import decoder_config
from githubrepostorag_amd.models.qwen2 import Qwen2Model

from _logits import greedy_within_tolerance

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup(dev):
    cfg = decoder_config("qwen2-small")
    model = Qwen2Model(cfg, device=dev, seed=0)
    tok = ByteBPETokenizer(cfg.vocab_size)
    return model, tok


def _prompts(tok):
    return [tok.encode("def retry(policy): " * n) for n in (1, 7, 33, 90)]


def test_graph_vs_eager_identical(setup):
    model, tok = setup
    sp = SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True)
    a = LLMEngine(model, tok, EngineConfig(max_num_seqs=8, max_model_len=2048, num_blocks=1024,
                                           use_cuda_graph=True)).generate(_prompts(tok), sp)
    b = LLMEngine(model, tok, EngineConfig(max_num_seqs=8, max_model_len=2048, num_blocks=1024,
                                           use_cuda_graph=False)).generate(_prompts(tok), sp)
    assert [x.token_ids for x in a] == [x.token_ids for x in b]


def test_decode_matches_recompute(setup, dev):
    """Greedy tokens of the batched engine (prefix cache, hipGraph decode windows, split-KV decode attention)
    against a prefill recompute of each full prefix: every chosen token's recomputed logit is within bf16
    noise (2 % of the logit scale) of the recompute's maximum — a logit tolerance, not an agreement rate."""
    model, tok = setup
    sp = SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True)
    eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=8, max_model_len=2048, num_blocks=1024))
    outs = eng.generate(_prompts(tok), sp)
    for p, o in zip(_prompts(tok), outs):
        assert len(o.token_ids) == 8
        greedy_within_tolerance(model, dev, p, o.token_ids)


def test_prefix_cache_and_sampling(setup):
    model, tok = setup
    eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=16, max_model_len=2048, num_blocks=1024))
    base = tok.encode("You are a senior developer assistant. " * 20)
    prompts = [base + tok.encode(f" question {i}") for i in range(12)]
    eng.generate(prompts[:1], SamplingParams(max_tokens=2, ignore_eos=True))
    outs = eng.generate(prompts[1:], SamplingParams(max_tokens=16, temperature=0.7, top_p=0.9,
                                                    repetition_penalty=1.2, ignore_eos=True))
    assert all(len(o.token_ids) == 16 for o in outs)
    assert all(o.cached_tokens > 0 for o in outs)
    st = eng.kv.stats()
    assert st["prefix_hits"] > 0


def test_multistep_window_sampling_and_stop(setup):
    """K-step decode windows (one hipGraph replay per window) must sample the
    same tokens as one-step eager decode — top-p + repetition penalty with a
    per-request seed — and stop exactly at a stop token met inside a window."""
    model, tok = setup
    sp = SamplingParams(max_tokens=19, temperature=0.7, top_p=0.9, repetition_penalty=1.2, ignore_eos=True, seed=5)
    mk = lambda g: LLMEngine(model, tok, EngineConfig(max_num_seqs=8, max_model_len=2048, num_blocks=1024,  # noqa
                                                      use_cuda_graph=g, decode_window=8))
    a = mk(True).generate(_prompts(tok), sp)
    b = mk(False).generate(_prompts(tok), sp)
    assert [x.token_ids for x in a] == [x.token_ids for x in b]
    stop_at = a[2].token_ids[5]
    first = a[2].token_ids.index(stop_at)
    sp2 = SamplingParams(max_tokens=19, temperature=0.7, top_p=0.9, repetition_penalty=1.2, ignore_eos=True, seed=5,
                         stop_token_ids=[stop_at])
    c = mk(True).generate(_prompts(tok), sp2)
    assert c[2].token_ids == a[2].token_ids[: first + 1] and c[2].finish_reason == "stop"


def test_long_context_chunked_prefill_and_split_kv_decode(dev):
    """prompts past the reference's --max-model-len (11712) up to
    32K run on one GPU through chunked prefill (4096-token chunks attending to
    the paged context) and split-KV decode; the generated tokens must match a
    one-token recompute of the full prefix in a single unchunked prefill."""
    cfg = decoder_config("qwen2-small", max_position=32768)
    model = Qwen2Model(cfg, device=dev, seed=5)
    tok = ByteBPETokenizer(cfg.vocab_size)
    g = torch.Generator().manual_seed(11)
    prompts = [torch.randint(10, 4000, (n,), generator=g).tolist() for n in (12000, 30000)]
    sp = SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True)
    eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=4, max_num_batched_tokens=4096, max_model_len=32768,
                                             num_blocks=4096))
    outs = eng.generate(prompts, sp)
    assert all(len(o.token_ids) == 4 for o in outs)
    del eng
    torch.cuda.empty_cache()
    for p, o in zip(prompts, outs):  # logit tolerance against one unchunked prefill of the whole prefix
        greedy_within_tolerance(model, dev, p, o.token_ids)


def test_sampler_scratch_outlives_graphs_captured_before_it_grew(setup, dev):
    """A decode graph captured at a small bucket keeps replaying after a larger bucket's warm-up grew the
    sampler scratch (the outgrown buffer is retired, not freed; the engine also reserves its largest
    bucket up front).  Replays must match the eager engine token for token."""
    from githubrepostorag_amd.ops.sampling import SamplerState

    s = SamplerState(4, 1000, dev)
    w1 = s.workspace(8)
    w2 = s.workspace(4096)
    assert w2.numel() > w1.numel() and any(r is w1 for r in s._retired)

    model, tok = setup
    sp = SamplingParams(max_tokens=10, temperature=0.7, top_p=0.9, ignore_eos=True, seed=3)
    cfg = dict(max_num_seqs=8, max_model_len=2048, num_blocks=1024,
               graph_batch_sizes=(1, 2, 4, 8, 320, 512))
    eng = LLMEngine(model, tok, EngineConfig(use_cuda_graph=True, **cfg))
    assert eng.sampler._ws.numel() >= int(__import__("githubrepostorag_amd.ops._lib", fromlist=["lib"]).lib()
                                          .grag_sample_ws_floats(512, model.cfg.vocab_size))
    eng.warmup_graphs([4, 8], max_ctx=2048, windows=(1,))
    old = eng.sampler._ws
    eng.sampler.workspace(2048)  # a regrowth after the small graphs were captured
    assert eng.sampler._ws is not old and any(r is old for r in eng.sampler._retired)
    eng.warmup_graphs([512], max_ctx=2048, windows=(1,))
    a = eng.generate(_prompts(tok), sp)
    b = LLMEngine(model, tok, EngineConfig(use_cuda_graph=False, **cfg)).generate(_prompts(tok), sp)
    assert [x.token_ids for x in a] == [x.token_ids for x in b]


def test_mixed_steps_match_separate_steps(setup, dev):
    """Stall-free batching (decode rows riding in prefill steps, their attention on the split-KV decode kernel,
    inputs from the per-slot block table) against separate prefill / hipGraph decode steps: every greedy token
    of the mixed engine passes the same logit-tolerance check against a prefill recompute."""
    model, tok = setup
    sp = SamplingParams(max_tokens=10, temperature=0.0, ignore_eos=True)
    eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=8, max_model_len=2048, num_blocks=1024,
                                             max_num_batched_tokens=64, mixed_batches=True))
    prompts = _prompts(tok)
    ids = [eng.add_request(prompts[0], sp)]
    for p in prompts[1:]:  # later arrivals prefill in 64-token chunks while the earlier ones decode
        eng.step()
        ids.append(eng.add_request(p, sp))
    while eng.has_unfinished():
        eng.step()
    assert eng.stats["mixed_steps"] > 0
    for p, r in zip(prompts, ids):
        out = eng.get(r).output_ids
        assert len(out) == 10
        greedy_within_tolerance(model, dev, p, out)
