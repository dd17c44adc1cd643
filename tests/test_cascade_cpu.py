"""Shared-prefix decode planning (ops/attention.prefix_groups) and its engine plumbing on CPU: which rows
group, the prefix length each group shares, the saved-keys rule, and an engine whose decode rows share cached
prompt blocks producing the same tokens with the shared-prefix layout as without it.  The kernel numerics are
in test_cascade_gpu.py."""
import numpy as np
import pytest
import torch

from githubrepostorag_amd.engine.llm_engine import EngineConfig, LLMEngine
from githubrepostorag_amd.engine.sequence import SamplingParams
from githubrepostorag_amd.engine.tokenizer import ByteBPETokenizer
from githubrepostorag_amd.models.configs import decoder_config
from githubrepostorag_amd.models.qwen2 import Qwen2Model
from githubrepostorag_amd.ops.attention import prefix_groups


def _table(rows, width=None):
    width = width or max(len(r) for r in rows)
    bt = np.zeros((len(rows), width), dtype=np.int32)
    for i, r in enumerate(rows):
        bt[i, :len(r)] = r
    return bt


def test_groups_follow_common_leading_blocks():
    a = list(range(100, 120))  # 20 shared blocks
    b = list(range(200, 210))  # 10
    rows = [a + [1, 2], a + [3], a + [4, 5, 6], b + [7], b + [8], [9] * 12, list(range(300, 330))]
    L = np.array([(len(r) - 1) * 16 + 5 for r in rows])
    pre, spans, saved = prefix_groups(_table(rows), L, 16, G=7)
    assert spans == [(0, 3), (3, 5)]
    assert pre.tolist() == [320, 320, 320, 160, 160, 0, 0]
    assert saved == 2 * 320 + 160


def test_current_block_and_min_blocks_limit_the_prefix():
    a = list(range(10, 40))
    # identical block lists (e.g. a stale table tail): only blocks wholly before the current token count
    rows = [a, a]
    L = np.array([20 * 16 + 3, 30 * 16])  # row 0's current token is in block 20; row 1's in block 29
    pre, spans, _ = prefix_groups(_table(rows), L, 16, G=7)
    assert spans == [(0, 2)] and pre.tolist() == [320, 320]
    short = [list(range(50, 57)) + [1], list(range(50, 57)) + [2]]  # 7 shared blocks < min_blocks 8
    assert prefix_groups(_table(short), np.array([8 * 16, 8 * 16]), 16, G=7) is None


def test_group_cap_and_saved_keys_rule():
    a = list(range(1000, 1064))
    rows = [a + [i] for i in range(9)]  # 9 rows share 64 blocks; G = 7, rg = 2: 4 members per group
    L = np.array([64 * 16 + 9] * 9)
    pre, spans, saved = prefix_groups(_table(rows), L, 16, G=7, rg=2)
    assert spans == [(0, 4), (4, 8)] and pre[8] == 0
    assert saved == 2 * 3 * 64 * 16
    # a fourth member that shares only 10 of the 40 blocks would cut the group's saved keys: it stays out
    x = list(range(500, 540))
    rows = [x + [1], x + [2], x[:10] + [3] * 30 + [4]]
    L = np.array([40 * 16 + 2] * 3)
    pre, spans, saved = prefix_groups(_table(rows), L, 16, G=7, rg=2)
    assert spans == [(0, 2)] and pre.tolist() == [640, 640, 0]


@pytest.fixture(scope="module")
def model():
    return Qwen2Model(decoder_config("qwen2-tiny"), device="cpu", dtype=torch.float32, seed=0, init_std=0.05)


def test_engine_groups_rows_on_cached_prefixes(model, monkeypatch):
    import githubrepostorag_amd.engine.llm_engine as LE

    monkeypatch.setattr(LE, "CASCADE_MIN_WAVES", 0)  # the tiny batch's prefix grid is far below the GPU gate
    tok = ByteBPETokenizer(512)
    sp = SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True)
    pa = [(3 * j) % 400 + 1 for j in range(200)]  # 12 full blocks of 16
    pb = [(7 * j + 5) % 400 + 1 for j in range(170)]
    prompts = [pa + [401 + i] for i in range(5)] + [pb + [420 + i] for i in range(3)] + [[9, 8, 7, 6] * 5]
    outs = {}
    for cas in (True, False):
        eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=16, max_model_len=512, num_blocks=512,
                                                 use_cuda_graph=False, cascade_decode=cas))
        eng.generate([pa + [400], pb + [400]], SamplingParams(max_tokens=1, temperature=0.0))  # cache prefixes
        outs[cas] = [o.token_ids for o in eng.generate(prompts, sp)]
        if cas:
            st = eng.stats
            assert st["cascade_windows"] >= 5 and st["cascade_rows"] >= 5 * 8
            assert st["cascade_saved_keys"] > 0.5 * st["decode_keys"]
        else:
            assert eng.stats["cascade_windows"] == 0
    assert outs[True] == outs[False]


def test_layout_cuts_prefixes_into_work_items():
    from githubrepostorag_amd.ops.attention import cascade_layout

    pre = np.array([640, 640, 640, 0, 160, 160, 4096, 4096], dtype=np.int32)
    spans = [(0, 3), (4, 6), (6, 8)]
    part, items, used = cascade_layout(pre.copy(), spans, 16, parts=4, min_part=256)
    # 640 keys -> 256-key parts (min part) x 3; 160 -> one part; 4096 -> 4 parts of 1024
    assert part.tolist() == [256, 256, 256, 0, 256, 256, 1024, 1024]
    got = [tuple(r) for r in items[:used]]
    assert got[:4] == [(0, 3, 0, 256), (0, 3, 256, 512), (0, 3, 512, 640), (4, 6, 0, 160)]
    assert got[4:] == [(6, 8, 1024 * j, 1024 * (j + 1)) for j in range(4)]
    assert (items[used:] == 0).all()
    # no room for a group's parts: that group drops out (its rows attend to all their keys themselves)
    pre2 = pre.copy()
    part, items, used = cascade_layout(pre2, spans, 5, parts=4, min_part=256)
    assert used == 4 and pre2[6] == 0 and pre2[7] == 0 and part[6] == 0 and part[0] == 256
