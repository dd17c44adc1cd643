"""Shared-prefix ("cascade") decode attention (csrc/kernels/attention.hip paged_decode_prefix_kernel + the
per-sequence decode kernel over each row's own keys, merging the prefix parts) against the fp32 reference
paged_attention_ref over the full contexts, on cuda:0."""
import math

import numpy as np
import pytest
import torch

from githubrepostorag_amd.ops import attention as A

pytestmark = pytest.mark.gpu


def shared_prefix_batch(groups, Hq, Hkv, D, BS=16, seed=0):
    """groups: [(members, prefix_blocks)]; each member gets the group's prefix block ids plus its own blocks
    for a random 1..300-key suffix.  Returns q, caches, AttnMetadata (cpu), block table (numpy), ctx lens."""
    g = torch.Generator().manual_seed(seed)
    rs = np.random.RandomState(seed)
    rows = []  # (prefix ids, ctx)
    nb = 0
    for members, pb in groups:
        pre_ids = list(range(nb, nb + pb))
        nb += pb
        for _ in range(members):
            suf = int(rs.randint(1, 300))
            own = -(-(pb * BS + suf) // BS) - pb
            rows.append((pre_ids + list(range(nb, nb + own)), pb * BS + suf))
            nb += own
    NB = nb + 2
    perm = torch.randperm(NB, generator=g).numpy().astype(np.int32)  # scatter blocks over the cache
    width = max(len(ids) for ids, _ in rows)
    bt = np.zeros((len(rows), width), dtype=np.int32)
    for i, (ids, _) in enumerate(rows):
        bt[i, :len(ids)] = perm[ids]
    lens = [c for _, c in rows]
    B = len(rows)
    kc = torch.randn(NB, Hkv, BS, D, generator=g).to(torch.bfloat16)
    vc = torch.randn(NB, Hkv, BS, D, generator=g).to(torch.bfloat16)
    q = torch.randn(B, Hq, D, generator=g).to(torch.bfloat16)
    meta = A.AttnMetadata(q_start=torch.arange(B + 1, dtype=torch.int32), ctx_len=torch.tensor(lens, dtype=torch.int32),
                          block_tables=torch.from_numpy(bt), slot_mapping=torch.zeros(B, dtype=torch.int32),
                          max_q_len=1, num_seqs=B, num_tokens=B, is_decode=True)
    return q, kc, vc, meta, bt, lens


def _dev_meta(meta, dev):
    return A.AttnMetadata(q_start=meta.q_start.to(dev), ctx_len=meta.ctx_len.to(dev),
                          block_tables=meta.block_tables.to(dev), slot_mapping=meta.slot_mapping.to(dev),
                          max_q_len=1, num_seqs=meta.num_seqs, num_tokens=meta.num_tokens, is_decode=True)


def cascade_for(bt, lens, G, dev, B, n_items=None, min_part=256, rg=2, planes=16):
    r = A.prefix_groups(bt, np.asarray(lens), 16, G, rg=rg)
    assert r is not None
    pre, spans, saved = r
    part, items, used = A.cascade_layout(pre, spans, n_items or A.cascade_items(B), min_part=min_part)
    assert used > 0
    return A.Cascade(pre_len=torch.from_numpy(pre).to(dev), pre_part=torch.from_numpy(part).to(dev),
                     items=torch.from_numpy(items.reshape(-1)).to(dev), planes=planes,
                     pre_o=torch.full((planes * B * 64 * 128,), float("nan"), device=dev),
                     pre_ml=torch.full((planes * B * 64 * 2,), float("nan"), device=dev), rg=rg), spans, saved


@pytest.mark.parametrize("Hq,Hkv,D", [(28, 4, 128), (12, 2, 64), (16, 2, 128)])
@pytest.mark.parametrize("nsplit_len", [(1, 0), (2, 2048), (8, 256)])
@pytest.mark.parametrize("rg", [2, 4])
@pytest.mark.parametrize("parts", [(None, 256), (8, 512), (200, 32)])
def test_cascade_decode_matches_reference(dev, Hq, Hkv, D, nsplit_len, rg, parts):
    G = Hq // Hkv
    cap = 16 * rg // G
    groups = [(3, 40), (2, 20), (1, 9), (min(cap, 4), 70), (2, 8), (1, 0), (min(cap, 5), 131)]
    q, kc, vc, meta, bt, lens = shared_prefix_batch(groups, Hq, Hkv, D, seed=Hq + rg)
    B = len(lens)
    scale = 1 / math.sqrt(D)
    ref = A.paged_attention_ref(q, kc, vc, meta, scale).reshape(B, -1)
    m = _dev_meta(meta, dev)
    ns, sl = nsplit_len
    if ns > 1:
        ns = -(-max(lens) // sl)
        m.num_splits, m.split_len = ns, sl
        m.part_o = torch.empty(ns * B * Hq * D, dtype=torch.float32, device=dev)
        m.part_ml = torch.empty(ns * B * Hq * 2, dtype=torch.float32, device=dev)
    c, spans, saved = cascade_for(bt, lens, G, dev, B, n_items=parts[0], min_part=parts[1], rg=rg)
    assert saved > 0 and all(b - a >= 2 for a, b in spans)
    m.cascade = c
    qd, kd, vd = q.to(dev), kc.to(dev), vc.to(dev)
    for code in (3, 12):  # 2-stage ring; 3-stage ring with non-temporal loads
        m.extra = {"decode_nw": code}
        out = A.paged_attention(qd, kd, vd, m, scale)
        torch.cuda.synchronize()
        assert torch.isfinite(out.float()).all()
        err = (out.float().cpu() - ref.float()).abs().max().item()
        assert err < 2e-2, (code, err)


def test_cascade_graph_replay_and_guard(dev):
    """Captured once in a hipGraph and replayed with new group layouts / prefix lengths written into the same
    device tensors (what the engine's decode graphs do), then a corrupt prefix length: the index guard
    reports it and the row falls back to attending all its keys itself (still the exact answer)."""
    from githubrepostorag_amd.ops._lib import bind_error_guard, check_device_errors, device_errors, DeviceIndexError
    from githubrepostorag_amd.ops._lib import lib

    lib()
    assert bind_error_guard(0)
    check_device_errors("before")
    Hq, Hkv, D = 28, 4, 128
    scale = 1 / math.sqrt(D)
    layouts = [[(3, 40), (2, 20), (3, 90), (1, 3), (3, 12)], [(1, 5), (4, 60), (4, 33), (2, 9), (1, 50), (1, 1)]]
    batches = [shared_prefix_batch(gs, Hq, Hkv, D, seed=11 + i) for i, gs in enumerate(layouts)]
    B = max(len(b[5]) for b in batches)
    W = max(b[4].shape[1] for b in batches)
    NB = max(b[1].shape[0] for b in batches)
    kd = torch.zeros(NB, Hkv, 16, D, dtype=torch.bfloat16, device=dev)
    vd = torch.zeros_like(kd)
    qd = torch.zeros(B, Hq, D, dtype=torch.bfloat16, device=dev)
    bt_d = torch.zeros(B, W, dtype=torch.int32, device=dev)
    ctx_d = torch.ones(B, dtype=torch.int32, device=dev)
    pre_d = torch.zeros(B, dtype=torch.int32, device=dev)
    part_d = torch.zeros(B, dtype=torch.int32, device=dev)
    NI = A.cascade_items(B)
    items_d = torch.zeros(NI * 4, dtype=torch.int32, device=dev)
    npl = 16
    c = A.Cascade(pre_len=pre_d, pre_part=part_d, items=items_d, planes=npl,
                  pre_o=torch.zeros(npl * B * Hq * D, device=dev), pre_ml=torch.zeros(npl * B * Hq * 2, device=dev))
    m = A.AttnMetadata(q_start=torch.arange(B + 1, dtype=torch.int32, device=dev), ctx_len=ctx_d, block_tables=bt_d,
                       slot_mapping=torch.zeros(B, dtype=torch.int32, device=dev), max_q_len=1, num_seqs=B,
                       num_tokens=B, is_decode=True, cascade=c)
    m.extra = {"decode_nw": 3}
    out = torch.zeros(B, Hq * D, dtype=torch.bfloat16, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        A.paged_attention(qd, kd, vd, m, scale, out=out)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        A.paged_attention(qd, kd, vd, m, scale, out=out)
    for q, kc, vc, meta, bt, lens in batches:
        n = len(lens)
        pre, spans, _ = A.prefix_groups(bt, np.asarray(lens), 16, Hq // Hkv)
        part, items, _ = A.cascade_layout(pre, spans, NI)
        kd.zero_()
        vd.zero_()
        kd[: kc.shape[0]].copy_(kc)
        vd[: vc.shape[0]].copy_(vc)
        qd.zero_()
        qd[:n].copy_(q)
        bt_d.zero_()
        bt_d[:n, : bt.shape[1]].copy_(torch.from_numpy(bt))
        ctx_d.fill_(1)
        ctx_d[:n].copy_(meta.ctx_len)
        pre_d.zero_()
        pre_d[:n].copy_(torch.from_numpy(pre))
        part_d.zero_()
        part_d[:n].copy_(torch.from_numpy(part))
        items_d.copy_(torch.from_numpy(items.reshape(-1)))
        graph.replay()
        torch.cuda.synchronize()
        ref = A.paged_attention_ref(q, kc, vc, meta, scale).reshape(n, -1)
        err = (out[:n].float().cpu() - ref.float()).abs().max().item()
        assert err < 2e-2, err
    check_device_errors("replays")
    # a prefix length past a member's context: reported, and that row attends to all its keys itself
    q, kc, vc, meta, bt, lens = batches[-1]
    n = len(lens)
    bad = int(np.flatnonzero(pre_d[:n].cpu().numpy() == 0)[0])  # a row outside any group
    pre_d[bad] = lens[bad] + 5
    graph.replay()
    torch.cuda.synchronize()
    ref = A.paged_attention_ref(q, kc, vc, meta, scale).reshape(n, -1)
    assert (out[:n].float().cpu() - ref.float()).abs().max().item() < 2e-2
    codes, _, _, _ = device_errors()
    assert codes & (1 << 9)
    with pytest.raises(DeviceIndexError):
        check_device_errors("bad prefix")


def test_engine_decode_graphs_take_the_shared_prefix_path(dev, monkeypatch):
    """The engine end to end: rows whose prompts share cached blocks are grouped, the window takes the
    shared-prefix variant of its decode graph (cascade_windows > 0), and every greedy token stays within bf16
    tolerance of a prefill recompute of the full prefix."""
    import githubrepostorag_amd.engine.llm_engine as LE
    from githubrepostorag_amd.engine.sequence import SamplingParams
    from githubrepostorag_amd.engine.tokenizer import ByteBPETokenizer
    from githubrepostorag_amd.models.configs import decoder_config
    from githubrepostorag_amd.models.qwen2 import Qwen2Model

    from _logits import greedy_within_tolerance

    monkeypatch.setattr(LE, "CASCADE_MIN_WAVES", 0)  # 15 rows: a prefix grid far below the production gate
    cfg = decoder_config("qwen2-small")
    model = Qwen2Model(cfg, device=dev, seed=0)
    tok = ByteBPETokenizer(cfg.vocab_size)
    base = [tok.encode(f"shared context block {g}: the widgets module retries failed jobs. " * 16) for g in range(3)]
    eng = LE.LLMEngine(model, tok, LE.EngineConfig(max_num_seqs=32, max_model_len=2048, num_blocks=2048,
                                                   use_cuda_graph=True))
    eng.generate([b + [7] for b in base], SamplingParams(max_tokens=1, temperature=0.0))  # cache the prefixes
    prompts = [b + tok.encode(f" question {i}?") for b in base for i in range(5)]
    outs = eng.generate(prompts, SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True))
    st = eng.stats
    assert st["cascade_windows"] > 0 and st["cascade_saved_keys"] > 0.3 * st["decode_keys"], st
    assert st["graph_replays"] > 0
    for p, o in list(zip(prompts, outs))[::3]:
        assert len(o.token_ids) == 8
        greedy_within_tolerance(model, dev, p, o.token_ids)
