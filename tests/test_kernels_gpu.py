"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the
same op (run on cuda:0).  Inputs are random (not zero-filled), shapes are the
real model shapes where cheap."""
import math

import pytest
import torch

from githubrepostorag_amd.ops import attention as A
from githubrepostorag_amd.ops import elementwise as E
from githubrepostorag_amd.ops import norm as N
from githubrepostorag_amd.ops import sampling as S
from githubrepostorag_amd.ops import topk as K

pytestmark = pytest.mark.gpu


def rnd(*shape, dev, scale=1.0, dtype=torch.bfloat16, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dtype).to(dev)


def close(a, b, atol, rtol=2e-2):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    assert torch.allclose(a, b, atol=atol, rtol=rtol), f"max err {err}"


def test_lib_loads():
    from githubrepostorag_amd.ops import lib

    assert lib() is not None


@pytest.mark.parametrize("H", [384, 1536, 3584, 8192])
def test_rmsnorm(dev, H):
    x, r, w = rnd(37, H, dev=dev), rnd(37, H, dev=dev, seed=1), rnd(H, dev=dev, seed=2)
    y = N.rmsnorm(x, w, 1e-6)
    close(y, N.rmsnorm_ref(x.cpu(), w.cpu(), 1e-6), 3e-2)
    r1, r2 = r.clone(), r.cpu().clone()
    y = N.rmsnorm(x, w, 1e-6, residual=r1)
    yr = N.rmsnorm_ref(x.cpu(), w.cpu(), 1e-6, residual=r2)
    close(r1, r2, 1e-2)
    close(y, yr, 3e-2)


@pytest.mark.parametrize("H", [384, 1024])
def test_layernorm(dev, H):
    x, b, r = rnd(33, H, dev=dev), rnd(H, dev=dev, seed=1), rnd(33, H, dev=dev, seed=2)
    g, be = rnd(H, dev=dev, seed=3), rnd(H, dev=dev, seed=4)
    y = N.layernorm(x, g, be, 1e-12, bias=b, residual=r)
    close(y, N.layernorm_ref(x.cpu(), g.cpu(), be.cpu(), 1e-12, b.cpu(), r.cpu()), 5e-2)


def test_embeddings(dev):
    V, H, P = 1000, 384, 512
    word, pos, typ = rnd(V, H, dev=dev), rnd(P, H, dev=dev, seed=1), rnd(2, H, dev=dev, seed=2)
    g, b = rnd(H, dev=dev, seed=3), rnd(H, dev=dev, seed=4)
    ids = torch.randint(0, V, (50,), dtype=torch.int32).to(dev)
    pids = torch.arange(50, dtype=torch.int32).to(dev)
    y = N.bert_embed_ln(ids, pids, None, word, pos, typ, g, b, 1e-12)
    yr = N.bert_embed_ln_ref(ids.cpu(), pids.cpu(), None, word.cpu(), pos.cpu(), typ.cpu(), g.cpu(), b.cpu(), 1e-12)
    close(y, yr, 5e-2)
    close(N.embed_gather(ids, word), word.cpu()[ids.cpu().long()], 0)


def test_qkv_rope_kvstore(dev):
    T, Hq, Hkv, D, BS, NB = 29, 28, 4, 128, 16, 8
    qkv = rnd(T, (Hq + 2 * Hkv) * D, dev=dev)
    bias = rnd((Hq + 2 * Hkv) * D, dev=dev, seed=1)
    pos = torch.randint(0, 4000, (T,), dtype=torch.int32).to(dev)
    cs = E.rope_cos_sin(4096, D, 1e6, dev)
    slots = torch.randperm(NB * BS)[:T].to(torch.int32).to(dev)
    slots[3] = -1
    kc, vc = torch.zeros(NB, Hkv, BS, D, dtype=torch.bfloat16, device=dev), torch.zeros(NB, Hkv, BS, D,
                                                                                    dtype=torch.bfloat16, device=dev)
    kr, vr = kc.cpu().clone(), vc.cpu().clone()
    q = E.qkv_rope_kvstore(qkv, bias, pos, cs, slots, kc, vc, Hq, Hkv, D)
    qr = E.qkv_rope_kvstore_ref(qkv.cpu(), bias.cpu(), pos.cpu(), cs.cpu(), slots.cpu(), kr, vr, Hq, Hkv, D)
    close(q, qr, 3e-2)
    close(kc, kr, 3e-2)
    close(vc, vr, 1e-2)


@pytest.mark.parametrize("T", [1, 4, 16, 32, 48, 190, 240])
def test_qkv_rope_kvstore_from_splitk_planes(dev, T):
    """Qwen2-7B qkv at decode batches as deferred K-split planes (reduce folded into the RoPE / KV-store pass)
    against the unfused path (split-K reduce to bf16, then RoPE): identical q / K / V bits."""
    from githubrepostorag_amd.ops import gemm as G
    from githubrepostorag_amd.ops.linear import linear, linear_deferred

    Hq, Hkv, D, BS, NB, K = 28, 4, 128, 16, 64, 3584
    N = (Hq + 2 * Hkv) * D
    x = rnd(T, K, dev=dev, scale=0.5)
    w = rnd(N, K, dev=dev, scale=0.05, seed=1)
    bias = rnd(N, dev=dev, seed=2)
    pos = torch.randint(0, 4000, (T,), dtype=torch.int32).to(dev)
    cs = E.rope_cos_sin(4096, D, 1e6, dev)
    slots = torch.randperm(NB * BS)[:T].to(torch.int32).to(dev)
    part = linear_deferred(x, w)
    assert isinstance(part, G.SplitKPartial) and part.S > 1, G.deferred_plan(T, N, K)
    caches = [(torch.zeros(NB, Hkv, BS, D, dtype=torch.bfloat16, device=dev),
               torch.zeros(NB, Hkv, BS, D, dtype=torch.bfloat16, device=dev)) for _ in range(2)]
    q1 = E.qkv_rope_kvstore(part, bias, pos, cs, slots, *caches[0], Hq, Hkv, D)
    q2 = E.qkv_rope_kvstore(linear(x, w), bias, pos, cs, slots, *caches[1], Hq, Hkv, D)
    if T >= 33:  # linear() runs the same K-split plan + reduce there: identical bits
        assert torch.equal(q1, q2)
        assert torch.equal(caches[0][0], caches[1][0]) and torch.equal(caches[0][1], caches[1][1])
    else:  # 1-32 rows: linear() is the library / skinny GEMM (other accumulation order)
        close(q1, q2, 3e-2)
        close(caches[0][0], caches[1][0], 3e-2)
        close(caches[0][1], caches[1][1], 3e-2)


def test_silu_mul_bias_act(dev):
    gu = rnd(17, 2 * 1024, dev=dev)
    close(E.silu_mul(gu), E.silu_mul(gu.cpu()), 2e-2)
    for T in (192, 2051):  # one row per thread (decode) / 8 rows per thread with a ragged tail (prefill)
        gu = rnd(T, 2 * 18944, dev=dev, seed=T)
        close(E.silu_mul(gu), E.silu_mul(gu.cpu()), 2e-2)
    x, b = rnd(17, 1536, dev=dev), rnd(1536, dev=dev, seed=1)
    close(E.bias_act(x, b, E.ACT_GELU), E.bias_act(x.cpu(), b.cpu(), E.ACT_GELU), 2e-2)


@pytest.mark.parametrize("mode", [E.POOL_MEAN, E.POOL_CLS])
def test_pool_l2norm(dev, mode):
    lens = torch.tensor([5, 1, 17, 9], dtype=torch.int32)
    starts = torch.cat([torch.zeros(1, dtype=torch.int32), lens.cumsum(0)[:-1].to(torch.int32)])
    h = rnd(int(lens.sum()), 768, dev=dev)
    f = E.pool_l2norm(h, starts.to(dev), lens.to(dev), mode)
    close(f, E.pool_l2norm_ref(h.cpu(), starts, lens, mode), 1e-2)


def _paged_setup(dev, lens_q, lens_ctx, Hq, Hkv, D, BS=16, seed=0):
    g = torch.Generator().manual_seed(seed)
    nseq = len(lens_q)
    nblk = [(c + BS - 1) // BS for c in lens_ctx]
    NB = sum(nblk) + 3
    perm = torch.randperm(NB, generator=g) + 0
    width = max(nblk)
    bt = torch.zeros(nseq, width, dtype=torch.int32)
    o = 0
    for s in range(nseq):
        bt[s, : nblk[s]] = perm[o:o + nblk[s]]
        o += nblk[s]
    kc = (torch.randn(NB, Hkv, BS, D, generator=g)).to(torch.bfloat16)
    vc = (torch.randn(NB, Hkv, BS, D, generator=g)).to(torch.bfloat16)
    T = sum(lens_q)
    q = (torch.randn(T, Hq, D, generator=g)).to(torch.bfloat16)
    qs = torch.tensor([0] + list(torch.tensor(lens_q).cumsum(0)), dtype=torch.int32)
    meta = A.AttnMetadata(q_start=qs, ctx_len=torch.tensor(lens_ctx, dtype=torch.int32), block_tables=bt,
                          slot_mapping=torch.zeros(T, dtype=torch.int32), max_q_len=max(lens_q), num_seqs=nseq,
                          num_tokens=T)
    return q, kc, vc, meta


def _to(meta, dev):
    return A.AttnMetadata(q_start=meta.q_start.to(dev), ctx_len=meta.ctx_len.to(dev),
                          block_tables=meta.block_tables.to(dev), slot_mapping=meta.slot_mapping.to(dev),
                          max_q_len=meta.max_q_len, num_seqs=meta.num_seqs, num_tokens=meta.num_tokens)


@pytest.mark.parametrize("Hq,Hkv,D", [(28, 4, 128), (12, 2, 128), (16, 16, 64), (14, 2, 64)])
def test_paged_prefill(dev, Hq, Hkv, D):
    lens_q = [37, 130, 1, 64]
    lens_ctx = [37, 200, 70, 64]  # seq 1 and 2 have cached prefixes (chunked prefill)
    q, kc, vc, meta = _paged_setup(dev, lens_q, lens_ctx, Hq, Hkv, D)
    scale = 1 / math.sqrt(D)
    ref = A.paged_attention_ref(q, kc, vc, meta, scale).reshape(q.shape[0], -1)
    for code in (4, 5, 6):  # register-staged 4-wave; LDS-DMA 8-wave (2-stage / staggered 3-stage ring)
        m = _to(meta, dev)
        m.extra = {"prefill_nw": code}
        out = A.paged_attention(q.to(dev), kc.to(dev), vc.to(dev), m, scale)
        close(out, ref, 2e-2)


def test_paged_prefill_long_context(dev):
    """Chunked prefill deep into a long context (many K/V tiles, a block-table
    window wider than one tile, 256-row workgroups cut by the GQA packing)."""
    Hq, Hkv, D = 28, 4, 128
    lens_q = [300, 5, 513]
    lens_ctx = [2100, 1030, 513]
    q, kc, vc, meta = _paged_setup(dev, lens_q, lens_ctx, Hq, Hkv, D, seed=7)
    scale = 1 / math.sqrt(D)
    ref = A.paged_attention_ref(q, kc, vc, meta, scale).reshape(q.shape[0], -1)
    for code in (4, 5, 6):
        m = _to(meta, dev)
        m.extra = {"prefill_nw": code}
        close(A.paged_attention(q.to(dev), kc.to(dev), vc.to(dev), m, scale), ref, 2e-2)


def test_paged_prefill_block_size_fallback(dev):
    """KV blocks of 32 are outside the 8-wave kernel's compiled block size: the launcher runs the 4-wave
    kernel for the same request (codes 5/6 must still return the right answer, not an error)."""
    Hq, Hkv, D = 28, 4, 128
    q, kc, vc, meta = _paged_setup(dev, [40, 90], [40, 150], Hq, Hkv, D, BS=32, seed=9)
    scale = 1 / math.sqrt(D)
    ref = A.paged_attention_ref(q, kc, vc, meta, scale).reshape(q.shape[0], -1)
    for code in (5, 6):
        m = _to(meta, dev)
        m.extra = {"prefill_nw": code}
        close(A.paged_attention(q.to(dev), kc.to(dev), vc.to(dev), m, scale), ref, 2e-2)


@pytest.mark.parametrize("nsplit_len", [(1, 0), (4, 64), (8, 128)])
def test_paged_decode(dev, nsplit_len):
    Hq, Hkv, D = 28, 4, 128
    lens_ctx = [1, 17, 300, 1200, 64]
    q, kc, vc, meta = _paged_setup(dev, [1] * 5, lens_ctx, Hq, Hkv, D, seed=3)
    scale = 1 / math.sqrt(D)
    m = _to(meta, dev)
    m.is_decode = True
    ns, sl = nsplit_len
    if ns > 1:
        ns = -(-1200 // sl)
        m.num_splits, m.split_len = ns, sl
        m.part_o = torch.empty(ns * 5 * Hq * D, dtype=torch.float32, device=dev)
        m.part_ml = torch.empty(ns * 5 * Hq * 2, dtype=torch.float32, device=dev)
    ref = A.paged_attention_ref(q, kc, vc, meta, scale).reshape(q.shape[0], -1)
    for code in (1, 3, 8, 7, 11, 12, 2):  # 64-key LDS-DMA tiles, 32-key tiles in a 2 / 3 / 4-stage ring (11 / 12: 2 / 3 stages, nt loads), generic kernel
        m.extra = {"decode_nw": code}
        out = A.paged_attention(q.to(dev), kc.to(dev), vc.to(dev), m, scale)
        close(out, ref, 2e-2)


@pytest.mark.parametrize("Hq,Hkv,D", [(28, 4, 128), (14, 2, 64)])
@pytest.mark.parametrize("sl", [0, 32, 128, 256])
def test_paged_decode_small_batch_mw(dev, Hq, Hkv, D, sl):
    """The small-batch decode kernel (2 / 4 waves per split, in-launch last-arriver merge of the splits):
    sequences with different split counts (early-exit workgroups), a 1-key context, a context ending
    mid-tile; replayed three times in one hipGraph (the tickets reset themselves) against the fp32 reference."""
    lens_ctx = [1, 45, 300, 1200, 4100]
    B = len(lens_ctx)
    q, kc, vc, meta = _paged_setup(dev, [1] * B, lens_ctx, Hq, Hkv, D, seed=5)
    scale = 1 / math.sqrt(D)
    ref = A.paged_attention_ref(q, kc, vc, meta, scale).reshape(B, -1)
    A.decode_counters(dev)
    for code in (22, 24):
        m = _to(meta, dev)
        m.is_decode = True
        if sl:
            ns = -(-max(lens_ctx) // sl)
            m.num_splits, m.split_len = ns, sl
            m.part_o = torch.empty(ns * B * Hq * D, dtype=torch.float32, device=dev)
            m.part_ml = torch.empty(ns * B * Hq * 2, dtype=torch.float32, device=dev)
        m.extra = {"decode_nw": code}
        qd, kd, vd = q.to(dev), kc.to(dev), vc.to(dev)
        out = A.paged_attention(qd, kd, vd, m, scale)
        close(out, ref, 2e-2)
        o2 = torch.empty_like(out)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(3):
                A.paged_attention(qd, kd, vd, m, scale, out=o2)
        for _ in range(2):
            o2.zero_()
            g.replay()
            torch.cuda.synchronize()
            close(o2, ref, 2e-2)
        assert int(A.decode_counters(dev)[: B * Hkv].abs().sum()) == 0


@pytest.mark.parametrize("H,D", [(12, 32), (12, 64), (16, 64)])
def test_varlen_attention(dev, H, D):
    lens = [5, 130, 64, 1]
    st = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32)
    qkv = rnd(int(st[-1]), 3 * H * D, dev=dev)
    out = A.varlen_attention(qkv, st.to(dev), torch.tensor(lens, dtype=torch.int32).to(dev), max(lens), H, D,
                             1 / math.sqrt(D))
    close(out, A.varlen_attention_ref(qkv.cpu(), st, H, D, 1 / math.sqrt(D)), 2e-2)


def _unit(n, d, dev, seed):
    x = rnd(n, d, dev=dev, dtype=torch.float32, seed=seed)
    return (x / x.norm(dim=1, keepdim=True)).to(torch.bfloat16)


@pytest.mark.parametrize("nq,k,d", [(1, 10, 384), (5, 16, 1024), (40, 10, 768), (64, 8, 256), (20, 32, 384),
                                    (32, 5, 32), (40, 10, 64), (16, 8, 96)])
def test_score_topk(dev, nq, k, d):
    X = _unit(20000, d, dev, 1)
    Q = _unit(nq, d, dev, 2)
    s, i = K.score_topk(X, Q, k)
    rs, ri = K.score_topk_ref(X.cpu(), Q.cpu(), k)
    close(s, rs, 2e-3, 1e-3)
    # ids agree except for near-ties
    agree = (i.cpu() == ri).float().mean().item()
    assert agree > 0.97, agree


def test_score_topk_filters(dev):
    X = _unit(5000, 384, dev, 3)
    Q = _unit(3, 384, dev, 4)
    col = torch.randint(0, 5, (5000,), dtype=torch.int32).to(dev)
    bits = torch.randint(0, 8, (5000,), dtype=torch.int32).to(dev)
    preds = [K.Predicate(col, 2), K.Predicate(bits, 4, K.OP_BITAND)]
    s, i = K.score_topk(X, Q, 10, preds=preds)
    predc = [K.Predicate(col.cpu(), 2), K.Predicate(bits.cpu(), 4, K.OP_BITAND)]
    rs, ri = K.score_topk_ref(X.cpu(), Q.cpu(), 10, preds=predc)
    close(s, rs, 2e-3, 1e-3)
    assert ((i.cpu() == ri).float().mean() > 0.95)
    # per-query predicates (graph traversal batch)
    sel = torch.tensor([0, -1, 0], dtype=torch.int32)
    vals = torch.tensor([3, 0, 1], dtype=torch.int32)
    s2, i2 = K.score_topk(X, Q, 5, qpred=([col], sel.to(dev), vals.to(dev)))
    rs2, ri2 = K.score_topk_ref(X.cpu(), Q.cpu(), 5, qpred=([col.cpu()], sel, vals))
    close(s2, rs2, 2e-3, 1e-3)


def test_ivf_recall(dev):
    from githubrepostorag_amd.index.ivf import IVFIndex
    from githubrepostorag_amd.utils.synthetic import clustered_vectors

    X = clustered_vectors(100_000, 256, n_centers=256, device=dev, seed=5)
    ivf = IVFIndex(256, 128, dev)
    ivf.train(X[:20000], iters=6)
    ivf.add(X)
    Q = X[torch.randint(0, 100_000, (37,))].float() + 0.05 * torch.randn(37, 256, device=dev) / 16
    Q = (Q / Q.norm(dim=1, keepdim=True)).to(torch.bfloat16)
    s, i = ivf.search(Q, 10, nprobe=16)
    fs, fi = K.score_topk(X, Q, 10)
    rec = sum(len(set(a) & set(b)) for a, b in zip(i.cpu().tolist(), fi.cpu().tolist())) / (37 * 10)
    assert rec > 0.8, rec


def test_sampler(dev):
    V = 152064
    st = S.SamplerState(4, V, dev, seed=1)
    logits = rnd(3, V, dev=dev, dtype=torch.float32, scale=3.0)
    st.reset_slot(0, 0.0, 1.0, 0, 1.0, [])
    st.reset_slot(1, 0.7, 0.9, 0, 1.3, [5, 6, 7])
    st.reset_slot(2, 1.0, 1.0, 5, 1.0, [])
    slots = torch.tensor([0, 1, 2], dtype=torch.int32, device=dev)
    out = S.sample(logits, st, slots)
    assert int(out[0]) == int(logits[0].argmax())
    top5 = set(logits[2].topk(5).indices.tolist())
    for _ in range(20):
        o = S.sample(logits, st, slots)
        assert int(o[2]) in top5
    # top-p: every sampled token lies inside the nucleus of the penalised, tempered distribution
    x = logits[1].float().clone()
    x[[5, 6, 7]] = torch.where(x[[5, 6, 7]] > 0, x[[5, 6, 7]] / 1.3, x[[5, 6, 7]] * 1.3)
    p = torch.softmax(x / 0.7, 0)
    sp, si = p.sort(descending=True)
    nucleus = set(si[: int((sp.cumsum(0) < 0.9).sum()) + 1].tolist())
    assert int(out[1]) in nucleus
    # bf16 logits path + seen-bit bookkeeping
    out2 = S.sample(logits.to(torch.bfloat16), st, slots)
    assert out2.shape == (3,)


@pytest.mark.parametrize("M,N,K", [(1, 4608, 3584), (7, 3584, 3584), (33, 1000, 512), (64, 37888, 3584),
                                   (64, 3584, 18944), (50, 2048, 128)])
def test_gemm_skinny(dev, M, N, K):
    from githubrepostorag_amd.ops.linear import gemm_skinny

    x = rnd(M, K, dev=dev, scale=0.5)
    w = rnd(N, K, dev=dev, scale=0.05, seed=1)
    b = rnd(N, dev=dev, seed=2)
    y = gemm_skinny(x, w, b)
    ref = x.float().cpu() @ w.float().cpu().T + b.float().cpu()
    close(y, ref, 3e-2, 2e-2)
    for nt in (16, 32, 64):
        close(gemm_skinny(x, w, None, nt), ref - b.float().cpu(), 3e-2, 2e-2)


@pytest.mark.parametrize("M,N,K", [(64, 3584, 18944), (64, 4608, 3584), (37, 1000, 512), (17, 3584, 3696),
                                   (128, 3584, 3584), (9, 2048, 1024)])
def test_gemm_stream(dev, M, N, K):
    """Stream-K weight-streaming GEMM: auto plan + forced (mt, bn, grid) plans —
    tiles split across 1..many workgroups (slab + in-launch last-arriver
    combine), a K % 64 != 0 tail, M not a multiple of 16."""
    from githubrepostorag_amd.ops.linear import gemm_stream

    x = rnd(M, K, dev=dev, scale=0.5)
    w = rnd(N, K, dev=dev, scale=0.05, seed=1)
    b = rnd(N, dev=dev, seed=2)
    ref = x.float().cpu() @ w.float().cpu().T
    close(gemm_stream(x, w, b), ref + b.float().cpu(), 3e-2, 2e-2)
    for plan in ((4, 128, 256), (4, 64, 100), (2, 128, 37), (2, 64, 512), (4, 256, 3), (2, 256, 1), (4, 256, 256)):
        for _ in range(2):  # second call re-uses the ticket counters the first call reset
            close(gemm_stream(x, w, None, plan), ref, 3e-2, 2e-2)


def test_sampler_matches_reference_stream(dev):
    """The HIP sampler and the CPU reference share the counter-based Gumbel
    stream: same logits + state -> the same token (up to rare rounding ties)."""
    V, B = 5000, 16
    g = torch.Generator().manual_seed(11)
    logits = torch.randn(B, V, generator=g) * 3
    agree = 0
    for dev_state in (True,):
        st_g = S.SamplerState(B, V, dev, seed=123)
        st_c = S.SamplerState(B, V, "cpu", seed=123)
        for i in range(B):
            for st in (st_g, st_c):
                st.reset_slot(i, 0.8, 0.9 if i % 2 else 1.0, 50 if i % 3 == 0 else 0, 1.3, list(range(0, 400, 3)),
                              seed=i)
        slots = torch.arange(B, dtype=torch.int32)
        for _ in range(3):
            a = S.sample(logits.to(dev), st_g, slots.to(dev)).cpu()
            b = S.sample_ref(logits, st_c, slots)
            agree += int((a == b).sum())
    assert agree >= 3 * B - 2, agree


@pytest.mark.parametrize("M", [64, 96, 160, 192, 256])
def test_linear_splitk_down_proj(dev, M):
    """Deep-K decode GEMMs at decode batches dispatch to the split-K library
    path (2 or 8 K-slices, fp32 partials reduced in fp32); numerics vs the
    fp32 reference."""
    from githubrepostorag_amd.ops.linear import gemm_splitk, linear, use_splitk

    N, K = 3584, 18944
    assert use_splitk(M, N, K) and not use_splitk(128, N, K) and not use_splitk(M, 37888, 3584)
    assert not use_splitk(1024, N, K) and not use_splitk(M, 1024, 4096)  # prefill M, encoder FFN2
    x = rnd(M, K, dev=dev, scale=0.5)
    w = rnd(N, K, dev=dev, scale=0.05, seed=1)
    b = rnd(N, dev=dev, seed=2)
    ref = x.float().cpu() @ w.float().cpu().T
    close(linear(x, w), ref, 3e-2, 2e-2)
    close(gemm_splitk(x, w, b), ref + b.float().cpu(), 3e-2, 2e-2)
    close(gemm_splitk(x, w, None, 2), ref, 3e-2, 2e-2)


@pytest.mark.parametrize("M,Nn,K", [(1, 3584, 3584), (4, 3584, 18944), (16, 3584, 3584), (48, 3584, 3584),
                                   (128, 3584, 18944), (190, 3584, 3584), (190, 3584, 18944),
                                   (240, 3584, 3584), (384, 3584, 18944), (512, 3584, 3584)])
def test_splitk_deferred_rmsnorm(dev, M, Nn, K):
    """o_proj / down_proj at decode batches: the K-split planes left unreduced (EPI_PARTIAL) and reduced
    inside the residual-add + RMSNorm kernel; vs the fp32 reference of linear -> residual add -> RMSNorm
    and vs the unfused bf16 path (splitk_reduce + rmsnorm)."""
    from githubrepostorag_amd.ops import gemm as G
    from githubrepostorag_amd.ops.linear import linear, linear_deferred

    how = G.deferred_plan(M, Nn, K)
    assert how is not None and how[1] > 1, how
    x = rnd(M, K, dev=dev, scale=0.5)
    w = rnd(Nn, K, dev=dev, scale=0.05, seed=1)
    r = rnd(M, Nn, dev=dev, seed=2)
    g = rnd(Nn, dev=dev, seed=3)
    part = linear_deferred(x, w)
    assert isinstance(part, G.SplitKPartial) and part.S == how[1]
    r1 = r.clone()
    y = N.rmsnorm(part, g, 1e-6, residual=r1)
    h32 = x.float().cpu() @ w.float().cpu().T
    s32 = (h32 + r.float().cpu()).to(torch.bfloat16).float()
    y32 = s32 * torch.rsqrt(s32.pow(2).mean(-1, keepdim=True) + 1e-6) * g.float().cpu()
    close(r1, s32, 3e-2)
    close(y, y32, 5e-2)
    r2 = r.clone()  # the unfused path agrees to bf16 rounding of h
    y2 = N.rmsnorm(linear(x, w), g, 1e-6, residual=r2)
    close(r1, r2, 3e-2)
    close(y, y2, 5e-2)


@pytest.mark.parametrize("M,Nn,K", [(1, 3584, 3584), (4, 3584, 18944), (16, 3584, 3584), (3, 896, 4864)])
def test_splitk_rmsnorm_small_rows_graph(dev, M, Nn, K):
    """1-16 rows: the chunked split-K RMSNorm (ticket merge) against the one-block kernel's fp32 reference,
    eagerly and replayed twice in a hipGraph (the tickets reset themselves)."""
    from githubrepostorag_amd.ops import gemm as G
    from githubrepostorag_amd.ops.linear import linear_deferred

    x = rnd(M, K, dev=dev, scale=0.5)
    w = rnd(Nn, K, dev=dev, scale=0.05, seed=1)
    r = rnd(M, Nn, dev=dev, seed=2)
    g = rnd(Nn, dev=dev, seed=3)
    N.norm_ws(dev)
    h32 = x.float().cpu() @ w.float().cpu().T
    s32 = (h32 + r.float().cpu()).to(torch.bfloat16).float()
    y32 = s32 * torch.rsqrt(s32.pow(2).mean(-1, keepdim=True) + 1e-6) * g.float().cpu()
    part = linear_deferred(x, w)
    assert isinstance(part, G.SplitKPartial), G.deferred_plan(M, Nn, K)
    r1 = r.clone()
    y = N.rmsnorm(part, g, 1e-6, residual=r1)
    close(r1, s32, 3e-2)
    close(y, y32, 5e-2)
    r2 = r.clone()
    out = torch.empty(M, Nn, dtype=torch.bfloat16, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        N.rmsnorm(linear_deferred(x, w), g, 1e-6, residual=r2, out=out)
    for _ in range(2):
        r2.copy_(r)
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(r2, r1) and torch.equal(out, y)
    assert int(N.norm_ws(dev)[0].abs().sum()) == 0


def test_splitk_deferred_in_graph(dev):
    """The deferred projection + fused norm replay correctly inside a hipGraph (workspace sized eagerly)."""
    from githubrepostorag_amd.ops.linear import linear_deferred

    M, Nn, K = 190, 3584, 3584
    x = rnd(M, K, dev=dev, scale=0.5)
    w = rnd(Nn, K, dev=dev, scale=0.05, seed=1)
    r0 = rnd(M, Nn, dev=dev, seed=2)
    g = rnd(Nn, dev=dev, seed=3)
    r = r0.clone()
    eager = N.rmsnorm(linear_deferred(x, w), g, 1e-6, residual=r)
    r_g = r0.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph):
            out = N.rmsnorm(linear_deferred(x, w), g, 1e-6, residual=r_g)
    torch.cuda.current_stream().wait_stream(s)
    r_g.copy_(r0)
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, eager) and torch.equal(r_g, r)


class _ThreadGroup:
    """W simulated TP ranks as W threads of one process (one GPU): all_gather / all_reduce are host
    rendezvous over device tensors (each rank's stream synchronised first)."""

    def __init__(self, world, rank, shared):
        self.size, self.rank, self.trivial, self.sh = world, rank, False, shared

    def _exchange(self, t):
        import threading  # noqa: F401

        torch.cuda.current_stream().synchronize()
        self.sh["buf"][self.rank] = t.clone()
        self.sh["bar"].wait()
        allt = torch.stack([x.to(t.device) for x in self.sh["buf"]])
        self.sh["bar"].wait()
        return allt

    def all_gather(self, t):
        return self._exchange(t)

    def all_reduce(self, t):
        t.copy_(self._exchange(t).sum(0))
        return t


@pytest.mark.parametrize("world", [2, 4])
def test_sampler_vocab_parallel_matches_full(dev, world):
    """each simulated TP rank samples from its own vocab shard of the logits (max pairs,
    radix histograms and Gumbel winners exchanged); every rank gets the same token as the full-row
    sampler on the whole vocabulary (greedy rows exactly, sampled rows up to histogram rounding)."""
    import copy
    import threading

    V, B = 152064, 24
    g = torch.Generator().manual_seed(5)
    logits = (torch.randn(B, V, generator=g) * 3).to(dev).to(torch.bfloat16)
    base = S.SamplerState(B, V, dev, seed=77)
    for i in range(B):
        base.reset_slot(i, 0.0 if i % 6 == 0 else 0.7, 0.8 if i % 2 else 1.0, 40 if i % 3 == 0 else 0, 1.2,
                        list(range(i, 3000, 7)), seed=i)
    slots = torch.arange(B, dtype=torch.int32, device=dev)
    full_state = copy.deepcopy(base)
    ref = [S.sample(logits, full_state, slots).cpu() for _ in range(2)]
    shard = -(-V // world)
    shard = -(-shard // 8) * 8
    shared = {"buf": [None] * world, "bar": threading.Barrier(world)}
    outs, errs = [None] * world, []

    def rank_fn(r):
        try:
            st = copy.deepcopy(base)
            grp = _ThreadGroup(world, r, shared)
            loc = torch.zeros(B, shard, dtype=logits.dtype, device=dev)
            n = min(shard, V - r * shard)
            loc[:, :n] = logits[:, r * shard:r * shard + n]
            with torch.cuda.stream(torch.cuda.Stream()):
                outs[r] = [S.sample_tp(loc, st, slots, grp, r * shard).cpu() for _ in range(2)]
                torch.cuda.current_stream().synchronize()
        except Exception as e:  # pragma: no cover
            errs.append(e)
            shared["bar"].abort()

    th = [threading.Thread(target=rank_fn, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for r in range(1, world):
        assert all(torch.equal(outs[0][k], outs[r][k]) for k in range(2))  # every rank: the same tokens
    for k in range(2):
        greedy = torch.arange(B) % 6 == 0
        assert torch.equal(outs[0][k][greedy], ref[k][greedy])
        assert int((outs[0][k] == ref[k]).sum()) >= B - 1, (outs[0][k], ref[k])


def test_sampler_reset_slots_batched_matches_per_slot(dev):
    """The engine's batched admission reset (one upload + index_copy per field + one seen-bit scatter) leaves
    the same sampler state as one reset_slot per sequence."""
    from githubrepostorag_amd.ops.sampling import SamplerState, reset_slots

    V = 152064
    entries = [(3, 0.4, 0.8, 0, 1.2, list(range(100, 1124)), None), (7, 0.0, 1.0, 50, 1.0, [5, 6], 11),
               (0, 0.7, 0.9, 40, 1.1, [1, 2, 3, 152063], 5)]
    a, b = SamplerState(8, V, dev, seed=1), SamplerState(8, V, dev, seed=1)
    for s in (a, b):  # dirty state from a previous occupant
        s.seen.fill_(-1)
        s.temperature.fill_(9.0)
    reset_slots(a, entries)
    for e in entries:
        b.reset_slot(*e)
    for name in ("temperature", "top_p", "top_k", "penalty", "rng", "seen"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    assert a._uses_topk == b._uses_topk and a._uses_topp == b._uses_topp
