"""Concurrency of the kernels that keep cross-workgroup state, and the device index guard.

Round 5 left an intermittent illegal-address fault at the start of the bench's serving loop, where the
retrieval thread (encoder graph replays + eager encoder GEMMs + search) and the engine's runner thread first
run GPU work side by side.  The suspects were scratch buffers more than one thread's launches could reach at
once: the process-wide stream-K slab / ticket array of ``grag_gemm_stream`` (ops/linear.py, taken by every
ownerless thread), the small-batch decode attention's and split-K RMSNorm's process-wide tickets, and encoder
graphs captured on one thread with that thread's workspace and replayed from another beside eager batches.
A ticket word two launches share can be left non-zero, after which a later launch's first arriver "merges"
partials nobody wrote.  Every such buffer is now owned (an engine, an embedder, or the calling thread), and
the encoder runs on the embedder's own stream.  These tests run the ticketed kernels from two threads on two
streams at once and check every result; and they check that an out-of-range index input is reported
(ops/_lib.py DeviceIndexError) instead of faulting the device.
"""
import math
import threading

import pytest
import torch

from githubrepostorag_amd.ops import _lib
from githubrepostorag_amd.ops import attention as A
from githubrepostorag_amd.ops import gemm as G
from githubrepostorag_amd.ops import linear as L
from githubrepostorag_amd.ops import norm as N

pytestmark = pytest.mark.gpu


def rnd(*shape, dev, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16).to(dev)


def _close(a, b, atol=3e-2, rtol=3e-2):
    return torch.allclose(a.float(), b.float(), atol=atol, rtol=rtol)


def _decode_case(dev, seed):
    """A 4-sequence decode batch whose contexts span 1..9 splits of 128 keys (small-batch kernel, merged in
    launch by tickets)."""
    Hq, Hkv, D, BS = 28, 4, 128, 16
    lens = [1, 130, 700, 1100]
    g = torch.Generator(device="cpu").manual_seed(seed)
    nblk = [-(-n // BS) for n in lens]
    NB = sum(nblk) + 4
    perm = torch.randperm(NB, generator=g)[: sum(nblk)].to(torch.int32)
    bt = torch.zeros(len(lens), max(nblk), dtype=torch.int32)
    o = 0
    for s, n in enumerate(nblk):
        bt[s, :n] = perm[o:o + n]
        o += n
    kc = torch.randn(NB, Hkv, BS, D, generator=g).to(torch.bfloat16)
    vc = torch.randn(NB, Hkv, BS, D, generator=g).to(torch.bfloat16)
    q = torch.randn(len(lens), Hq, D, generator=g).to(torch.bfloat16)
    meta = A.AttnMetadata(q_start=torch.arange(len(lens) + 1, dtype=torch.int32),
                          ctx_len=torch.tensor(lens, dtype=torch.int32), block_tables=bt,
                          slot_mapping=torch.zeros(len(lens), dtype=torch.int32), max_q_len=1,
                          num_seqs=len(lens), num_tokens=len(lens), is_decode=True)
    scale = 1 / math.sqrt(D)
    ref = A.paged_attention_ref(q, kc, vc, meta, scale).reshape(len(lens), -1)
    ns, sl = -(-max(lens) // 128), 128
    m = A.AttnMetadata(q_start=meta.q_start.to(dev), ctx_len=meta.ctx_len.to(dev), block_tables=bt.to(dev),
                       slot_mapping=meta.slot_mapping.to(dev), max_q_len=1, num_seqs=len(lens), num_tokens=len(lens),
                       is_decode=True, num_splits=ns, split_len=sl,
                       part_o=torch.empty(ns * len(lens) * Hq * D, dtype=torch.float32, device=dev),
                       part_ml=torch.empty(ns * len(lens) * Hq * 2, dtype=torch.float32, device=dev),
                       extra={"decode_nw": 24})
    return (q.to(dev), kc.to(dev), vc.to(dev), m, scale), ref


def test_two_owners_ticketed_kernels_concurrently(dev):
    """Two threads on two streams, each with its own workspace owner (as two engines, or an engine and the
    embedder), run stream-K GEMMs (grag_gemm_stream), a stream-K-round tile GEMM (grag_gemm_tile, sk grid)
    and the small-batch decode attention (in-launch split merge) 60 times each, interleaved on the device;
    every output must match its fp32 reference, no ticket word may be left set, and the index guard must
    stay silent.  A third thread does the same with NO owner (thread-local scratch)."""
    _lib.lib()
    _lib.bind_error_guard(dev.index or 0)
    _lib.check_device_errors()
    xs = rnd(24, 4096, dev=dev, scale=0.5, seed=1)
    ws = rnd(1024, 4096, dev=dev, scale=0.05, seed=2)
    ref_s = (xs.float().cpu() @ ws.float().cpu().T)
    xt = rnd(1536, 4096, dev=dev, scale=0.5, seed=3)
    wt = rnd(4096, 4096, dev=dev, scale=0.05, seed=4)
    ref_t = (xt.float().cpu() @ wt.float().cpu().T)
    assert G.sk_ok(1536, 4096, 4096, 1, 64)
    att_args, ref_a = _decode_case(dev, seed=5)
    errors: list = []
    barrier = threading.Barrier(3)

    def worker(owned: bool, it: int):
        try:
            torch.cuda.set_device(dev)
            s = torch.cuda.Stream(dev)
            owner: dict = {}
            ctx = G.WS.owned_by(owner) if owned else _nullctx()
            with torch.cuda.stream(s), ctx:
                A.decode_counters(dev)
                barrier.wait()
                for _ in range(it):
                    ys = L.gemm_stream(xs, ws)
                    yt = G.gemm(xt, wt, ksplit=1, sk=64)
                    ya = A.paged_attention(*att_args)
                    s.synchronize()
                    if not _close(ys.cpu(), ref_s):
                        raise AssertionError("gemm_stream result wrong under concurrency")
                    if not _close(yt.cpu(), ref_t, atol=0.15):
                        raise AssertionError("stream-K tile GEMM result wrong under concurrency")
                    if not _close(ya.cpu(), ref_a):
                        raise AssertionError("small-batch decode attention wrong under concurrency")
                cnt = A.decode_counters(dev)
                assert int(cnt[:16].abs().sum()) == 0, "decode ticket words left set"
        except BaseException as e:  # surfaced by the main thread
            errors.append(e)

    th = [threading.Thread(target=worker, args=(o, 60)) for o in (True, True, False)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "worker hung"
    if errors:
        raise errors[0]
    _lib.check_device_errors("concurrency test")


class _nullctx:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


def test_embedder_graph_replays_beside_eager_batches(dev):
    """The round-5 fault's setting: one thread replays the encoder's query-bucket graphs (bge-large: its
    FFN2 at query sizes is a stream-K GEMM) while another embeds documents eagerly through the SAME
    embedder and a third runs ownerless stream-K GEMMs on its own stream.  Every embedding must equal the
    single-threaded result and the index guard must stay silent."""
    from githubrepostorag_amd.embed.service import Embedder

    emb = Embedder.from_name("bge-large-en-v1.5", device=dev, seed=3)
    queries = [[f"how does module {i} handle retries and {j} timeouts?" for i in range(n)] for j, n in
               enumerate((1, 3, 5, 8))]
    docs = [f"def handler_{i}(x):\n    return x * {i}  # file {i % 7} of the service" * (1 + i % 5) for i in range(96)]
    ref_q = [emb.embed_queries(q).float().cpu() for q in queries]  # captures the buckets
    ref_d = emb.embed_documents(docs).float().cpu()
    torch.cuda.synchronize()
    xs = rnd(24, 4096, dev=dev, scale=0.5, seed=11)
    ws = rnd(1024, 4096, dev=dev, scale=0.05, seed=12)
    ref_s = xs.float().cpu() @ ws.float().cpu().T
    errors: list = []
    barrier = threading.Barrier(3)

    def queries_thread():
        try:
            torch.cuda.set_device(dev)
            s = torch.cuda.Stream(dev)
            with torch.cuda.stream(s):
                barrier.wait()
                for it in range(40):
                    k = it % len(queries)
                    v = emb.embed_queries(queries[k])
                    s.synchronize()
                    if not torch.allclose(v.float().cpu(), ref_q[k], atol=2e-2):
                        raise AssertionError(f"query bucket {k} embedding changed under concurrency")
        except BaseException as e:
            errors.append(e)

    def docs_thread():
        try:
            torch.cuda.set_device(dev)
            s = torch.cuda.Stream(dev)
            with torch.cuda.stream(s):
                barrier.wait()
                for _ in range(6):
                    v = emb.embed_documents(docs)
                    s.synchronize()
                    if not torch.allclose(v.float().cpu(), ref_d, atol=2e-2):
                        raise AssertionError("document embeddings changed under concurrency")
        except BaseException as e:
            errors.append(e)

    def gemm_thread():
        try:
            torch.cuda.set_device(dev)
            s = torch.cuda.Stream(dev)
            with torch.cuda.stream(s):
                barrier.wait()
                for _ in range(80):
                    y = L.gemm_stream(xs, ws)
                    s.synchronize()
                    if not _close(y.cpu(), ref_s):
                        raise AssertionError("ownerless stream-K GEMM wrong beside the encoder")
        except BaseException as e:
            errors.append(e)

    th = [threading.Thread(target=f) for f in (queries_thread, docs_thread, gemm_thread)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "worker hung"
    if errors:
        raise errors[0]
    assert emb.graphs.stats["replays"] >= 40
    _lib.check_device_errors("embedder concurrency test")


def test_index_guard_reports_instead_of_faulting(dev):
    """Out-of-range index inputs are skipped and reported: a token id far past the vocabulary in the
    embedding gather, a KV slot past the cache in the RoPE / KV store, a block-table entry past the cache
    in prefill and decode attention.  The rows with valid indices are still right; check_device_errors
    names the kernel, then the block is clear."""
    _lib.lib()
    assert _lib.bind_error_guard(dev.index or 0)
    _lib.check_device_errors()
    table = rnd(1000, 256, dev=dev, seed=21)
    ids = torch.tensor([1, 2, 1 << 30, 3], dtype=torch.int32, device=dev)
    out = N.embed_gather(ids, table)
    torch.cuda.synchronize()
    with pytest.raises(_lib.DeviceIndexError, match="embed_gather"):
        _lib.check_device_errors()
    assert torch.equal(out[[0, 1, 3]].cpu(), table[[1, 2, 3]].cpu())
    _lib.check_device_errors()  # cleared

    (q, kc, vc, m, scale), ref = _decode_case(dev, seed=22)
    bt = m.block_tables.clone()
    bt[2, 3] = 1 << 28  # sequence 2's 4th block
    m.block_tables = bt
    A.paged_attention(q, kc, vc, m, scale)
    torch.cuda.synchronize()
    with pytest.raises(_lib.DeviceIndexError, match="decode attention"):
        _lib.check_device_errors()
    m.extra = {"decode_nw": 3}  # the single-wave split kernel
    A.paged_attention(q, kc, vc, m, scale)
    torch.cuda.synchronize()
    with pytest.raises(_lib.DeviceIndexError, match="decode attention"):
        _lib.check_device_errors()

    from githubrepostorag_amd.ops import elementwise as E

    Hq, Hkv, D = 4, 2, 64
    T, NB, BS = 3, 8, 16
    qkv = rnd(T, (Hq + 2 * Hkv) * D, dev=dev, seed=23)
    kcache = torch.zeros(NB, Hkv, BS, D, dtype=torch.bfloat16, device=dev)
    vcache = torch.zeros_like(kcache)
    pos = torch.arange(T, dtype=torch.int32, device=dev)
    inv = 1.0 / (10000 ** (torch.arange(0, D, 2, dtype=torch.float32) / D))
    ang = torch.arange(64, dtype=torch.float32)[:, None] * inv[None, :]
    cs = torch.cat([ang.cos(), ang.sin()], 1).to(dev).contiguous()
    slots = torch.tensor([0, NB * BS + 5, 2], dtype=torch.int32, device=dev)
    E.qkv_rope_kvstore(qkv, None, pos, cs, slots, kcache, vcache, Hq, Hkv, D)
    torch.cuda.synchronize()
    with pytest.raises(_lib.DeviceIndexError, match="KV slot"):
        _lib.check_device_errors()
    _lib.check_device_errors()
