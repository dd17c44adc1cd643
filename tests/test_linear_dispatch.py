"""Decode-GEMM dispatch rules of ops/linear.py (CPU: predicates only; the
numerics of every path are in tests/test_kernels_gpu.py)."""
import torch

from githubrepostorag_amd.ops.linear import splitk_parts, use_splitk
from githubrepostorag_amd.ops import gemm as G


def test_splitk_only_for_decode_sized_deep_k_down_proj():
    assert use_splitk(192, 3584, 18944) and use_splitk(256, 3584, 18944)  # Qwen2-7B down_proj
    assert use_splitk(160, 2048, 11008 // 512 * 512)
    assert not use_splitk(128, 3584, 18944)  # the tuned library wins at M <= 128
    assert not use_splitk(1024, 3584, 18944)  # prefill-sized M
    assert not use_splitk(192, 1024, 4096)  # bge-large FFN2
    assert not use_splitk(192, 768, 3072)  # GPT-2 MLP
    assert not use_splitk(192, 37888, 3584)  # gate_up (wide N)
    assert not use_splitk(192, 1536, 8960)  # K not a multiple of 8 x 64


def test_splitk_parts_by_batch():
    assert [splitk_parts(M, 3584, 18944) for M in (16, 48, 64, 96, 128, 192, 256, 512)] == [0, 2, 2, 2, 0, 8, 8, 0]


def test_two_slice_splitk_only_for_measured_shape():
    # 2-slice branch was timed only on Qwen2-7B down_proj (N=3584, K=18944)
    assert splitk_parts(64, 1536, 8960) == 0  # Qwen2-1.5B down_proj
    assert splitk_parts(64, 2048, 11008) == 0  # Qwen2.5-3B down_proj
    assert splitk_parts(64, 3584, 18944) == 2


def test_decode_gemm_plan_rules():
    from githubrepostorag_amd.ops import gemm as G

    assert G.dec_plan(96, 4608, 1000) is None             # K % 256
    assert G.dec_ksplit(3584, 9) == 7                     # 14 rounds of 4 steps -> 2 rounds per split
    assert G.dec_variants(100) == [(8, 4, 2), (8, 5, 2)]
    assert G.dec_variants(190) == [(12, 5, 2), (12, 8, 2)]
    G_ncu = G._num_cus
    try:
        G._num_cus = lambda: 256
        assert G.dec_plan(64, 4608, 3584) == (4, 4, 2, 7)   # 36 tiles x 7 splits
        assert G.dec_plan(128, 3584, 18944) == (8, 4, 2, 9)  # 28 tiles x 9 splits
        assert G.dec_plan(128, 37888, 3584, silu=True) == (8, 5, 2, 1, 256)  # 1184 units: 4-5 per CU
        assert G.dec_plan(192, 4608, 3584) == (12, 5, 2, 7, 36)  # 144 units: 4 per group x 7 splits
        assert G.dec_plan(192, 37888, 3584, silu=True) == (12, 5, 2, 1, 256)
        assert G.dec_plan(192, 3584, 18944) is None          # deep-K down_proj: tile kernel split-K
        assert G.dec_plan(256, 3584, 3584) == (16, 4, 2, 7)
        assert G.dec_plan(256, 37888, 3584, silu=True) is None  # gate/up at 193..256: tile kernel
        assert G.dec_plan(300, 4608, 3584) is None
    finally:
        G._num_cus = G_ncu


def test_dec_pack_layout():
    N, K = 128, 256
    w = torch.arange(N * K, dtype=torch.float32).reshape(N, K)
    pk = G.dec_pack(w)
    assert pk.shape == (4, 4, 32, 64)
    assert torch.equal(pk[1, 2, 5], w[32 + 5, 128:192])
    pks = G.dec_pack(w, silu=True)
    # silu unit 3: block 1, second 16-wide group -> gate rows 80..95, up rows 112..127
    assert torch.equal(pks[3, 0, 0], w[80, :64]) and torch.equal(pks[3, 0, 16], w[112, :64])


def test_prefill_plan_from_measured_table():
    """Prefill GEMMs (M > 256) follow the dense M sweep (tuning/gemm_prefill_gfx950.json)."""
    ms, rows = G._prefill_table()[(3584, 18944, 0)]  # Qwen2-7B down_proj
    assert ms == sorted(ms) and ms[0] <= 512 and ms[-1] >= 16000
    # the bench's ~7.1K-row prefill steps: the library's heuristic is ~1.45x slower there
    assert G.prefill_plan(7104, 3584, 18944) is not None
    # the library is kept only where it won at both buckets around M
    for i in range(1, len(ms)):
        lo, hi = rows[i - 1], rows[i]
        p = G.prefill_plan(ms[i] - 1, 3584, 18944)
        lib_both = all(r[2] is None or r[2] >= r[1] for r in (lo, hi))
        assert (p is None) == lib_both
    # SwiGLU shapes are always owned; unmeasured plain shapes stay on the library
    assert G.prefill_plan(5000, 37888, 3584, silu=True) is not None
    assert G.prefill_plan(5000, 1000, 1024) is None
    assert G.prefill_plan(5000, 1000, 1024, silu=True) == G.plan(5000, 1000, 1024)
    # decode-sized M keeps the split-K planner
    assert G.schedule(192, 3584, 18944) == G.plan(192, 3584, 18944)


def test_prefill_plan_schedules_pass_launcher_rule():
    G_ncu = G._num_cus
    try:
        G._num_cus = lambda: 256
        for (N, K, silu), (ms, _) in G._prefill_table().items():
            for M in range(300, 16500, 97):
                p = G.prefill_plan(M, N, K, bool(silu))
                if p is not None:
                    assert G.sk_ok(M, N, K, *p), (M, N, K, p)
    finally:
        G._num_cus = G_ncu


def test_sk_ok_mirrors_launcher():
    # 28 x 14 = 392 tiles on 256 CUs, K = 18944 (296 K-steps): tail-only needs 136 * 296 >= 256 * 74
    assert G.sk_ok(7104, 3584, 18944, 1, -256)
    assert G.sk_ok(7104, 3584, 18944, 1, 0)
    # 17 x 14 = 238 tiles < one round: the stream-K round gets all of them, 238 * 56 >= 256 * 28
    assert G.sk_ok(4352, 3584, 3584, 1, 256)
    # 257 tiles, tail of 1 tile over 256 workgroups: far below a quarter tile each
    assert not G.sk_ok(257 * 256, 256, 3584, 1, -256)


def test_deferred_splitk_plan():
    """o_proj / down_proj K-splits whose reduce folds into the residual-add + RMSNorm kernel: exactly the
    owned-kernel K-split cases of linear(); prefill sizes, the fused gate/up and un-split shapes are not."""
    assert G.deferred_plan(190, 3584, 3584)[:2] == ("decode", 7)
    assert G.deferred_plan(128, 3584, 18944)[:2] == ("decode", 9)
    assert G.deferred_plan(190, 3584, 18944)[0] == "tile"
    assert G.deferred_plan(384, 3584, 18944)[0] == "tile"  # 257-512-row decode: measured K-split plans
    assert G.deferred_plan(4096, 3584, 3584) is None
    assert G.deferred_plan(190, 37888, 3584) is None


def test_config4_per_rank_projections_are_measured_and_owned_unless_the_library_won():
    """BASELINE config 4 (Qwen2-72B TP=8): every per-rank projection has measured dispatch rows -- the
    prefill table (scripts/sweep_prefill_gemm.py --models qwen2-72b-tp8, 512-row buckets) and the decode
    table (scripts/gemm_dispatch_table.py --models qwen2-72b:8) -- so none falls to the library by default
    (round 3: K = 3696 failed every owned kernel's K % 64; the FFN shard is now zero-padded to 3712,
    models/qwen2.py FFN_PAD).  kernel_for() picks an owned kernel wherever the sweep did not measure the
    library clearly faster; gate/up (fused SwiGLU) is owned at every M.  The measured library wins are
    narrow-N / odd-K buckets (profiles/sweep_prefill_tp_r4.jsonl); owned overall >= 75 % of the buckets."""
    from githubrepostorag_amd.models.configs import decoder_config
    from githubrepostorag_amd.models.qwen2 import FFN_PAD
    from githubrepostorag_amd.ops import linear as L

    c = decoder_config("qwen2-72b")
    tp = 8
    hq, hkv, D, H = c.num_heads // tp, c.num_kv_heads // tp, c.head_dim, c.hidden_size
    inter = -(-(c.intermediate_size // tp) // FFN_PAD) * FFN_PAD
    assert inter == 3712 and inter % 64 == 0
    plain = {"qkv": ((hq + 2 * hkv) * D, H), "o": (H, hq * D), "down": (H, inter)}
    ncu = G._num_cus
    try:
        G._num_cus = lambda: 256
        L.enable_tuned_gemms()
        table = G._prefill_table()
        owned = total = 0
        for name, (N, K) in plain.items():
            assert (N, K, 0) in table, name  # measured prefill rows
            assert L._TUNED["table"].get((N, K)) is not None, name  # measured decode rows
            ms, rows = table[(N, K, 0)]
            for M in [1, 4, 16, 32, 64, 96, 128, 192, 256] + list(range(512, 16385, 512)):
                kind = L.kernel_for(M, N, K)
                total += 1
                if kind in L.OWNED_KINDS:
                    owned += 1
                    continue
                # the library only where a measurement put it ahead
                if M <= 128:
                    assert L.measured_choice(M, N, K) == "library", (name, M, kind)
                else:
                    assert G.prefill_plan(M, N, K) is None and M >= G.PREFILL_MIN_M or \
                        L.measured_choice(M, N, K) == "library", (name, M, kind)
        assert owned >= 0.75 * total, (owned, total)
        # gate/up: the fused SwiGLU kernel at every prefill M
        assert all(G.prefill_plan(M, 2 * inter, H, silu=True) is not None for M in range(384, 16385, 512))
    finally:
        G._num_cus = ncu


def test_workspace_owned_by_engine_not_thread(monkeypatch):
    """ops/gemm.py WS.owned_by: inside the block a thread's split-K workspace requests go to the owner's dict
    (an engine's, kept for its lifetime: its captured decode graphs point at it), outside to the thread's
    own; another thread never sees the owner's buffer."""
    import threading

    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: False)
    dev = torch.device("cpu")
    own = {}
    with G.WS.owned_by(own):
        b = G.WS.get(dev, 10)
        assert G.WS.ready(dev, 10) and G.WS.get(dev, 5) is b
    assert own["bufs"][None] is b
    assert G.WS.get(dev, 10) is not b  # the thread's own buffer outside the block
    seen = []

    def other():
        seen.append(G.WS.get(dev, 10) is b)
        with G.WS.owned_by(own):
            seen.append(G.WS.get(dev, 10) is b)

    t = threading.Thread(target=other)
    t.start()
    t.join()
    assert seen == [False, True]


def test_deferred_decode_launch_gets_the_split_count_its_planes_were_sized_for(monkeypatch):
    """gemm_deferred sizes the fp32 planes with dec_ksplit of the plan's K-split request and must launch the
    kernel with that same count: a request the 4-step rounding lowers (K = 3584: 28 -> 14) once wrote 28 planes
    into a 14-plane slab (a GPU fault in scripts/sweep_dec_mid.py)."""
    seen = {}

    def fake_call(name, *args):
        seen["ks"] = args[15]  # (..., mt, nwv, ntw, ksplit, gs, ...) of grag_gemm_decode_t

    monkeypatch.setattr(G, "call", fake_call)
    monkeypatch.setattr(G.WS, "get", lambda dev, fl: torch.empty(fl))
    x, w = torch.zeros(176, 3584, dtype=torch.bfloat16), torch.zeros(4608, 3584, dtype=torch.bfloat16)
    for req in (7, 14, 28):
        part = G.gemm_deferred(x, w, ("decode", G.dec_ksplit(3584, req), (12, 5, 2, req)))
        assert seen["ks"] == part.S == G.dec_ksplit(3584, req)
    assert G.dec_ksplit(3584, 28) == 14
