"""Owned 256x256 MFMA GEMM (csrc/kernels/gemm_tile.hip) against an fp32
PyTorch reference: plain / bias / GELU / SiLU*mul epilogues, ragged M and N
tails, split-K partial slabs + combine, and hipGraph replay."""
import pytest
import torch

from githubrepostorag_amd.ops import gemm as G

pytestmark = pytest.mark.gpu


def rnd(*shape, dev, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16).to(dev)


def ref(x, w, b=None):
    y = x.float().cpu() @ w.float().cpu().T
    return y if b is None else y + b.float().cpu()


def check(y, r, K):
    # bf16 output rounding + fp32 accumulation-order differences; |y| ~ sqrt(K) * scale^2
    y = y.float().cpu()
    tol = 2e-2 * r.abs().max().item() + 1e-2
    err = (y - r).abs().max().item()
    assert err <= tol, f"max err {err} > {tol}"


@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (512, 768, 256), (300, 520, 192), (1, 264, 128),
                                   (4096, 4608, 3584), (777, 3584, 640)])
def test_gemm_plain(dev, M, N, K):
    x, w = rnd(M, K, dev=dev, scale=0.5), rnd(N, K, dev=dev, seed=1, scale=0.5)
    y = G.gemm(x, w, ksplit=1)
    check(y, ref(x, w), K)


def test_gemm_bias_identity_asymmetric(dev):
    # A = I with an asymmetric B catches a transposed C write (cdna guide §3)
    K = 256
    x = torch.eye(K, dtype=torch.bfloat16, device=dev)
    w = (torch.arange(K * 264, dtype=torch.float32).reshape(264, K) % 251 - 125).to(torch.bfloat16).to(dev)
    b = rnd(264, dev=dev, seed=3)
    y = G.gemm(x, w, b, ksplit=1)
    assert torch.equal(y.cpu(), (w.float().T + b.float()).to(torch.bfloat16).cpu())


@pytest.mark.parametrize("act", [G.ACT_GELU, G.ACT_GELU_TANH])
def test_gemm_gelu(dev, act):
    M, N, K = 333, 1024, 384
    x, w, b = rnd(M, K, dev=dev, scale=0.3), rnd(N, K, dev=dev, seed=1, scale=0.3), rnd(N, dev=dev, seed=2)
    y = G.gemm(x, w, b, act=act, ksplit=1)
    r = ref(x, w, b)
    r = torch.nn.functional.gelu(r, approximate="tanh" if act == G.ACT_GELU_TANH else "none")
    check(y, r, K)


@pytest.mark.parametrize("M", [5, 192, 700])
def test_gemm_silu(dev, M):
    I, K = 512, 384
    x = rnd(M, K, dev=dev, scale=0.5)
    wg, wu = rnd(I, K, dev=dev, seed=1, scale=0.3), rnd(I, K, dev=dev, seed=2, scale=0.3)
    bg, bu = rnd(I, dev=dev, seed=3), rnd(I, dev=dev, seed=4)
    wgu = G.interleave_gate_up(wg, wu)
    bgu = G.interleave_gate_up(bg.view(I, 1), bu.view(I, 1)).view(2 * I)
    h = G.gemm_silu(x, wgu, bgu, ksplit=1)
    r = torch.nn.functional.silu(ref(x, wg, bg)) * ref(x, wu, bu)
    check(h, r, K)


@pytest.mark.parametrize("M,N,K,S", [(192, 3584, 18944, 8), (64, 4608, 3584, 7), (200, 1024, 1024, 4)])
def test_gemm_splitk(dev, M, N, K, S):
    x, w, b = rnd(M, K, dev=dev, scale=0.2), rnd(N, K, dev=dev, seed=1, scale=0.2), rnd(N, dev=dev, seed=2)
    y = G.gemm(x, w, b, ksplit=S)
    check(y, ref(x, w, b), K)


def test_gemm_silu_splitk(dev):
    M, I, K = 160, 1024, 2048
    x = rnd(M, K, dev=dev, scale=0.3)
    wg, wu = rnd(I, K, dev=dev, seed=1, scale=0.2), rnd(I, K, dev=dev, seed=2, scale=0.2)
    h = G.gemm_silu(x, G.interleave_gate_up(wg, wu), ksplit=6)
    check(h, torch.nn.functional.silu(ref(x, wg)) * ref(x, wu), K)


def test_plan_ksplit():
    assert G.plan_ksplit(8192, 4608, 3584) == 1
    s = G.plan_ksplit(192, 3584, 18944)
    assert 14 * s <= 256 + 14 and s >= 8


def test_gemm_graph_replay(dev):
    M, N, K = 192, 2048, 1024
    x, w = rnd(M, K, dev=dev, scale=0.3), rnd(N, K, dev=dev, seed=1, scale=0.3)
    S = G.plan_ksplit(M, N, K)
    G.WS.reserve(dev, S * M * N)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    G.gemm(x, w, out=out)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        G.gemm(x, w, out=out)
    x.copy_(rnd(M, K, dev=dev, seed=7, scale=0.3))
    g.replay()
    torch.cuda.synchronize()
    check(out, ref(x, w), K)


@pytest.mark.parametrize("M,N,K,sk", [(512, 1536, 512, 16), (512, 1536, 512, 20), (2560, 1024, 384, 16),
                                      (4096, 4608, 1024, 256), (192, 37888, 1024, 256),
                                      # sk < 0: every full round of the CUs data-parallel, |sk| workgroups
                                      # stream the rest (fewer tiles than CUs: all of them are streamed)
                                      (512, 1536, 512, -20), (2560, 1024, 384, -16), (1280, 4608, 1024, -64),
                                      (4352, 4096, 512, -40), (4352, 4096, 512, -16),
                                      # K-aligned tail splits with more stream-K workgroups than CUs: 392 tiles
                                      # = 256 + 136, every leftover tile in 3 K parts (408 workgroups); 90 tiles
                                      # in 3 parts (270)
                                      (7040, 3584, 2048, -408), (1280, 4608, 1024, -270)])
def test_gemm_stream_k(dev, M, N, K, sk):
    x, w, b = rnd(M, K, dev=dev, scale=0.3), rnd(N, K, dev=dev, seed=1, scale=0.3), rnd(N, dev=dev, seed=2)
    y = G.gemm(x, w, b, ksplit=1, sk=sk)
    check(y, ref(x, w, b), K)
    y2 = G.gemm(x, w, b, ksplit=1, sk=sk)
    assert torch.equal(y, y2), "stream-K fixup must be bitwise reproducible"


@pytest.mark.parametrize("M,I,sk", [(192, 4096, 48), (768, 2048, -20), (768, 2048, -192)])
def test_gemm_silu_stream_k(dev, M, I, sk):
    K = 1024  # (192, 48): 32 tiles over 48 stream-K workgroups, every tile split; (768, -20): 8-tile remainder
    x = rnd(M, K, dev=dev, scale=0.3)
    wg, wu = rnd(I, K, dev=dev, seed=1, scale=0.2), rnd(I, K, dev=dev, seed=2, scale=0.2)
    h = G.gemm_silu(x, G.interleave_gate_up(wg, wu), ksplit=1, sk=sk)
    check(h, torch.nn.functional.silu(ref(x, wg)) * ref(x, wu), K)


def test_plan_stream_k():
    if G._num_cus() != 256:
        pytest.skip("plan thresholds are stated for 256 CUs")
    assert G.plan(192, 37888, 3584) == (1, 0)     # 148 tiles: whole tiles (all-stream-K measured slower)
    assert G.plan(16384, 4608, 3584) == (1, 256)  # 1152 tiles = 4.5 rounds
    assert G.plan(16384, 37888, 3584) == (1, 0)   # 9472 tiles = 37 full rounds


# ---------------------------------------------------------------- decode kernel (csrc/kernels/gemm_decode.hip)
@pytest.mark.parametrize("M,N,K,plan", [(1, 256, 256, (4, 4, 2, 1)), (37, 512, 1024, (4, 4, 2, 2)),
                                        (128, 1024, 512, (8, 4, 2, 1)), (192, 4608, 3584, (12, 8, 2, 14)),
                                        (64, 3584, 3584, (4, 4, 2, 7)), (256, 1536, 1024, (16, 4, 2, 2)),
                                        (100, 512, 256, (8, 4, 2, 1)), (120, 1024, 1024, (8, 4, 2, 3)),
                                        (96, 3584, 18944, (8, 4, 2, 9))])
def test_gemm_decode_plain(dev, M, N, K, plan):
    x, w, b = rnd(M, K, dev=dev, scale=0.3), rnd(N, K, dev=dev, seed=1, scale=0.3), rnd(N, dev=dev, seed=2)
    G.WS.reserve(dev, G.dec_ws_floats(M, N, G.dec_ksplit(K, plan[3])))
    y = G.gemm_decode(x, w, b, plan=plan)
    check(y, ref(x, w, b), K)


# balanced grids: (mt, nwv, ntw, ksplit, gs) with 1..nwv wave units per workgroup (idle waves store nothing)
@pytest.mark.parametrize("M,N,K,plan", [(192, 4608, 3584, (12, 5, 2, 7, 36)), (200, 3584, 18944, (8, 5, 2, 9, 28)),
                                        (100, 1024, 512, (8, 5, 2, 1, 7)), (129, 1536, 1024, (12, 5, 2, 2, 13)),
                                        (256, 2048, 1024, (8, 5, 2, 1, 64)), (150, 1056, 512, (12, 5, 2, 1, 8)),
                                        (250, 1024, 512, (4, 5, 2, 2, 8)), (77, 1024, 512, (8, 4, 2, 1))])
def test_gemm_decode_balanced(dev, M, N, K, plan):
    x, w, b = rnd(M, K, dev=dev, scale=0.3), rnd(N, K, dev=dev, seed=1, scale=0.3), rnd(N, dev=dev, seed=2)
    G.WS.reserve(dev, G.dec_ws_floats(M, N, G.dec_ksplit(K, plan[3])))
    y = G.gemm_decode(x, w, b, plan=plan)
    check(y, ref(x, w, b), K)


@pytest.mark.parametrize("M,plan", [(192, (12, 5, 2, 1, 14)), (250, (8, 5, 2, 1, 16)), (100, (8, 5, 2, 1, 33)),
                                    (230, (16, 4, 2, 1, 17)), (200, (12, 8, 2, 2, 9))])
def test_gemm_decode_silu_balanced(dev, M, plan):
    I, K = 1056, 1024  # 66 wave units: 4-5, 4-5, 2 per workgroup
    x = rnd(M, K, dev=dev, scale=0.5)
    wg, wu = rnd(I, K, dev=dev, seed=1, scale=0.2), rnd(I, K, dev=dev, seed=2, scale=0.2)
    wgu = G.interleave_gate_up(wg, wu)
    h = G.gemm_decode(x, wgu, None, epi=G.EPI_SILU, plan=plan)
    check(h, torch.nn.functional.silu(ref(x, wg)) * ref(x, wu), K)


# unit-packed weights (ops/gemm.py dec_pack): same results as the natural layout
@pytest.mark.parametrize("M,N,K,plan,silu", [(192, 4608, 3584, (12, 5, 2, 7, 36), False),
                                             (64, 3584, 18944, (4, 4, 2, 9), False),
                                             (250, 2048, 1024, (8, 5, 2, 1, 64), False),
                                             (192, 2112, 1024, (12, 5, 2, 1, 14), True),
                                             (100, 2048, 512, (8, 4, 2, 2), True)])
def test_gemm_decode_packed(dev, M, N, K, plan, silu):
    x, w = rnd(M, K, dev=dev, scale=0.3), rnd(N, K, dev=dev, seed=1, scale=0.3)
    b = rnd(N, dev=dev, seed=2)
    G.WS.reserve(dev, G.dec_ws_floats(M, N, G.dec_ksplit(K, plan[3])))
    epi = G.EPI_SILU if silu else G.EPI_STORE
    y0 = G.gemm_decode(x, w, b, epi=epi, plan=plan)
    y1 = G.gemm_decode(x, w, b, epi=epi, plan=plan, packed=G.DecPacked(w, silu))
    if silu:
        wg, wu = G.deinterleave_gate_up(w.float())
        bg, bu = G.deinterleave_gate_up(b.float().view(N, 1))
        r = torch.nn.functional.silu(ref(x, wg.bfloat16(), bg.view(-1).bfloat16())) * ref(x, wu.bfloat16(), bu.view(-1).bfloat16())
    else:
        r = ref(x, w, b)
    check(y0, r, K)
    check(y1, r, K)
    assert torch.equal(y0.cpu(), y1.cpu())


# tail split (8 waves: 4 own units + a 5th unit split by row tiles over waves 4-7): 4- and 5-unit workgroups
# in one grid, every mt, plain / split-K / SiLU / packed, ragged M
@pytest.mark.parametrize("M,N,K,plan", [(176, 4608, 3584, (12, 8, 2, 7, 32, 1)), (64, 3584, 3584, (4, 8, 2, 7, 25, 1)),
                                        (250, 3584, 18944, (16, 8, 2, 8, 25, 1)), (120, 2080, 512, (8, 8, 2, 1, 14, 1)),
                                        (33, 1024, 256, (4, 8, 2, 1, 7, 1))])
def test_gemm_decode_tail_split(dev, M, N, K, plan):
    x, w, b = rnd(M, K, dev=dev, scale=0.3), rnd(N, K, dev=dev, seed=1, scale=0.3), rnd(N, dev=dev, seed=2)
    G.WS.reserve(dev, G.dec_ws_floats(M, N, G.dec_ksplit(K, plan[3])))
    y = G.gemm_decode(x, w, b, plan=plan)
    check(y, ref(x, w, b), K)
    y1 = G.gemm_decode(x, w, b, plan=plan, packed=G.DecPacked(w))
    assert torch.equal(y.cpu(), y1.cpu())


@pytest.mark.parametrize("M", [40, 128, 176, 256])
def test_gemm_decode_silu_tail_split(dev, M):
    I, K = 2336, 512  # 146 wave units over 32 workgroups: 4 and 5 per workgroup
    x = rnd(M, K, dev=dev, scale=0.5)
    wg, wu = rnd(I, K, dev=dev, seed=1, scale=0.2), rnd(I, K, dev=dev, seed=2, scale=0.2)
    bg, bu = rnd(I, dev=dev, seed=3), rnd(I, dev=dev, seed=4)
    wgu = G.interleave_gate_up(wg, wu)
    bgu = G.interleave_gate_up(bg.view(I, 1), bu.view(I, 1)).view(2 * I)
    plan = G.dec_tail_plan(M, 2 * I, ncu=32)
    assert plan is not None and plan[4] == 32 and plan[5] == 1
    h = G.gemm_decode(x, wgu, bgu, epi=G.EPI_SILU, plan=plan)
    check(h, torch.nn.functional.silu(ref(x, wg, bg)) * ref(x, wu, bu), K)
    h1 = G.gemm_decode(x, wgu, bgu, epi=G.EPI_SILU, plan=plan, packed=G.DecPacked(wgu, True))
    assert torch.equal(h.cpu(), h1.cpu())


def test_gemm_decode_identity_asymmetric(dev):
    # A = I with an asymmetric W catches a transposed C write
    K = 256
    w = (torch.arange(K * 256, dtype=torch.float32).reshape(256, K) % 251 - 125).to(torch.bfloat16).to(dev)
    for M, plan in ((200, (16, 4, 2, 1)), (190, (12, 8, 2, 1)), (190, (12, 5, 2, 1, 4)), (120, (8, 5, 2, 1, 3)),
                    (250, (4, 5, 2, 1, 2)), (190, (12, 8, 2, 1, 2, 1)), (250, (16, 8, 2, 1, 2, 1))):
        x = torch.eye(K, dtype=torch.bfloat16, device=dev)[:M].contiguous()
        y = G.gemm_decode(x, w, plan=plan)
        assert torch.equal(y.cpu(), w.float().T[:M].to(torch.bfloat16).cpu())


@pytest.mark.parametrize("act", [G.ACT_GELU, G.ACT_GELU_TANH])
def test_gemm_decode_gelu(dev, act):
    M, N, K = 77, 1024, 512
    x, w, b = rnd(M, K, dev=dev, scale=0.3), rnd(N, K, dev=dev, seed=1, scale=0.3), rnd(N, dev=dev, seed=2)
    for ks in (1, 2):
        G.WS.reserve(dev, G.dec_ws_floats(M, N, ks))
        y = G.gemm_decode(x, w, b, act=act, plan=(8, 4, 2, ks))
        r = torch.nn.functional.gelu(ref(x, w, b), approximate="tanh" if act == G.ACT_GELU_TANH else "none")
        check(y, r, K)


@pytest.mark.parametrize("M,plan", [(5, (4, 4, 2, 1)), (192, (12, 8, 2, 1)), (250, (16, 4, 2, 1)),
                                    (160, (12, 8, 2, 2)), (100, (8, 4, 2, 1))])
def test_gemm_decode_silu(dev, M, plan):
    I, K = 1024, 1024
    x = rnd(M, K, dev=dev, scale=0.5)
    wg, wu = rnd(I, K, dev=dev, seed=1, scale=0.2), rnd(I, K, dev=dev, seed=2, scale=0.2)
    bg, bu = rnd(I, dev=dev, seed=3), rnd(I, dev=dev, seed=4)
    wgu = G.interleave_gate_up(wg, wu)
    bgu = G.interleave_gate_up(bg.view(I, 1), bu.view(I, 1)).view(2 * I)
    G.WS.reserve(dev, G.dec_ws_floats(M, 2 * I, plan[3]))
    h = G.gemm_decode(x, wgu, bgu, epi=G.EPI_SILU, plan=plan)
    check(h, torch.nn.functional.silu(ref(x, wg, bg)) * ref(x, wu, bu), K)


def test_gemm_decode_graph_replay(dev):
    M, N, K = 96, 3584, 3584
    x, w = rnd(M, K, dev=dev, scale=0.3), rnd(N, K, dev=dev, seed=1, scale=0.3)
    plan = G.dec_plan(M, N, K)
    G.WS.reserve(dev, G.dec_ws_floats(M, N, plan[3]))
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    G.gemm_decode(x, w, out=out)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        G.gemm_decode(x, w, out=out)
    x.copy_(rnd(M, K, dev=dev, seed=7, scale=0.3))
    g.replay()
    torch.cuda.synchronize()
    check(out, ref(x, w), K)


@pytest.mark.parametrize("M,N,K", [(7104, 3584, 18944), (6016, 3584, 18944), (7296, 4608, 3584), (5000, 3584, 3584),
                                   (3000, 1024, 4096)])
def test_linear_prefill_dispatch(dev, M, N, K):
    """linear() at prefill-sized M routes by the measured table (owned kernel where it won) — same numbers
    as the fp32 reference whichever arm is taken; the Qwen2-7B down_proj at 7104 rows must be owned."""
    from githubrepostorag_amd.ops.linear import linear

    x, w = rnd(M, K, dev=dev, scale=0.5), rnd(N, K, dev=dev, seed=1, scale=0.05)
    b = rnd(N, dev=dev, seed=2)
    p = G.prefill_plan(M, N, K)
    if (M, N, K) == (7104, 3584, 18944):
        assert p is not None
    y = linear(x, w, b)
    rows = torch.arange(0, M, 37)
    check(y[rows], ref(x[rows], w, b), K)


@pytest.mark.parametrize("M", [320, 448, 512])
@pytest.mark.parametrize("N,K,silu", [(4608, 3584, False), (3584, 3584, False), (3584, 18944, False),
                                      (37888, 3584, True), (152064, 3584, False)])
def test_decode_batch_257_512_rows(dev, M, N, K, silu):
    """Decode batches of 257-512 live sequences: every Qwen2-7B projection
    and the vocab-wide LM head (N = 152064) through the production dispatch (linear() / mlp_gate_up(),
    whichever kernel and schedule it picks at this M: K-split tile plans, tail stream-K, the owned LM-head
    schedule) against the fp32 reference, on sampled rows."""
    from githubrepostorag_amd.ops.linear import linear

    x, w = rnd(M, K, dev=dev, scale=0.5, seed=M), rnd(N, K, dev=dev, seed=N % 97, scale=0.05)
    rows = torch.arange(0, M, 29)
    if silu:
        y = G.mlp_gate_up(x, w)
        r = ref(x[rows], w)
        v = r.view(len(rows), -1, 2, 32)
        r = (torch.nn.functional.silu(v[:, :, 0]) * v[:, :, 1]).reshape(len(rows), -1)
    else:
        y = linear(x, w)
        r = ref(x[rows], w)
    assert y.shape == (M, N // 2 if silu else N)
    check(y[rows], r, K)


@pytest.fixture()
def mfma32():
    prev = G.set_mfma(32)
    yield
    G.set_mfma(prev)


def test_gemm_mfma32_variant(dev, mfma32):
    """The v_mfma_f32_32x32x16_bf16 build of the tile kernel (same 64x32 quadrants per wave, its own
    fragment reads, chunk map, permlane32 wide stores): plain / bias / GELU / SiLU*mul epilogues, ragged
    tails, split-K planes and stream-K fixups against fp32, and the identity check for a transposed write."""
    K = 256
    x = torch.eye(K, dtype=torch.bfloat16, device=dev)
    w = (torch.arange(K * 264, dtype=torch.float32).reshape(264, K) % 251 - 125).to(torch.bfloat16).to(dev)
    b = rnd(264, dev=dev, seed=3)
    assert torch.equal(G.gemm(x, w, b, ksplit=1).cpu(), (w.float().T + b.float()).to(torch.bfloat16).cpu())
    for M, N, K in [(300, 520, 192), (1, 264, 128), (777, 3584, 640)]:
        x, w = rnd(M, K, dev=dev, scale=0.5), rnd(N, K, dev=dev, seed=1, scale=0.5)
        check(G.gemm(x, w, ksplit=1), ref(x, w), K)
    M, N, K = 333, 1024, 384
    x, w, b = rnd(M, K, dev=dev, scale=0.3), rnd(N, K, dev=dev, seed=1, scale=0.3), rnd(N, dev=dev, seed=2)
    check(G.gemm(x, w, b, act=G.ACT_GELU, ksplit=1), torch.nn.functional.gelu(ref(x, w, b)), K)
    for M, I, K, ks, sk in [(700, 512, 384, 1, None), (160, 1024, 2048, 6, None), (768, 2048, 1024, 1, -20)]:
        x = rnd(M, K, dev=dev, scale=0.3)
        wg, wu = rnd(I, K, dev=dev, seed=1, scale=0.2), rnd(I, K, dev=dev, seed=2, scale=0.2)
        bg, bu = rnd(I, dev=dev, seed=3), rnd(I, dev=dev, seed=4)
        bgu = G.interleave_gate_up(bg.view(I, 1), bu.view(I, 1)).view(2 * I)
        h = G.gemm_silu(x, G.interleave_gate_up(wg, wu), bgu, ksplit=ks, sk=sk)
        check(h, torch.nn.functional.silu(ref(x, wg, bg)) * ref(x, wu, bu), K)
    for M, N, K, S in [(192, 3584, 18944, 8), (200, 1024, 1024, 4)]:
        x, w, b = rnd(M, K, dev=dev, scale=0.2), rnd(N, K, dev=dev, seed=1, scale=0.2), rnd(N, dev=dev, seed=2)
        check(G.gemm(x, w, b, ksplit=S), ref(x, w, b), K)
    for M, N, K, sk in [(512, 1536, 512, 20), (7040, 3584, 2048, -408), (1280, 4608, 1024, -270)]:
        x, w, b = rnd(M, K, dev=dev, scale=0.3), rnd(N, K, dev=dev, seed=1, scale=0.3), rnd(N, dev=dev, seed=2)
        y = G.gemm(x, w, b, ksplit=1, sk=sk)
        check(y, ref(x, w, b), K)
        assert torch.equal(y, G.gemm(x, w, b, ksplit=1, sk=sk))


@pytest.mark.parametrize("depth", [6, 8])
@pytest.mark.parametrize("M,N,K,plan,silu", [(64, 3584, 3584, (4, 4, 2, 7), False), (128, 4608, 3584, (8, 4, 2, 7), False),
                                             (60, 2112, 1024, (4, 5, 2, 1, 14), True),
                                             (100, 2112, 1024, (8, 5, 2, 1, 14), True)])
def test_gemm_decode_deep_ring(dev, depth, M, N, K, plan, silu):
    """Deeper K-step rings (grag_gemm_decode_depth: 6 for mt 4 / 8, 8 for mt 4) give the default ring's
    results bit for bit (same accumulation order)."""
    from githubrepostorag_amd.ops._lib import lib

    if depth == 8 and plan[0] != 4:
        pytest.skip("depth 8: mt 4 only")
    x, w, b = rnd(M, K, dev=dev, scale=0.3), rnd(N, K, dev=dev, seed=1, scale=0.3), rnd(N, dev=dev, seed=2)
    epi = G.EPI_SILU if silu else G.EPI_STORE
    G.WS.reserve(dev, G.dec_ws_floats(M, N, G.dec_ksplit(K, plan[3])))
    y0 = G.gemm_decode(x, w, b, epi=epi, plan=plan)
    prev = lib().grag_gemm_decode_depth(depth)
    try:
        y1 = G.gemm_decode(x, w, b, epi=epi, plan=plan)
    finally:
        lib().grag_gemm_decode_depth(prev)
    assert torch.equal(y0.cpu(), y1.cpu())
    if not silu:
        check(y1, ref(x, w, b), K)


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [0, 8, 12])
@pytest.mark.parametrize("M,N,K,silu", [(1, 4608, 3584, False), (4, 3584, 18944, False), (16, 3584, 3584, False),
                                        (23, 4608, 1024, False), (32, 2112, 1024, True), (3, 2112, 1024, True)])
def test_gemm_decode_small_rows(dev, depth, M, N, K, silu):
    """The 1- / 2-row-tile decode variants (1-32 rows, the reference's 1-4 live sequences) at the default ring
    and the deep ones (8, 12): the dispatch plan's results against the fp32 reference, and every depth bit for
    bit the default's."""
    from githubrepostorag_amd.ops._lib import lib

    plan = G.dec_plan(M, N, K, silu)
    assert plan is not None and plan[0] == -(-M // 16), plan
    x, w, b = rnd(M, K, dev=dev, scale=0.3), rnd(N, K, dev=dev, seed=1, scale=0.3), rnd(N, dev=dev, seed=2)
    epi = G.EPI_SILU if silu else G.EPI_STORE
    G.WS.reserve(dev, G.dec_ws_floats(M, N, G.dec_ksplit(K, plan[3])))
    y0 = G.gemm_decode(x, w, b, epi=epi, plan=plan)
    prev = lib().grag_gemm_decode_depth(depth)
    try:
        y1 = G.gemm_decode(x, w, b, epi=epi, plan=plan)
    finally:
        lib().grag_gemm_decode_depth(prev)
    torch.cuda.synchronize()
    assert torch.equal(y0.cpu(), y1.cpu())
    if silu:
        r = ref(x, w, b).view(M, -1, 2, 32)
        want = torch.nn.functional.silu(r[:, :, 0]) * r[:, :, 1]
        check(y1, want.reshape(M, -1), K)
    else:
        check(y1, ref(x, w, b), K)


# ---------------------------------------------------------------- balanced phase schedule (gemm_tile.hip SCHED 1)
@pytest.fixture(params=[1, 2])
def sched1(request):
    prev = G.set_sched(request.param)
    yield
    G.set_sched(prev)


@pytest.mark.parametrize("M,N,K,ks,sk", [(256, 256, 128, 1, 0), (300, 520, 192, 1, 0), (777, 3584, 640, 1, 0),
                                         (4096, 4608, 3584, 1, 0), (200, 1024, 1024, 4, 0), (192, 3584, 18944, 8, 0),
                                         (512, 1536, 512, 1, 20), (2560, 1024, 384, 1, 16),
                                         (7040, 3584, 2048, 1, -408), (1280, 4608, 1024, 1, -270)])
@pytest.mark.parametrize("sched", [1, 2])
def test_gemm_balanced_schedule(dev, M, N, K, ks, sk, sched):
    # every K-tile count parity, 2- and 3-tile segments, split-K planes and stream-K shares; each accumulator
    # sees the same K order under every schedule (1: balanced 4-phase, 2: two-phase, 32 MFMAs per barrier
    # interval), so the results are bitwise equal to schedule 0's
    x, w, b = rnd(M, K, dev=dev, scale=0.3), rnd(N, K, dev=dev, seed=1, scale=0.3), rnd(N, dev=dev, seed=2)
    prev = G.set_sched(0)
    try:
        y0 = G.gemm(x, w, b, ksplit=ks, sk=sk)
        G.set_sched(sched)
        y1 = G.gemm(x, w, b, ksplit=ks, sk=sk)
    finally:
        G.set_sched(prev)
    check(y1, ref(x, w, b), K)
    assert torch.equal(y0, y1)


@pytest.mark.parametrize("M,I,K,sk", [(700, 512, 384, 0), (768, 2048, 1024, -20), (192, 4096, 1024, 48)])
def test_gemm_silu_balanced_schedule(dev, sched1, M, I, K, sk):
    x = rnd(M, K, dev=dev, scale=0.5)
    wg, wu = rnd(I, K, dev=dev, seed=1, scale=0.3), rnd(I, K, dev=dev, seed=2, scale=0.3)
    h = G.gemm_silu(x, G.interleave_gate_up(wg, wu), ksplit=1, sk=sk)
    check(h, torch.nn.functional.silu(ref(x, wg)) * ref(x, wu), K)


def test_gemm_balanced_identity_gelu(dev, sched1):
    K = 256
    x = torch.eye(K, dtype=torch.bfloat16, device=dev)
    w = (torch.arange(K * 264, dtype=torch.float32).reshape(264, K) % 251 - 125).to(torch.bfloat16).to(dev)
    b = rnd(264, dev=dev, seed=3)
    assert torch.equal(G.gemm(x, w, b, ksplit=1).cpu(), (w.float().T + b.float()).to(torch.bfloat16).cpu())
    M, N, K = 333, 1024, 384
    x, w, b = rnd(M, K, dev=dev, scale=0.3), rnd(N, K, dev=dev, seed=1, scale=0.3), rnd(N, dev=dev, seed=2)
    r = torch.nn.functional.gelu(ref(x, w, b))
    check(G.gemm(x, w, b, act=G.ACT_GELU, ksplit=1), r, K)
