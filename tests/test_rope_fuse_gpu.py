"""Small-batch decode with the RoPE + K/V-store pass folded into the attention launch
(csrc/kernels/attention.hip paged_decode_mw_kernel FR, ops/attention.py paged_decode_mw_rope) against the
two-launch path on the same split-K planes (ops/elementwise.qkv_rope_kvstore, then paged_attention): the same
K / V land in the cache, the same output (fp32 softmax of the new key instead of the bf16 P of the MFMA path,
hence a tolerance), and hipGraph replays leave the split tickets reset.  Also the Qwen2 model wiring: a decode
step with the fused launch gives the unfused step's hidden state and K/V caches."""
import math

import pytest
import torch

from githubrepostorag_amd.ops import attention as A
from githubrepostorag_amd.ops import elementwise as E
from githubrepostorag_amd.ops.gemm import SplitKPartial

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _setup(dev, lens_ctx, Hq, Hkv, D, S, BS=16, seed=0):
    g = torch.Generator().manual_seed(seed)
    B = len(lens_ctx)
    nblk = [(c + BS - 1) // BS for c in lens_ctx]
    NB = sum(nblk) + 3
    perm = torch.randperm(NB, generator=g)
    bt = torch.zeros(B, max(nblk), dtype=torch.int32)
    o = 0
    for s in range(B):
        bt[s, :nblk[s]] = perm[o:o + nblk[s]]
        o += nblk[s]
    kc = torch.randn(NB, Hkv, BS, D, generator=g).to(torch.bfloat16)
    vc = torch.randn(NB, Hkv, BS, D, generator=g).to(torch.bfloat16)
    # the new token of row s sits at key ctx - 1: its cache slot from the row's block table
    slots = torch.tensor([int(bt[s, (c - 1) // BS]) * BS + (c - 1) % BS for s, c in enumerate(lens_ctx)],
                         dtype=torch.int32)
    N = (Hq + 2 * Hkv) * D
    planes = (torch.randn(S, B, N, generator=g) * (0.6 / math.sqrt(S))).float()
    bias = (torch.randn(N, generator=g) * 0.1).to(torch.bfloat16)
    pos = torch.tensor([c - 1 for c in lens_ctx], dtype=torch.int32)
    meta = A.AttnMetadata(q_start=torch.arange(B + 1, dtype=torch.int32).to(dev),
                          ctx_len=torch.tensor(lens_ctx, dtype=torch.int32).to(dev), block_tables=bt.to(dev),
                          slot_mapping=slots.to(dev), max_q_len=1, num_seqs=B, num_tokens=B, is_decode=True)
    part = SplitKPartial(planes.to(dev).reshape(-1), S, B, N, torch.bfloat16)
    return part, bias.to(dev), pos.to(dev), kc.to(dev), vc.to(dev), meta


@pytest.mark.parametrize("Hq,Hkv,D", [(28, 4, 128), (14, 2, 64)])
@pytest.mark.parametrize("sl", [0, 32, 128, 256])
def test_mw_rope_matches_two_launch_path(dev, Hq, Hkv, D, sl):
    lens_ctx = [1, 33, 300, 1200, 4100]  # a 1-key context (only the new key), a split ending on the new key
    B = len(lens_ctx)
    part, bias, pos, kc0, vc0, meta = _setup(dev, lens_ctx, Hq, Hkv, D, S=4, seed=7 + sl)
    cs = E.rope_cos_sin(8192, D, 1e6, dev)
    scale = 1 / math.sqrt(D)
    A.decode_counters(dev)
    if sl:
        ns = -(-max(lens_ctx) // sl)
        meta.num_splits, meta.split_len = ns, sl
        meta.part_o = torch.empty(ns * B * Hq * D, dtype=torch.float32, device=dev)
        meta.part_ml = torch.empty(ns * B * Hq * 2, dtype=torch.float32, device=dev)
    for code in (22, 24):
        meta.extra = {"decode_nw": code}
        kr, vr = kc0.clone(), vc0.clone()
        q = E.qkv_rope_kvstore(part, bias, pos, cs, meta.slot_mapping, kr, vr, Hq, Hkv, D)
        ref = A.paged_attention(q, kr, vr, meta, scale)
        kf, vf = kc0.clone(), vc0.clone()
        out = A.paged_decode_mw_rope(part, bias, pos, cs, kf, vf, meta, scale, Hq, Hkv, D)
        assert out is not None
        torch.cuda.synchronize()
        torch.testing.assert_close(out.float(), ref.float(), atol=2e-2, rtol=2e-2)
        assert torch.equal(vf, vr)
        torch.testing.assert_close(kf.float(), kr.float(), atol=1e-2, rtol=1e-2)
        # replays inside one hipGraph: the in-launch split merge's tickets reset themselves
        o2 = torch.empty_like(out)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(3):
                o2.copy_(A.paged_decode_mw_rope(part, bias, pos, cs, kf, vf, meta, scale, Hq, Hkv, D))
        for _ in range(2):
            o2.zero_()
            g.replay()
            torch.cuda.synchronize()
            torch.testing.assert_close(o2.float(), ref.float(), atol=2e-2, rtol=2e-2)
        assert int(A.decode_counters(dev)[: B * Hkv].abs().sum()) == 0


def test_mw_rope_declines_what_it_does_not_cover(dev):
    part, bias, pos, kc, vc, meta = _setup(dev, [40, 70], 28, 4, 128, S=2)
    cs = E.rope_cos_sin(256, 128, 1e6, dev)
    meta.extra = {"decode_nw": 1}  # a one-wave decode variant asked for: not this kernel
    assert A.paged_decode_mw_rope(part, bias, pos, cs, kc, vc, meta, 0.1, 28, 4, 128) is None
    meta.extra = {}
    assert A.paged_decode_mw_rope(part, bias, pos, None, kc, vc, meta, 0.1, 28, 4, 128) is None  # no rotary
    assert A.paged_decode_mw_rope(part, bias, pos, cs, kc, vc, meta, 0.1, 28, 4, 128) is not None


def test_qwen2_decode_step_with_fused_rope(dev, monkeypatch):
    """A Qwen2-7B-shaped decode step (3 rows, qkv deferred as split-K planes) through the fused launch gives the
    two-launch step's hidden state and K/V caches, and the fused launch ran in every layer."""
    import dataclasses

    import githubrepostorag_amd.models.qwen2 as Q
    from githubrepostorag_amd.models.configs import decoder_config

    cfg = dataclasses.replace(decoder_config("qwen2-7b"), num_layers=3)
    model = Q.Qwen2Model(cfg, device=dev, seed=0)
    B, bs = 3, 16
    lens = [5, 40, 300]
    i32 = dict(dtype=torch.int32, device=dev)
    bt = torch.arange(3 * 19, **i32).view(3, 19)
    slots = torch.tensor([int(bt[s, (c - 1) // bs]) * bs + (c - 1) % bs for s, c in enumerate(lens)], **i32)
    meta = A.AttnMetadata(q_start=torch.arange(B + 1, **i32), ctx_len=torch.tensor(lens, **i32), block_tables=bt,
                          slot_mapping=slots, max_q_len=1, num_seqs=B, num_tokens=B, is_decode=True)
    ids = torch.tensor([11, 12, 13], **i32)
    pos = torch.tensor([c - 1 for c in lens], **i32)
    base = model.allocate_kv_cache(3 * 19, bs)
    for kc, vc in base:
        kc.normal_(0, 0.5)
        vc.normal_(0, 0.5)
    calls = []
    real = Q.paged_decode_mw_rope
    monkeypatch.setattr(Q, "paged_decode_mw_rope", lambda *a, **k: (lambda r: calls.append(r is not None) or r)(real(*a, **k)))
    outs = {}
    with torch.no_grad():
        for fused in (True, False):
            monkeypatch.setattr(A, "ROPE_FUSE", fused)
            kv = [(k.clone(), v.clone()) for k, v in base]
            outs[fused] = (model.forward(ids, pos, meta, kv).float(), kv)
    assert calls[:cfg.num_layers] == [True] * cfg.num_layers, calls
    h1, h2 = outs[True][0], outs[False][0]
    assert (h1 - h2).abs().max().item() <= 0.03 * h2.abs().max().item()
    # layer 0 stores the same K / V; later layers' inputs carry the attention's bf16-level differences
    for li, ((k1, v1), (k0, v0)) in enumerate(zip(outs[True][1], outs[False][1])):
        tol = 3e-2 if li == 0 else 1e-1
        torch.testing.assert_close(k1.float(), k0.float(), atol=tol, rtol=3e-2)
        torch.testing.assert_close(v1.float(), v0.float(), atol=tol, rtol=3e-2)
