"""The decoder layer's post-attention RMSNorm folded into the gate/up projection at 1-4 rows
(csrc/kernels/gemm_decode.hip NRM kernel, ops/gemm.py gemm_decode_norm) against the unfused launches
(split-K RMSNorm, then the gate/up GEMM) and a plain PyTorch fp32 reference, on cuda:0."""
import pytest
import torch

from githubrepostorag_amd.ops import gemm as G
from githubrepostorag_amd.ops.linear import linear_deferred
from githubrepostorag_amd.ops.norm import rmsnorm

pytestmark = pytest.mark.gpu


def rnd(*shape, dev, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16).to(dev)


@pytest.mark.parametrize("M", [1, 2, 3, 4])
@pytest.mark.parametrize("H,I", [(3584, 18944), (1536, 8960)])
def test_gate_up_with_folded_post_attention_norm(dev, M, H, I, monkeypatch):
    monkeypatch.setattr(G, "NORM_FUSE", True)  # off by default (measured slower); the kernel stays tested
    x = rnd(M, H, dev=dev, scale=0.5)
    wo = rnd(H, H, dev=dev, scale=0.03, seed=1)
    wg, wu = rnd(I, H, dev=dev, scale=0.03, seed=2), rnd(I, H, dev=dev, scale=0.03, seed=3)
    w_gu = G.interleave_gate_up(wg, wu)
    gamma = rnd(H, dev=dev, seed=4)
    res = rnd(M, H, dev=dev, seed=5)
    eps = 1e-6
    part = linear_deferred(x, wo)
    assert isinstance(part, G.SplitKPartial), "o_proj at 1-4 rows leaves its split-K planes to the consumer"
    plan = G.norm_fuse_plan(M, w_gu.shape[0], H, True)
    assert plan is not None
    r_in = res.clone()
    r_out = torch.full_like(res, float("nan"))
    y = G.gemm_decode_norm(part, r_in, r_out, gamma, eps, w_gu, G.EPI_SILU, plan)
    torch.cuda.synchronize()
    assert torch.equal(r_in, res), "the input residual is read only"
    # the unfused launches on the same planes
    part2 = linear_deferred(x, wo)
    r2 = res.clone()
    xn = rmsnorm(part2, gamma, eps, residual=r2)
    y2 = G.mlp_gate_up(xn, w_gu)
    torch.cuda.synchronize()
    assert torch.equal(r_out, r2), "new residual: the same bf16 sum as the split-K RMSNorm"
    err_unfused = (y.float() - y2.float()).abs().max().item()
    # fp32 reference of the whole block
    h = (res.float() + x.float() @ wo.float().T).to(torch.bfloat16).float()
    n = (h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + eps) * gamma.float()).to(torch.bfloat16).float()
    ref = torch.nn.functional.silu(n @ wg.float().T) * (n @ wu.float().T)
    scale = ref.abs().max().item()
    assert err_unfused <= 0.02 * scale, (err_unfused, scale)
    assert (y.float() - ref).abs().max().item() <= 0.03 * scale


def test_decoder_forward_uses_the_fold_and_matches_unfused(dev, monkeypatch):
    """Qwen2 decode forward at 2 rows with the fold (GRAG_NORM_FUSE on) and without: the same hidden state up to
    bf16 noise, and the fused launches really ran."""
    from githubrepostorag_amd.models.configs import decoder_config
    from githubrepostorag_amd.models.qwen2 import Qwen2Model
    from githubrepostorag_amd.ops.attention import AttnMetadata

    model = Qwen2Model(decoder_config("qwen2-small"), device=dev, seed=0)
    B, ctx, bs = 2, 40, 16
    kv = model.allocate_kv_cache(16, bs)
    for kc, vc in kv:
        kc.normal_(0, 0.5)
        vc.normal_(0, 0.5)
    i32 = dict(dtype=torch.int32, device=dev)
    meta = AttnMetadata(q_start=torch.arange(B + 1, **i32), ctx_len=torch.full((B,), ctx, **i32),
                        block_tables=torch.arange(6, **i32).view(2, 3), slot_mapping=torch.tensor([ctx - 1, 48 + ctx - 1], **i32),
                        max_q_len=1, num_seqs=B, num_tokens=B, is_decode=True)
    ids = torch.tensor([11, 12], **i32)
    pos = torch.full((B,), ctx - 1, **i32)
    monkeypatch.setattr(G, "NORM_FUSE", True)
    monkeypatch.setattr(G, "FOLD_NORM", False)  # the fold would take the post-attention norm first
    calls = []
    real = G.gemm_decode_norm
    monkeypatch.setattr("githubrepostorag_amd.models.qwen2.gemm_decode_norm",
                        lambda *a, **k: calls.append(1) or real(*a, **k))
    with torch.no_grad():
        h1 = model.forward(ids, pos, meta, kv).float()
        n_fused = len(calls)
        monkeypatch.setattr(G, "NORM_FUSE", False)
        h2 = model.forward(ids, pos, meta, kv).float()
    assert n_fused == model.cfg.num_layers and len(calls) == n_fused
    scale = h2.abs().max().item()
    assert (h1 - h2).abs().max().item() <= 0.02 * scale


@pytest.mark.parametrize("M", [1, 3, 4])
def test_folded_norm_producer_and_consumers(dev, M, monkeypatch):
    """The folded RMSNorm (ops/gemm.py gemm_decode_red / gemm_decode_scaled): the producer's last splits add
    the o_proj planes into the residual stream -- bitwise the split-K RMSNorm's residual -- and leave per-group
    sums of squares; the gate/up (SiLU) and qkv (split-K planes) consumers scale A by the norm weight and the
    accumulators by 1 / rms.  Against the unfused launches and an fp32 reference."""
    monkeypatch.setattr(G, "FOLD_NORM", True)
    H, I, NQ = 3584, 18944, 4608
    x = rnd(M, H, dev=dev, scale=0.5)
    wo = rnd(H, H, dev=dev, scale=0.03, seed=1)
    wg, wu = rnd(I, H, dev=dev, scale=0.03, seed=2), rnd(I, H, dev=dev, scale=0.03, seed=3)
    w_gu = G.interleave_gate_up(wg, wu)
    wq = rnd(NQ, H, dev=dev, scale=0.03, seed=6)
    gamma = rnd(H, dev=dev, seed=4)
    res = rnd(M, H, dev=dev, seed=5)
    eps = 1e-6
    G.fold_ws(dev)
    r1 = res.clone()
    fold = G.gemm_decode_red(x, wo, r1, 0)
    assert fold is not None and fold.residual is r1
    y = G.gemm_decode_scaled(fold, gamma, eps, w_gu, G.EPI_SILU)
    qp = G.gemm_decode_scaled(fold, gamma, eps, wq, G.EPI_PARTIAL)
    assert y is not None and isinstance(qp, G.SplitKPartial)
    q = qp.materialize().float()
    torch.cuda.synchronize()
    # unfused
    r2 = res.clone()
    xn = rmsnorm(linear_deferred(x, wo), gamma, eps, residual=r2)
    y2 = G.mlp_gate_up(xn, w_gu)
    q2 = (xn.float() @ wq.float().T)
    torch.cuda.synchronize()
    assert torch.equal(r1, r2), "residual stream: the same bf16 sums as the split-K RMSNorm"
    sy, sq = y2.float().abs().max().item(), q2.abs().max().item()
    assert (y.float() - y2.float()).abs().max().item() <= 0.02 * sy
    assert (q - q2).abs().max().item() <= 0.02 * sq
    # fp32 reference
    h = (res.float() + x.float() @ wo.float().T).to(torch.bfloat16).float()
    n = h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + eps) * gamma.float()
    ref = torch.nn.functional.silu(n @ wg.float().T) * (n @ wu.float().T)
    assert (y.float() - ref).abs().max().item() <= 0.03 * ref.abs().max().item()
    assert (q - n @ wq.float().T).abs().max().item() <= 0.03 * sq


def test_decoder_forward_with_folded_norms_matches_unfused(dev, monkeypatch):
    """Qwen2 decode forward at 3 rows: every layer's norms folded (o_proj / down producers, gate/up / qkv
    consumers) against the unfused launches; the same hidden state up to bf16 noise, and the folded kernels ran
    (num_layers - 1 down_proj folds, num_layers o_proj folds)."""
    import githubrepostorag_amd.models.qwen2 as Q
    from githubrepostorag_amd.models.configs import decoder_config
    from githubrepostorag_amd.ops.attention import AttnMetadata

    import dataclasses

    cfg = dataclasses.replace(decoder_config("qwen2-7b"), num_layers=3)
    model = Q.Qwen2Model(cfg, device=dev, seed=0)
    B, ctx, bs = 3, 40, 16
    kv = model.allocate_kv_cache(12, bs)
    for kc, vc in kv:
        kc.normal_(0, 0.5)
        vc.normal_(0, 0.5)
    i32 = dict(dtype=torch.int32, device=dev)
    meta = AttnMetadata(q_start=torch.arange(B + 1, **i32), ctx_len=torch.full((B,), ctx, **i32),
                        block_tables=torch.arange(9, **i32).view(3, 3),
                        slot_mapping=torch.tensor([ctx - 1, 48 + ctx - 1, 96 + ctx - 1], **i32),
                        max_q_len=1, num_seqs=B, num_tokens=B, is_decode=True)
    ids = torch.tensor([11, 12, 13], **i32)
    pos = torch.full((B,), ctx - 1, **i32)
    calls = []
    real = G.gemm_decode_red
    monkeypatch.setattr(Q, "gemm_decode_red", lambda *a, **k: (lambda r: calls.append(r is not None) or r)(real(*a, **k)))
    monkeypatch.setattr(G, "FOLD_NORM", True)
    with torch.no_grad():
        h1 = model.forward(ids, pos, meta, kv).float()
        n_folds = sum(calls)
        monkeypatch.setattr(G, "FOLD_NORM", False)
        h2 = model.forward(ids, pos, meta, kv).float()
    assert n_folds == 2 * cfg.num_layers - 1, calls
    assert (h1 - h2).abs().max().item() <= 0.03 * h2.abs().max().item()
