"""AWQ W4A16 checkpoint support (ops/quant.py, csrc/kernels/quant.hip).

Parity note: no AutoAWQ checkpoint or the autoawq package is available
offline, so the packing convention (nibble i of a word = column 8c +
(0,2,4,6,1,3,5,7)[i]) is pinned by a hand-written packer in this file that
follows AutoAWQ's documented layout, not by a real checkpoint file ("parity
unpinned" against a downloaded model).
"""
import pytest
import torch

from githubrepostorag_amd.ops import quant


def _quantize(w: torch.Tensor, G: int, seed: int = 0):
    """w [N, K] fp32 -> AWQ (qweight [K, N/8], qzeros [K/G, N/8], scales fp16
    [K/G, N]) with asymmetric 4-bit groups along K."""
    N, K = w.shape
    wt = w.t().reshape(K // G, G, N)
    lo, hi = wt.amin(1), wt.amax(1)
    scale = ((hi - lo) / 15).clamp_min(1e-5).half().float()
    zero = (-lo / scale).round().clamp(0, 15)
    q = (wt / scale[:, None] + zero[:, None]).round().clamp(0, 15).reshape(K, N)
    return (quant.pack_awq(q.to(torch.int32)), quant.pack_awq(zero.to(torch.int32)), scale.half())


def _manual_dequant(qweight, qzeros, scales):
    K, NP = qweight.shape
    N, G = NP * 8, K // scales.shape[0]
    order = quant.AWQ_ORDER
    W = torch.empty(N, K)
    for k in range(K):
        for c in range(NP):
            word, zword = int(qweight[k, c]) & 0xFFFFFFFF, int(qzeros[k // G, c]) & 0xFFFFFFFF
            for i in range(8):
                n = 8 * c + order[i]
                W[n, k] = (((word >> 4 * i) & 0xF) - ((zword >> 4 * i) & 0xF)) * float(scales[k // G, n])
    return W


def test_pack_unpack_roundtrip():
    g = torch.Generator().manual_seed(1)
    q = torch.randint(0, 16, (12, 64), generator=g, dtype=torch.int32)
    assert torch.equal(quant.unpack_awq(quant.pack_awq(q)), q)


def test_reference_dequant_matches_bit_loop():
    g = torch.Generator().manual_seed(2)
    w = torch.randn(16, 32, generator=g)
    qw, qz, sc = _quantize(w, G=8)
    ref = quant.awq_dequant_reference(qw, qz, sc)
    assert torch.allclose(ref, _manual_dequant(qw, qz, sc))
    # 4-bit asymmetric groups: error within half a step of each group's scale
    step = sc.float().repeat_interleave(8, 0).t()
    assert ((ref - w).abs() <= 0.5 * step + 1e-4).all()


def test_state_dict_dequant_and_loader(tmp_path):
    from githubrepostorag_amd.models.weights import load_state_dict, save_state_dict

    g = torch.Generator().manual_seed(3)
    w = torch.randn(64, 128, generator=g)
    qw, qz, sc = _quantize(w, G=32)
    sd = {"model.layers.0.mlp.down_proj.qweight": qw, "model.layers.0.mlp.down_proj.qzeros": qz,
          "model.layers.0.mlp.down_proj.scales": sc, "model.norm.weight": torch.ones(64, dtype=torch.float16)}
    save_state_dict(sd, tmp_path / "model.safetensors")
    out = load_state_dict(tmp_path)
    assert set(out) == {"model.layers.0.mlp.down_proj.weight", "model.norm.weight"}
    W = out["model.layers.0.mlp.down_proj.weight"]
    assert W.shape == (64, 128) and W.dtype == torch.bfloat16
    assert torch.allclose(W.float(), quant.awq_dequant_reference(qw, qz, sc), atol=1e-2, rtol=1e-2)


def test_awq_qwen2_generates_like_dequantised_fp32():
    """A Qwen2 built from an AWQ checkpoint equals one built from the same
    weights dequantised in fp32 (same greedy tokens)."""
    from githubrepostorag_amd.models.configs import decoder_config
    from githubrepostorag_amd.models.qwen2 import Qwen2Model
    from tests.test_parallel_cpu import _generate, _hf_state_dict

    cfg = decoder_config("qwen2-tiny")
    sd = _hf_state_dict(cfg, seed=4)
    awq, deq = {}, {}
    for k, v in sd.items():
        if k.endswith("proj.weight"):
            qw, qz, sc = _quantize(v.float(), G=64)
            p = k[:-len(".weight")]
            awq.update({p + ".qweight": qw, p + ".qzeros": qz, p + ".scales": sc})
            deq[k] = quant.awq_dequant_reference(qw, qz, sc)
        else:
            awq[k] = deq[k] = v
    loaded = quant.dequantize_awq_state_dict(awq, dtype=torch.float32)
    assert set(loaded) == set(sd)
    prompts = [[5, 17, 99, 3, 250], [1, 2, 3, 4, 5, 6, 7, 8]]
    a = _generate(Qwen2Model(cfg, device="cpu", dtype=torch.float32, state_dict=loaded), prompts)
    b = _generate(Qwen2Model(cfg, device="cpu", dtype=torch.float32, state_dict=deq), prompts)
    assert a == b


@pytest.mark.gpu
@pytest.mark.parametrize("K,N,G", [(512, 4608, 128), (3584, 512, 128), (256, 128, 64), (128, 192, 32)])
def test_awq_dequant_kernel_matches_fp32_reference(K, N, G):
    from githubrepostorag_amd.ops._lib import lib

    lib()  # the HIP path must be the one under test
    g = torch.Generator().manual_seed(K + N)
    qw = quant.pack_awq(torch.randint(0, 16, (K, N), generator=g, dtype=torch.int32))
    qz = quant.pack_awq(torch.randint(0, 16, (K // G, N), generator=g, dtype=torch.int32))
    sc = (torch.rand(K // G, N, generator=g) * 0.02 + 1e-3).half()
    ref = quant.awq_dequant_reference(qw, qz, sc)
    out = quant.awq_dequant(qw.cuda(), qz.cuda(), sc.cuda())
    torch.cuda.synchronize()
    assert out.shape == (N, K) and out.dtype == torch.bfloat16
    torch.testing.assert_close(out.float().cpu(), ref, atol=1e-6, rtol=8e-3)

