"""AWQ (W4A16, AutoAWQ "GEMM" packing) checkpoint dequantisation.

The reference serves ``Qwen/Qwen2.5-Coder-7B-Instruct-AWQ`` through vLLM's
AWQ GEMM (reference ``helm/values.yaml:67``).  Here the
4-bit weights are expanded once at load time into bf16 ``[out, in]`` (the
layout every engine GEMM consumes) by ``grag_awq_dequant``
(``csrc/kernels/quant.hip``) on the GPU; CPU tensors use the fp32 reference
below.  Packing (AutoAWQ): ``qweight`` int32 ``[in, out/8]``, nibble ``i`` of
word ``c`` holds output column ``8c + AWQ_ORDER[i]``; ``qzeros`` int32
``[in/G, out/8]`` packed the same way; ``scales`` fp16 ``[in/G, out]``.
"""
from __future__ import annotations

import torch

from ._lib import call, ptr

AWQ_ORDER = (0, 2, 4, 6, 1, 3, 5, 7)
_TILE = 64


def unpack_awq(packed: torch.Tensor) -> torch.Tensor:
    """int32 ``[R, C]`` -> int ``[R, 8C]`` 4-bit values in column order."""
    shifts = torch.arange(0, 32, 4, dtype=torch.int32, device=packed.device)
    nib = (packed.to(torch.int32).unsqueeze(-1) >> shifts) & 0xF  # [R, C, 8], nibble order
    cols = torch.empty_like(nib)
    cols[..., list(AWQ_ORDER)] = nib  # nibble i -> column AWQ_ORDER[i]
    return cols.reshape(packed.shape[0], -1)


def pack_awq(q: torch.Tensor) -> torch.Tensor:
    """Inverse of :func:`unpack_awq` (tests / offline quantisation)."""
    R, N = q.shape
    cols = q.to(torch.int64).reshape(R, N // 8, 8)
    out = torch.zeros(R, N // 8, dtype=torch.int64, device=q.device)
    for i, c in enumerate(AWQ_ORDER):
        out |= (cols[..., c] & 0xF) << (4 * i)
    out = torch.where(out >= 2 ** 31, out - 2 ** 32, out)
    return out.to(torch.int32)


def awq_dequant_reference(qweight, qzeros, scales) -> torch.Tensor:
    """fp32 reference: ``W[n, k] = (q[k, n] - z[k//G, n]) * s[k//G, n]``."""
    K = qweight.shape[0]
    G = K // scales.shape[0]
    q = unpack_awq(qweight).float()
    z = unpack_awq(qzeros).float().repeat_interleave(G, 0)
    s = scales.float().repeat_interleave(G, 0)
    return ((q - z) * s).t().contiguous()


def awq_dequant(qweight: torch.Tensor, qzeros: torch.Tensor, scales: torch.Tensor,
                dtype: torch.dtype = torch.bfloat16) -> torch.Tensor:
    """Dequantise one AWQ linear to ``[out, in]`` ``dtype``."""
    K, NP = qweight.shape
    N = NP * 8
    if qzeros.shape[1] != NP or scales.shape[1] != N or K % scales.shape[0] or qzeros.shape[0] != scales.shape[0]:
        raise ValueError(f"inconsistent AWQ shapes: qweight {tuple(qweight.shape)}, qzeros "
                         f"{tuple(qzeros.shape)}, scales {tuple(scales.shape)}")
    G = K // scales.shape[0]
    if not qweight.is_cuda:
        return awq_dequant_reference(qweight, qzeros, scales).to(dtype)
    if K % _TILE or N % _TILE or dtype != torch.bfloat16:
        raise ValueError(f"grag_awq_dequant needs bf16 output and in/out multiples of {_TILE}: K={K} N={N}")
    qweight = qweight.contiguous().to(torch.int32)
    qzeros = qzeros.to(device=qweight.device, dtype=torch.int32).contiguous()
    scales = scales.to(device=qweight.device, dtype=torch.float16).contiguous()
    out = torch.empty(N, K, dtype=torch.bfloat16, device=qweight.device)
    call("grag_awq_dequant", ptr(qweight), ptr(qzeros), ptr(scales), ptr(out), K, N, G)
    return out


def dequantize_awq_state_dict(sd: dict, device: torch.device | str | None = None,
                              dtype: torch.dtype = torch.bfloat16) -> dict:
    """Replace every ``<prefix>.qweight/.qzeros/.scales`` triple by
    ``<prefix>.weight`` (HF Linear layout) and cast the remaining floating
    tensors (norms, biases, embeddings) to ``dtype``; non-AWQ dicts pass
    through unchanged."""
    prefixes = [k[:-len(".qweight")] for k in sd if k.endswith(".qweight")]
    if not prefixes:
        return sd
    dev = torch.device(device) if device is not None else None
    out = {}
    skip = set()
    for p in prefixes:
        qw, qz, sc = sd[p + ".qweight"], sd[p + ".qzeros"], sd[p + ".scales"]
        if dev is not None:
            qw, qz, sc = qw.to(dev), qz.to(dev), sc.to(dev)
        out[p + ".weight"] = awq_dequant(qw, qz, sc, dtype if qw.is_cuda else torch.float32).to(dtype)
        skip.update((p + ".qweight", p + ".qzeros", p + ".scales"))
    for k, v in sd.items():
        if k in skip:
            continue
        out[k] = v.to(dtype) if v.is_floating_point() else v
    return out
