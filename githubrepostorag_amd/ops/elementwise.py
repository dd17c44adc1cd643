"""Fused elementwise ops: QKV bias+RoPE+paged-KV store, SiLU*mul, bias+act,
pooling + L2 normalisation."""
from __future__ import annotations

import math

import torch

from ._lib import call, ptr

ACT_NONE, ACT_GELU, ACT_SILU, ACT_GELU_TANH = 0, 1, 2, 3


def rope_cos_sin(max_pos: int, head_dim: int, theta: float, device=None) -> torch.Tensor:
    """NeoX rotary table [max_pos, head_dim] fp32: cos in [:D/2], sin in [D/2:]."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    return torch.cat([f.cos(), f.sin()], dim=-1).float().to(device)


def qkv_rope_kvstore_ref(qkv, bias, positions, cos_sin, slot_mapping, k_cache, v_cache, Hq, Hkv, D):
    T = qkv.shape[0]
    x = qkv.float()
    if bias is not None:
        x = (x + bias.float()).to(qkv.dtype).float()
    q = x[:, : Hq * D].view(T, Hq, D)
    k = x[:, Hq * D : (Hq + Hkv) * D].view(T, Hkv, D)
    v = x[:, (Hq + Hkv) * D : (Hq + 2 * Hkv) * D].view(T, Hkv, D)
    if cos_sin is not None:  # None: no rotary (GPT-2 absolute positions)
        cs = cos_sin[positions.long()]
        cos, sin = cs[:, : D // 2].unsqueeze(1), cs[:, D // 2 :].unsqueeze(1)

        def rot(t):
            a, b = t[..., : D // 2], t[..., D // 2 :]
            return torch.cat([a * cos - b * sin, b * cos + a * sin], dim=-1)

        q, k = rot(q), rot(k)
    if slot_mapping is not None and k_cache is not None:
        BS = k_cache.shape[2]
        sm = slot_mapping.long()
        ok = sm >= 0
        blk, off = sm[ok] // BS, sm[ok] % BS
        k_cache[blk, :, off] = k[ok].to(k_cache.dtype)
        v_cache[blk, :, off] = v[ok].to(v_cache.dtype)
    return q.to(qkv.dtype).contiguous()


def qkv_rope_kvstore(qkv, bias, positions, cos_sin, slot_mapping, k_cache, v_cache, Hq, Hkv, D):
    """Split packed QKV [T, (Hq+2Hkv)*D], add bias, apply NeoX RoPE to q/k
    (skipped when ``cos_sin`` is None), return q [T, Hq, D] and scatter k/v
    into the paged caches [blocks, Hkv, BS, D].  ``qkv`` may be the deferred fp32 split-K planes of the
    projection (ops/gemm.py SplitKPartial): the kernel then folds the split-K reduce into this pass."""
    from .gemm import SplitKPartial

    if isinstance(qkv, SplitKPartial):
        if not qkv.device.type == "cuda":
            qkv = qkv.materialize()
        else:
            T = qkv.M
            q = torch.empty(T, Hq, D, dtype=qkv.dtype, device=qkv.device)
            call("grag_qkv_rope_kvstore_planes", ptr(qkv.planes), qkv.S, qkv.N, ptr(bias), ptr(positions),
                 ptr(cos_sin), ptr(slot_mapping), ptr(q), ptr(k_cache), ptr(v_cache), T, Hq, Hkv, D,
                 k_cache.shape[2], *_bounds(k_cache, cos_sin, D))
            return q
    if not qkv.is_cuda:
        return qkv_rope_kvstore_ref(qkv, bias, positions, cos_sin, slot_mapping, k_cache, v_cache, Hq, Hkv, D)
    T = qkv.shape[0]
    q = torch.empty(T, Hq, D, dtype=qkv.dtype, device=qkv.device)
    BS = k_cache.shape[2]
    call("grag_qkv_rope_kvstore", ptr(qkv), qkv.stride(0), ptr(bias), ptr(positions), ptr(cos_sin),
         ptr(slot_mapping), ptr(q), ptr(k_cache), ptr(v_cache), T, Hq, Hkv, D, BS, *_bounds(k_cache, cos_sin, D))
    return q


def _bounds(k_cache, cos_sin, D) -> tuple[int, int]:
    """(KV slots, cos/sin rows): the kernel's index-guard limits for slot_mapping / positions."""
    nslots = 0 if k_cache is None else k_cache.shape[0] * k_cache.shape[2]
    npos = 0 if cos_sin is None else cos_sin.numel() // D
    return nslots, npos


def silu_mul(gu: torch.Tensor) -> torch.Tensor:
    I = gu.shape[-1] // 2
    if not gu.is_cuda:
        g, u = gu[..., :I].float(), gu[..., I:].float()
        return (torch.nn.functional.silu(g) * u).to(gu.dtype)
    gu = gu.contiguous()
    T = gu.numel() // (2 * I)
    out = torch.empty(*gu.shape[:-1], I, dtype=gu.dtype, device=gu.device)
    call("grag_silu_mul", ptr(gu), ptr(out), T, I)
    return out


def bias_act(x: torch.Tensor, b: torch.Tensor | None, act: int, inplace: bool = False) -> torch.Tensor:
    if not x.is_cuda:
        v = x.float() + (b.float() if b is not None else 0.0)
        if act == ACT_GELU:
            v = torch.nn.functional.gelu(v)
        elif act == ACT_SILU:
            v = torch.nn.functional.silu(v)
        elif act == ACT_GELU_TANH:
            v = torch.nn.functional.gelu(v, approximate="tanh")
        return v.to(x.dtype)
    x = x.contiguous()
    N = x.shape[-1]
    T = x.numel() // N
    y = x if inplace else torch.empty_like(x)
    call("grag_bias_act", ptr(x), ptr(b), ptr(y), T, N, act)
    return y


POOL_MEAN, POOL_CLS = 0, 1


def pool_l2norm_ref(hidden, starts, lengths, mode, normalize=True):
    """hidden [T, H] packed rows; sequence b = rows starts[b] .. +lengths[b]."""
    outs = []
    h = hidden.float()
    for st, ln in zip(starts.tolist(), lengths.tolist()):
        ln = max(1, ln)
        v = h[st] if mode == POOL_CLS else h[st:st + ln].mean(0)
        outs.append(v)
    v = torch.stack(outs) if outs else torch.zeros(0, hidden.shape[-1], device=hidden.device)
    if normalize:
        v = v / v.norm(dim=-1, keepdim=True).clamp_min(1e-12)
    return v


def pool_l2norm(hidden: torch.Tensor, starts: torch.Tensor, lengths: torch.Tensor, mode: int = POOL_MEAN,
                normalize: bool = True, want_bf16: bool = False):
    """Packed hidden rows [T, H] -> fp32 [B, H] (and a bf16 copy) pooled over
    each sequence (mean or CLS) and L2-normalised, in one kernel."""
    if not hidden.is_cuda:
        f = pool_l2norm_ref(hidden, starts, lengths, mode, normalize)
        return (f, f.to(torch.bfloat16)) if want_bf16 else f
    B, H = lengths.numel(), hidden.shape[-1]
    starts = starts.to(torch.int32).contiguous()
    lengths = lengths.to(torch.int32).contiguous()
    outf = torch.empty(B, H, dtype=torch.float32, device=hidden.device)
    outb = torch.empty(B, H, dtype=torch.bfloat16, device=hidden.device) if want_bf16 else None
    call("grag_pool_l2norm", ptr(hidden.contiguous()), ptr(starts), ptr(lengths), ptr(outf), ptr(outb), B, 0,
         H, mode, 1 if normalize else 0)
    return (outf, outb) if want_bf16 else outf


def softmax_scale(head_dim: int) -> float:
    return 1.0 / math.sqrt(head_dim)
