"""Normalisation / embedding ops (HIP on device tensors, fp32 reference on CPU)."""
from __future__ import annotations

import os

import torch

from ._lib import call, ptr
from .gemm import SplitKPartial


def _on_gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


def rmsnorm_ref(x, w, eps, residual=None):
    if residual is not None:
        s = (x.float() + residual.float()).to(x.dtype)
        residual.copy_(s)
        xf = s.float()
    else:
        xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    return y.to(x.dtype)


# the chunked ticket-merge kernel measured slower than one workgroup per row at B = 1 (8.6 vs 5.6 us: the
# agent-scope release / acquire round trips outweigh the parallel plane reads; profiles/decode_step_b1_r5.txt)
SMALL_ROWS = int(os.environ.get("GRAG_NORM_SMALL_ROWS", "0"))


def norm_ws(dev) -> tuple[torch.Tensor, torch.Tensor]:
    """(tickets [64] int32, zeroed; chunk sums [64 * 64] fp32) of the small-batch split-K RMSNorm, owned by
    the caller's workspace owner (ops/gemm.py WS.scratch); allocated before any hipGraph capture (LLMEngine
    does, under its owner) -- every last arriver resets its ticket."""
    from .gemm import WS

    return WS.scratch("norm_tickets", torch.device(dev),
                      lambda d: (torch.zeros(64, dtype=torch.int32, device=d), torch.zeros(64 * 64, device=d)))


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, residual: torch.Tensor | None = None,
            out: torch.Tensor | None = None) -> torch.Tensor:
    """y = RMSNorm(x [+ residual]) * w.  With ``residual`` the sum is written
    back into ``residual`` (the decoder's residual stream), fused in one pass."""
    if isinstance(x, SplitKPartial):  # deferred split-K projection: reduce + residual add + norm in one pass
        if residual is None:
            x = x.materialize()
        else:
            out = torch.empty(x.M, x.N, dtype=x.dtype, device=x.device) if out is None else out
            if x.M <= SMALL_ROWS:  # 1-16 rows: the row's planes reduced by ceil(N / 512) workgroups
                ws = norm_ws(x.device)
                call("grag_splitk_add_rmsnorm_small", ptr(x.planes), x.S, ptr(residual), ptr(w), ptr(out), x.M, x.N,
                     float(eps), ptr(ws[1]), ptr(ws[0]))
            else:
                call("grag_splitk_add_rmsnorm", ptr(x.planes), x.S, ptr(residual), ptr(w), ptr(out), x.M, x.N,
                     float(eps))
            return out
    if not _on_gpu(x):
        return rmsnorm_ref(x, w, eps, residual)
    x = x.contiguous()
    T, H = x.shape[0] if x.dim() == 2 else x.numel() // x.shape[-1], x.shape[-1]
    out = torch.empty_like(x) if out is None else out
    call("grag_rmsnorm", ptr(x), ptr(residual), ptr(w), ptr(out), T, H, float(eps))
    return out


def layernorm_ref(x, gamma, beta, eps, bias=None, residual=None):
    v = x.float()
    if bias is not None:
        v = v + bias.float()
    if residual is not None:
        v = v + residual.float()
    return torch.nn.functional.layer_norm(v, (v.shape[-1],), gamma.float(), beta.float(), eps).to(x.dtype)


def layernorm(x, gamma, beta, eps, bias=None, residual=None):
    """y = LN(x [+ bias] [+ residual]) * gamma + beta (BERT post-LN block)."""
    if not _on_gpu(x):
        return layernorm_ref(x, gamma, beta, eps, bias, residual)
    x = x.contiguous()
    H = x.shape[-1]
    T = x.numel() // H
    out = torch.empty_like(x)
    call("grag_layernorm", ptr(x), ptr(bias), ptr(residual), ptr(gamma), ptr(beta), ptr(out), T, H, float(eps))
    return out


def add_layernorm_ref(x, gamma, beta, eps, residual, bias=None):
    v = x.float() + residual.float()
    if bias is not None:
        v = v + bias.float()
    s = v.to(residual.dtype)
    residual.copy_(s)
    return torch.nn.functional.layer_norm(s.float(), (v.shape[-1],), gamma.float(), beta.float(),
                                          eps).to(x.dtype)


def add_layernorm(x, gamma, beta, eps, residual, bias=None):
    """Pre-LN block boundary (GPT-2): ``residual += x [+ bias]`` in place, then
    return LN(residual) * gamma + beta — one pass over the row."""
    if not _on_gpu(x):
        return add_layernorm_ref(x, gamma, beta, eps, residual, bias)
    x = x.contiguous()
    H = x.shape[-1]
    T = x.numel() // H
    out = torch.empty_like(x)
    call("grag_add_layernorm", ptr(x), ptr(bias), ptr(residual), ptr(gamma), ptr(beta), ptr(out), T, H,
         float(eps))
    return out


def bert_embed_ln_ref(ids, pos_ids, type_ids, word, pos, typ, gamma, beta, eps):
    v = word[ids.long()].float() + pos[pos_ids.long()].float()
    v = v + (typ[type_ids.long()].float() if type_ids is not None else typ[0].float())
    return torch.nn.functional.layer_norm(v, (v.shape[-1],), gamma.float(), beta.float(), eps).to(word.dtype)


def bert_embed_ln(ids, pos_ids, type_ids, word, pos, typ, gamma, beta, eps):
    if not _on_gpu(word):
        return bert_embed_ln_ref(ids, pos_ids, type_ids, word, pos, typ, gamma, beta, eps)
    T, H = ids.numel(), word.shape[1]
    out = torch.empty(T, H, dtype=word.dtype, device=word.device)
    ids = ids.to(torch.int32).contiguous()
    pos_ids = pos_ids.to(torch.int32).contiguous()
    type_ids = None if type_ids is None else type_ids.to(torch.int32).contiguous()
    call("grag_bert_embed_ln", ptr(ids), ptr(pos_ids), ptr(type_ids), ptr(word), ptr(pos), ptr(typ),
         ptr(gamma), ptr(beta), ptr(out), T, H, word.shape[0], pos.shape[0], float(eps))
    return out


def embed_gather(ids: torch.Tensor, table: torch.Tensor) -> torch.Tensor:
    if not _on_gpu(table):
        return table[ids.long()]
    ids = ids.to(torch.int32).contiguous()
    T, H = ids.numel(), table.shape[1]
    out = torch.empty(T, H, dtype=table.dtype, device=table.device)
    call("grag_embed_gather", ptr(ids), ptr(table), ptr(out), T, H, table.shape[0])
    return out
