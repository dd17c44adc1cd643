"""Linear layers.

* decode-sized inputs (M <= SKINNY_MAX_M rows, K % 32 == 0): the hand-written
  weight-streaming MFMA kernel ``grag_gemm_skinny`` (HBM-bound regime: every
  weight byte read once per step, nontemporal loads, intra-workgroup split-K);
* larger M (prefill, encoder batches): plain GEMMs go to hipBLASLt through
  ``torch.nn.functional.linear`` — the library is used only for plain
  (epilogue-free / bias-only) GEMMs; everything fused around them
  (bias+RoPE+KV store, SiLU*mul, bias+GELU, bias+residual+LayerNorm,
  residual+RMSNorm, pooling) is a hand-written HIP kernel in ops/*.
"""
from __future__ import annotations

import os

import torch

from ._lib import call, ptr

SKINNY_MAX_M = int(os.environ.get("GRAG_SKINNY_MAX_M", "64"))
_SKINNY_ON = os.environ.get("GRAG_SKINNY", "1") != "0"


def gemm_skinny(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None, nt: int = 0) -> torch.Tensor:
    M, K = x.shape
    N = w.shape[0]
    out = torch.empty(M, N, dtype=x.dtype, device=x.device)
    call("grag_gemm_skinny", ptr(x), ptr(w), ptr(b), ptr(out), x.stride(0), w.stride(0), out.stride(0), M, N, K, nt)
    return out


def use_skinny(M: int, N: int, K: int) -> bool:
    """Dispatch rule from the cold-cache A/B of scripts/microbench.py
    (profiles/microbench_gemm.json): the streaming kernel wins at M <= 16
    except for very wide outputs (N >= 8K with K <= 4K, e.g. gate_up), and at
    M <= 64 for square-ish projections (o_proj)."""
    if M <= 16:
        return not (N >= 8192 and K <= 4096 and N >= 8 * K)
    if M <= SKINNY_MAX_M:
        return N <= 4096 and K <= 4096
    return False


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None) -> torch.Tensor:
    """y = x @ w.T (+ b); w is [out, in] (K-contiguous, TN GEMM)."""
    if not x.is_cuda:
        if x.dtype == torch.bfloat16:
            y = torch.nn.functional.linear(x.float(), w.float(), None if b is None else b.float())
            return y.to(x.dtype)
        return torch.nn.functional.linear(x, w, b)
    if (_SKINNY_ON and x.dim() == 2 and x.shape[1] % 64 == 0 and use_skinny(x.shape[0], w.shape[0], x.shape[1])
            and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.stride(1) == 1 and w.stride(1) == 1):
        return gemm_skinny(x, w, b)
    return torch.nn.functional.linear(x, w, b)
