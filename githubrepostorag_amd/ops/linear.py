"""Plain linear layers.

Plain (epilogue-free or bias-only) GEMMs go to hipBLASLt through
``torch.nn.functional.linear`` — the task's rule is library GEMMs only for
plain GEMMs.  Everything fused around them (bias+RoPE+KV store, SiLU*mul,
bias+GELU, bias+residual+LayerNorm, residual+RMSNorm, pooling) is a
hand-written HIP kernel in ops/*.
"""
from __future__ import annotations

import torch


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None) -> torch.Tensor:
    """y = x @ w.T (+ b); w is [out, in] (K-contiguous, TN GEMM)."""
    if not x.is_cuda and x.dtype == torch.bfloat16:
        y = torch.nn.functional.linear(x.float(), w.float(), None if b is None else b.float())
        return y.to(x.dtype)
    return torch.nn.functional.linear(x, w, b)
