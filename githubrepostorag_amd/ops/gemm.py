"""Owned 256x256 MFMA GEMM (csrc/kernels/gemm_tile.hip) with fused epilogues.

    gemm(x, w, b, act)        y = act(x @ w.T + b)              (act: none / gelu-erf / gelu-tanh)
    gemm_silu(x, w_gu, b_gu)  h = silu(x @ wg.T + bg) * (x @ wu.T + bu)

``w_gu`` is the gate/up weight in the kernel's interleaved layout
(``interleave_gate_up``: 32-row gate block j, then 32-row up block j), so one
256-column output tile holds 128 gate and the 128 matching up columns and the
SiLU*mul happens in registers — the [T, 2I] intermediate never reaches HBM.

Decode-sized M (< 256 rows: one row tile) would leave most CUs idle, so the
K dimension is split (``ksplit``): partial fp32 slabs + one combine kernel
that applies the same epilogue.  ``plan_ksplit`` sizes the split so the grid
covers the chip.
"""
from __future__ import annotations

import os

import torch

from ._lib import call, ptr

ACT_NONE, ACT_GELU, ACT_SILU, ACT_GELU_TANH = 0, 1, 2, 3
EPI_STORE, EPI_SILU = 0, 1
_ON = os.environ.get("GRAG_TILE_GEMM", "1") != "0"


def interleave_gate_up(w_gate: torch.Tensor, w_up: torch.Tensor) -> torch.Tensor:
    """[I, K] x 2 -> [2I, K] with rows [64j, 64j+32) = gate[32j:32j+32], [64j+32, 64j+64) = up[32j:..]."""
    I, K = w_gate.shape
    if I % 32:
        raise ValueError("interleave_gate_up: I must be a multiple of 32")
    g = w_gate.reshape(I // 32, 32, *w_gate.shape[1:])
    u = w_up.reshape(I // 32, 32, *w_up.shape[1:])
    return torch.stack([g, u], dim=1).reshape(2 * I, *w_gate.shape[1:]).contiguous()


def deinterleave_gate_up(w: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    I2 = w.shape[0]
    v = w.reshape(I2 // 64, 2, 32, *w.shape[1:])
    return v[:, 0].reshape(I2 // 2, *w.shape[1:]), v[:, 1].reshape(I2 // 2, *w.shape[1:])


def supported(x: torch.Tensor, w: torch.Tensor) -> bool:
    """Shapes/layouts the tile kernel takes (everything else stays on the caller's path)."""
    if not (_ON and x.is_cuda and x.dim() == 2 and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16):
        return False
    M, K = x.shape
    N = w.shape[0]
    return (K % 64 == 0 and K >= 128 and N % 8 == 0 and x.stride(1) == 1 and w.stride(1) == 1
            and x.stride(0) % 8 == 0 and w.stride(0) % 8 == 0 and x.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0)


_NCU: list = []


def _num_cus() -> int:
    if not _NCU:
        _NCU.append(torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
                    if torch.cuda.is_available() else 256)
    return _NCU[0]


def plan_ksplit(M: int, N: int, K: int) -> int:
    """K-splits so tiles x splits covers the CUs (one 512-thread workgroup per CU):
    only when the output tiles alone leave more than half the chip idle, and
    never below 4 K-tiles (256 deep) per split."""
    tiles = -(-M // 256) * -(-N // 256)
    ncu = _num_cus()
    if tiles * 2 > ncu:
        return 1
    kt = K // 64
    s = max(1, min(ncu // tiles, kt // 4))
    while s > 1:
        kts = -(-kt // s)
        if (s - 1) * kts < kt and kt - (s - 1) * kts >= 2:
            break
        s -= 1
    return s


class _Workspace:
    """Per-device fp32 split-K slab; grown only outside hipGraph capture."""

    def __init__(self):
        self.buf: dict = {}
        self.retired: list = []

    def get(self, dev: torch.device, floats: int) -> torch.Tensor:
        b = self.buf.get(dev.index)
        if b is None or b.numel() < floats:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("gemm_tile split-K workspace must be sized before hipGraph capture")
            if b is not None:
                self.retired.append(b)  # captured graphs may still reference it
            b = torch.empty(max(floats, 1 << 20), dtype=torch.float32, device=dev)
            self.buf[dev.index] = b
        return b

    def reserve(self, dev: torch.device, floats: int) -> None:
        self.get(dev, floats)


WS = _Workspace()


def _launch(x, w, b, out, epi, act, ksplit):
    M, K = x.shape
    N = w.shape[0]
    ws = WS.get(x.device, ksplit * M * N) if ksplit > 1 else None
    call("grag_gemm_tile", ptr(x), ptr(w), ptr(b), ptr(out), x.stride(0), w.stride(0), out.stride(0),
         M, N, K, epi, act, ksplit, ptr(ws))
    return out


def gemm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None, act: int = ACT_NONE,
         ksplit: int | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
    """y = act(x @ w.T + b), bf16 [M, N] on the owned MFMA kernel (fp32 CPU reference)."""
    if not x.is_cuda:
        y = torch.nn.functional.linear(x.float(), w.float(), None if b is None else b.float())
        if act == ACT_GELU:
            y = torch.nn.functional.gelu(y)
        elif act == ACT_GELU_TANH:
            y = torch.nn.functional.gelu(y, approximate="tanh")
        return y.to(x.dtype)
    M, K = x.shape
    N = w.shape[0]
    if ksplit is None:
        ksplit = plan_ksplit(M, N, K)
    if out is None:
        out = torch.empty(M, N, dtype=x.dtype, device=x.device)
    return _launch(x, w, b, out, EPI_STORE, act, ksplit)


def gemm_silu(x: torch.Tensor, w_gu: torch.Tensor, b_gu: torch.Tensor | None = None,
              ksplit: int | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
    """h = silu(x @ wg.T + bg) * (x @ wu.T + bu) with ``w_gu`` interleaved (see module doc)."""
    M, K = x.shape
    N2 = w_gu.shape[0]
    if not x.is_cuda:
        wg, wu = deinterleave_gate_up(w_gu)
        bg, bu = (None, None) if b_gu is None else deinterleave_gate_up(b_gu)
        g = torch.nn.functional.linear(x.float(), wg.float(), None if bg is None else bg.float())
        u = torch.nn.functional.linear(x.float(), wu.float(), None if bu is None else bu.float())
        return (torch.nn.functional.silu(g) * u).to(x.dtype)
    if N2 % 64:
        raise ValueError("gemm_silu: 2I must be a multiple of 64")
    if ksplit is None:
        ksplit = plan_ksplit(M, N2, K)
    if out is None:
        out = torch.empty(M, N2 // 2, dtype=x.dtype, device=x.device)
    return _launch(x, w_gu, b_gu, out, EPI_SILU, ACT_NONE, ksplit)
