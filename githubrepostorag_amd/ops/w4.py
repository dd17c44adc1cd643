"""W4A16 weights for the decode GEMM (csrc/kernels/gemm_w4.hip).

The reference serves an AWQ checkpoint (4-bit weights, group-128 scales and
zero points, 16-bit activations; ``helm/values.yaml:67``).  ``W4Linear``
holds one projection in the kernel's packed layout:

* ``q`` 4-bit codes, ``s`` / ``z`` per (row, 128-column group): the weight is
  ``(q - z) * s`` — AWQ's GEMM format (``from_awq``) or round-to-nearest
  min/max quantisation of a bf16 weight (``quantize``);
* packed ``wq`` int32 ``[N/32, K/64, 64, 4]``: per 32-row block and 64-deep
  K-step, lane ``16*h4 + li`` holds 4 words = (tile 0, k-half 0), (0, 1),
  (1, 0), (1, 1); the word of (tile t, half s) carries row ``16t + li``,
  columns ``64*step + 32s + 8*h4 + j`` in nibble ``j`` (bits ``4j``) — the
  MFMA fragment order, so one 16-B load per lane per K-step feeds the wave;
* ``sz`` float32 ``[N, K/128, 2]`` = (s, -z*s) per row and group;
* rows are stored in the order the kernel's waves consume them: natural for
  a plain projection; for the SwiGLU gate/up weight (interleaved in 32-row
  blocks by ``ops/gemm.interleave_gate_up``) each 32-row block is the 16 gate
  rows of one 16-column output group followed by the 16 matching up rows.

Prefill stays on bf16 GEMMs: ``dequant()`` returns the bf16 weight these 4-bit
codes represent, so both phases compute with the same (quantised) weights.
"""
from __future__ import annotations

import os

import torch

from ._lib import call, ptr
from .gemm import ACT_NONE, EPI_SILU, EPI_STORE, WS, _num_cus

GROUP = 128
W4_VARIANTS = [(4, 4), (8, 4), (12, 4), (16, 4)]  # (mt, nwv) compiled (csrc/kernels/gemm_w4.hip)
W4_MAX_M = 256  # largest compiled row tiling (16 x 16 rows)


def quantize(w: torch.Tensor, group: int = GROUP) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Round-to-nearest asymmetric 4-bit quantisation per (row, group): returns q uint8 [N, K],
    s float32 [N, K/group], z uint8 [N, K/group] with w ~ (q - z) * s."""
    N, K = w.shape
    g = w.float().reshape(N, K // group, group)
    lo, hi = g.amin(-1), g.amax(-1)
    s = ((hi - lo) / 15.0).clamp_min(1e-8)
    z = torch.round(-lo / s).clamp(0, 15)
    q = torch.round(g / s.unsqueeze(-1) + z.unsqueeze(-1)).clamp(0, 15)
    return q.reshape(N, K).to(torch.uint8), s, z.to(torch.uint8)


def gate_up_order(n2: int) -> torch.Tensor:
    """Consumption row order of an interleaved [2I, K] gate/up weight: per 16-column output group b,
    its 16 gate rows then the 16 matching up rows."""
    o = torch.arange(n2 // 2)
    gate = (o // 32) * 64 + o % 32
    blocks = gate.view(-1, 16)
    return torch.cat([blocks, blocks + 32], 1).reshape(-1)


def pack(q: torch.Tensor, s: torch.Tensor, z: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """(q [N, K], s [N, G], z [N, G]) in consumption row order -> (wq int32 [N/32, K/64, 64, 4], sz)."""
    N, K = q.shape
    qq = q.to(torch.int64).view(N // 32, 2, 16, K // 64, 2, 4, 8)       # [b, nt, li, t, s, h4, j]
    qq = qq.permute(0, 3, 5, 2, 1, 4, 6).reshape(N // 32, K // 64, 64, 4, 8)  # [b, t, h4*16+li, nt*2+s, j]
    words = (qq << (4 * torch.arange(8, device=q.device))).sum(-1)
    words = torch.where(words >= 2 ** 31, words - 2 ** 32, words).to(torch.int32).contiguous()
    sz = torch.stack([s.float(), -z.float() * s.float()], -1).contiguous()
    return words, sz


class W4Linear:
    """One projection's 4-bit weight in the gemm_w4 layout (see module doc)."""

    def __init__(self, q: torch.Tensor, s: torch.Tensor, z: torch.Tensor, silu: bool = False):
        N, K = q.shape
        if N % 32 or K % 256 or K % GROUP:
            raise ValueError(f"W4Linear needs N % 32 == 0 and K % 256 == 0 (got {N} x {K})")
        self.N, self.K, self.silu = N, K, silu
        self.order = gate_up_order(N).to(q.device) if silu else None
        self.q, self.s, self.z = q, s, z  # natural row order (reference / dequant)
        qo, so, zo = (q, s, z) if self.order is None else (q[self.order], s[self.order], z[self.order])
        self.wq, self.sz = pack(qo, so, zo)

    @classmethod
    def quantize(cls, w: torch.Tensor, silu: bool = False) -> "W4Linear":
        q, s, z = quantize(w)
        return cls(q, s, z, silu)

    @classmethod
    def from_awq(cls, qweight: torch.Tensor, qzeros: torch.Tensor, scales: torch.Tensor,
                 silu: bool = False) -> "W4Linear":
        """AutoAWQ GEMM tensors (qweight int32 [K, N/8], qzeros int32 [K/G, N/8], scales fp16 [K/G, N])."""
        from .quant import unpack_awq

        if qweight.shape[0] // scales.shape[0] != GROUP:
            raise ValueError("gemm_w4 is built for group size 128")
        q = unpack_awq(qweight).t().contiguous().to(torch.uint8)
        z = unpack_awq(qzeros).t().contiguous().to(torch.uint8)
        return cls(q, scales.float().t().contiguous(), z, silu)

    def release_codes(self) -> None:
        """Drop the unpacked codes (1 B per weight) once the packed copy and any bf16 copy exist."""
        self.q = self.s = self.z = None

    def dequant(self, dtype=torch.bfloat16) -> torch.Tensor:
        """(q - z) * s as [N, K] in natural row order."""
        if self.q is None:
            raise RuntimeError("W4Linear codes were released")
        N, K = self.q.shape
        w = (self.q.float().view(N, K // GROUP, GROUP) - self.z.float().unsqueeze(-1)) * self.s.float().unsqueeze(-1)
        return w.view(N, K).to(dtype)

    def bytes(self) -> int:
        return self.wq.numel() * 4 + self.sz.numel() * 4


def w4_ksplit(K: int, ksplit: int) -> int:
    """Effective K-splits of the W4 kernel (same rule as grag_gemm_w4: ceil(kt / ksplit) steps each)."""
    kt = K // 64
    kts = -(-kt // max(1, ksplit))
    return -(-kt // kts)


def tiling(M: int, N: int, K: int, silu: bool = False) -> tuple[int, int, int] | None:
    """(mt, nwv, ksplit) the kernel runs M rows with: the smallest compiled row tiling that covers M and
    about one workgroup per CU (K-split for narrow outputs).  None when no tiling fits."""
    if M < 1 or M > W4_MAX_M:
        return None
    need = -(-M // 16)
    vs = [v for v in W4_VARIANTS if v[0] >= need and N % (32 * v[1]) == 0]
    if not vs:
        return None
    mt, nwv = min(vs)
    tiles = N // (32 * nwv)
    ncu = _num_cus()
    ks = 1 if silu or tiles >= ncu else w4_ksplit(K, max(1, ncu // tiles))
    return mt, nwv, ks


def w4_wins(M: int, N: int, K: int, silu: bool = False) -> bool:
    """Dispatch rule from the hipGraph-timed A/B of scripts/w4_probe.py --graph (profiles/w4_probe_graph_r3.jsonl:
    each arm captured as 12 back-to-back launches on cold weight copies, Qwen2-7B shapes, M 1..256):
      gate/up (SwiGLU, N = 37888): W4 1.55x at M <= 32, 1.13x at 64, loses from 96 on (0.53x at 256);
      down (deep K = 18944): W4 1.2-1.5x at M <= 64, 1.05-1.1x at 96-128, loses from 192 on;
      qkv / o (K = N-ish, 26-33 MB bf16): the bf16 decode kernels are at or ahead of W4 everywhere
      (0.72-1.06x): the 4x fewer weight bytes do not pay below ~40 MB of bf16 weight per launch.
    GRAG_W4_MIN_M / GRAG_W4_MAX_M (rows) pin the range for every projection instead (tests, sweeps)."""
    lo, hi = os.environ.get("GRAG_W4_MIN_M"), os.environ.get("GRAG_W4_MAX_M")
    if lo is not None or hi is not None:
        return int(lo or 1) <= M <= int(hi or W4_MAX_M)
    if silu:
        return M <= 64
    return K >= 4 * N and M <= 128


def plan(M: int, N: int, K: int, silu: bool = False) -> tuple[int, int, int] | None:
    """The W4 kernel's tiling for this decode batch when it is the faster path (``w4_wins``), else None
    (the caller runs the bf16 decode kernel on the dequantised copy of the same weights)."""
    return tiling(M, N, K, silu) if w4_wins(M, N, K, silu) else None


def gemm_w4(x: torch.Tensor, w: W4Linear, bias: torch.Tensor | None = None, act: int = ACT_NONE,
            plan_: tuple[int, int, int] | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
    """y = act(x @ dequant(w).T + bias) (SwiGLU product [M, N/2] for a gate/up weight; ``bias`` in the
    weight's natural row order)."""
    M, K = x.shape
    if K != w.K:
        raise ValueError(f"gemm_w4: x has K={K}, weight {w.K}")
    if not x.is_cuda:  # fp32 reference
        y = torch.nn.functional.linear(x.float(), w.dequant(torch.float32), None if bias is None else bias.float())
        if w.silu:
            v = y.view(M, -1, 2, 32)
            y = (torch.nn.functional.silu(v[:, :, 0]) * v[:, :, 1]).reshape(M, -1)
        return y.to(x.dtype)
    mt, nwv, ks = plan_ or tiling(M, w.N, K, w.silu)
    ks = 1 if w.silu else w4_ksplit(K, ks)
    if out is None:
        out = torch.empty(M, w.N // 2 if w.silu else w.N, dtype=x.dtype, device=x.device)
    fl = ks * M * w.N if ks > 1 else 0
    ws = WS.get(x.device, fl) if fl else None
    b = None if bias is None else (bias if w.order is None else bias[w.order]).contiguous()
    call("grag_gemm_w4", ptr(x), ptr(w.wq), ptr(w.sz), ptr(b), ptr(out), x.stride(0), out.stride(0), M, w.N, K,
         EPI_SILU if w.silu else EPI_STORE, act, mt, nwv, ks, ptr(ws))
    return out


def capture_ok(dev: torch.device, M: int, w: W4Linear) -> bool:
    p = plan(M, w.N, w.K, w.silu)
    if p is None:
        return False
    fl = p[2] * M * w.N if p[2] > 1 else 0
    return fl == 0 or not torch.cuda.is_current_stream_capturing() or WS.ready(dev, fl)
