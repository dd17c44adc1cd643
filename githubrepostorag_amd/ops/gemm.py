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

import bisect
import contextlib
import json
import os
import threading
from pathlib import Path

import torch

from ._lib import call, ptr

ACT_NONE, ACT_GELU, ACT_SILU, ACT_GELU_TANH = 0, 1, 2, 3
EPI_STORE, EPI_SILU, EPI_PARTIAL = 0, 1, 2
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


SK_EFF = float(os.environ.get("GRAG_TILE_SK_EFF", "0.92"))


def plan(M: int, N: int, K: int) -> tuple[int, int]:
    """(ksplit, sk_grid) for a shape.  Few tiles (<= half the CUs): split-K.
    Otherwise whole tiles per workgroup, unless the last round of tiles would
    leave the chip idle enough (tiles / (rounds * CUs) < SK_EFF): then the
    last full round plus the remainder are shared by one stream-K round.
    Measured (profiles/gemm_tile_ab_v2.jsonl): stream-K pays only with >= 2
    rounds ahead of it (down_proj M=16384: 1721 -> 1534 us); an all-stream-K
    grid (one round or less) loses to whole tiles (o_proj M=4096 95 -> 149 us,
    gate_up M=192 94 -> 102 us: the fixup slabs cost more than the idle CUs)."""
    ks = plan_ksplit(M, N, K)
    if ks > 1:
        return ks, 0
    tiles = -(-M // 256) * -(-N // 256)
    ncu = _num_cus()
    if tiles % ncu == 0 or tiles <= 2 * ncu:
        return 1, 0
    eff = tiles / (-(-tiles // ncu) * ncu)
    return (1, ncu) if eff < SK_EFF else (1, 0)


def sk_ok(M: int, N: int, K: int, ksplit: int, sk: int) -> bool:
    """The launcher's schedule rule (grag_gemm_tile): a stream-K round must give every workgroup at least
    half a tile of K-steps (a quarter for the tail-only mode, sk < 0)."""
    kt = K // 64
    if ksplit > 1:
        kts = -(-kt // ksplit)
        return kts >= 2 and (ksplit - 1) * kts < kt and kt - (ksplit - 1) * kts >= 2
    tiles = -(-M // 256) * -(-N // 256)
    skg = abs(sk)
    ncu = _num_cus()
    if skg == 0 or tiles % (ncu if sk < 0 else skg) == 0:
        return True
    rounds = tiles // skg
    dp = (tiles // ncu) * ncu if sk < 0 else (rounds - 1) * skg if rounds >= 1 else 0
    return (tiles - dp) * kt >= skg * ((kt + 3) // 4 if sk < 0 else (kt + 1) // 2)


_PREFILL = {"table": None}
PREFILL_TABLE = Path(__file__).resolve().parents[1] / "tuning" / "gemm_prefill_gfx950.json"


def _prefill_table() -> dict:
    if _PREFILL["table"] is None:
        t = {}
        env = os.environ.get("GRAG_PREFILL_TABLE", "1")  # "0": no table; a path: that table (A/B runs)
        path = Path(env) if env not in ("0", "1") else PREFILL_TABLE
        if env != "0" and path.exists():
            for k, rows in json.loads(path.read_text())["table"].items():
                t[tuple(map(int, k.split(",")))] = ([r[0] for r in rows], rows)
        _PREFILL["table"] = t
    return _PREFILL["table"]


def prefill_plan(M: int, N: int, K: int, silu: bool = False) -> tuple[int, int] | None:
    """(ksplit, sk) of the owned kernel for a prefill-sized GEMM, or None for the library.

    From the dense M sweep of scripts/sweep_prefill_gemm.py (tuning/gemm_prefill_gfx950.json; library
    with the TunableOp solutions loaded vs every owned schedule, 256-row buckets).  The library's
    heuristic swings with M (Qwen2-7B down_proj: 605 us at M = 5504, 1103 us at 6016, 678 us at 6784,
    1131 us at 7040; owned 650-770 us across the range), so the library is taken only where it won at
    both buckets around M; otherwise the owned schedule measured at the bucket at or above M (re-checked
    against the launcher rule at this M).  SwiGLU shapes are always owned (the library needs a separate
    SiLU*mul pass: owned won all 63 buckets on Qwen2-7B / 1.5B).  Of the two buckets around M, the one on M's
    own row-tile grid is preferred (its schedule was measured on the identical tile count), and a tail-only
    stream-K grid is re-derived for M's own remainder (``_tail_grid``).  Unmeasured shapes: None (library)
    for plain GEMMs, ``plan`` for SwiGLU."""
    t = _prefill_table().get((N, K, int(silu)))
    if t is None:
        return plan(M, N, K) if silu else None
    ms, rows = t
    i = bisect.bisect_left(ms, M)
    cand = [rows[min(i, len(rows) - 1)]]
    if 0 < i < len(rows) and ms[i] != M:
        cand.append(rows[i - 1])
    # SwiGLU: owned at every bucket; plain GEMMs: owned unless the library was clearly faster (OWN_SLACK:
    # near-ties, within box-to-box spread, go to the owned kernel)
    won = [r for r in cand if r[2] is not None and (silu or r[1] is None or r[2] < r[1] * OWN_SLACK)]
    if not won:
        return plan(M, N, K) if silu else None
    # a bucket with M's own row-tile count ran on the identical tile grid: its schedule transfers as is
    same = [r for r in won if -(-r[0] // 256) == -(-M // 256)]
    if same:
        won = same
    ks, sk = won[0][3], won[0][4]
    if ks == 1 and sk < 0:
        sk = _tail_grid(won[0][0], M, N, sk)
    return (ks, sk) if sk_ok(M, N, K, ks, sk) else (1, 0)


def _tail_grid(Mb: int, M: int, N: int, sk: int) -> int:
    """A tail-only stream-K grid measured at bucket Mb, re-derived for M: the sweep's grids are 1x / 2x / 4x
    the tiles left after the full CU rounds (or one per CU), so keep that ratio to M's own remainder (0: no
    remainder, whole tiles)."""
    ncu = _num_cus()
    tn = -(-N // 256)
    tail_b, tail = (-(-Mb // 256) * tn) % ncu, (-(-M // 256) * tn) % ncu
    if tail == 0:
        return 0
    if tail_b and -sk > tail_b and -sk % tail_b == 0:  # K-aligned split: s parts per leftover tile
        return -(-sk // tail_b) * tail
    if -sk >= ncu or tail_b == 0:
        return -ncu
    return -min(ncu, max(1, round(-sk * tail / tail_b)))


OWN_SLACK = float(os.environ.get("GRAG_OWN_SLACK", "1.06"))  # beyond the 3-5 % box-to-box spread
PREFILL_MIN_M = 257  # above one 256-row tile: the prefill regime (decode batches use plan())


def schedule(M: int, N: int, K: int, silu: bool = False) -> tuple[int, int]:
    """(ksplit, sk) the owned kernel runs a shape with when the caller does not pin one."""
    if M >= PREFILL_MIN_M:
        p = prefill_plan(M, N, K, silu)
        if p is not None:
            return p
    return plan(M, N, K)


def set_mfma(mf: int) -> int:
    """Select the tile kernel's MFMA shape for later launches (16: v_mfma_f32_16x16x32_bf16, the default;
    32: v_mfma_f32_32x32x16_bf16; csrc/kernels/gemm_tile.hip ``Shape``).  Returns the previous shape."""
    from ._lib import lib

    return int(lib().grag_gemm_tile_mfma(int(mf)))


def set_sched(sched: int) -> int:
    """Select the 16x16x32 tile kernel's phase schedule (0: 12/4/8/0 fragment reads per phase; 1: the
    balanced 8/4/8/4 order; 2: two phases of 32 MFMAs per K-tile -- csrc/kernels/gemm_tile.hip ``SCHED``).
    Returns the previous schedule."""
    from ._lib import lib

    return int(lib().grag_gemm_tile_sched(int(sched)))


def _ws_floats(M: int, N: int, ksplit: int, sk: int) -> int:
    return ksplit * M * N if ksplit > 1 else (2 * abs(sk) * 65536 if sk else 0)


class _Workspace:
    """fp32 split-K slabs, one per (thread, device): the engine thread and the
    retrieval threads run GEMMs on different streams concurrently, so a shared
    slab would race.  Grown only outside hipGraph capture (a capture reuses the
    slab its eager warm-up step sized); outgrown slabs stay alive because
    captured graphs may still point at them."""

    def __init__(self):
        self._tls = threading.local()
        self.retired: list = []

    def _bufs(self) -> dict:
        o = getattr(self._tls, "owner", None)  # an engine's own workspace while it runs (WS.owned_by)
        if o is not None:
            return o.setdefault("bufs", {})
        bufs = getattr(self._tls, "bufs", None)
        if bufs is None:
            bufs = self._tls.bufs = {}
        return bufs

    def _cnts(self) -> dict:
        o = getattr(self._tls, "owner", None)
        if o is not None:
            return o.setdefault("cnts", {})
        cs = getattr(self._tls, "cnts", None)
        if cs is None:
            cs = self._tls.cnts = {}
        return cs

    @contextlib.contextmanager
    def owned_by(self, owner: dict):
        """Route this thread's workspace requests to ``owner`` (a dict the caller keeps) for the block.  An
        engine runs its steps and graph captures under its own dict: a captured decode graph then points at
        memory the ENGINE owns -- not at the capturing thread's buffers, which another thread's eager GEMMs
        may be using when the graph replays (the harness captures on the main thread, an EngineRunner thread
        replays) and which a thread-local dict would free when that thread exits."""
        prev = getattr(self._tls, "owner", None)
        self._tls.owner = owner
        try:
            yield
        finally:
            self._tls.owner = prev

    def get(self, dev: torch.device, floats: int) -> torch.Tensor:
        bufs = self._bufs()
        b = bufs.get(dev.index)
        if b is None or b.numel() < floats:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("gemm_tile split-K workspace must be sized before hipGraph capture")
            if b is not None:
                self.retired.append(b)
            b = torch.empty(max(floats, 1 << 20), dtype=torch.float32, device=dev)
            bufs[dev.index] = b
        return b

    def ready(self, dev: torch.device, floats: int) -> bool:
        b = self._bufs().get(dev.index)
        return b is not None and b.numel() >= floats

    def has_counters(self, dev: torch.device) -> bool:
        return self._cnts().get(dev.index) is not None

    def counters(self, dev: torch.device) -> torch.Tensor:
        """Stream-K arrival tickets: zero at rest (each tile's last arriver resets its word)."""
        cs = self._cnts()
        c = cs.get(dev.index)
        if c is None:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("gemm_tile stream-K counters must be allocated before hipGraph capture")
            c = cs[dev.index] = torch.zeros(1 << 14, dtype=torch.int32, device=dev)
        return c

    def reserve(self, dev: torch.device, floats: int) -> None:
        self.get(dev, floats)

    def owner(self) -> dict | None:
        """The owner dict this thread's launches are routed to (None: thread-local scratch)."""
        return getattr(self._tls, "owner", None)

    def scratch(self, name: str, dev: torch.device, make):
        """A persistent per-owner scratch tensor (ticket arrays, small merge buffers) under ``name``: the
        owner's (an engine's, an embedder's) while one is set, else this thread's.  Every kernel that keeps
        cross-workgroup state between launches (stream-K / split-merge tickets, a last arriver's chunk sums)
        takes its buffer from here, so two owners' launches on different streams never share a word -- a
        process-global ticket array touched by two concurrent launches would leave a word non-zero and make
        a later launch merge partials that are not written yet.  Created outside hipGraph capture only."""
        o = getattr(self._tls, "owner", None)
        if o is None:
            o = getattr(self._tls, "misc", None)
            if o is None:
                o = self._tls.misc = {}
        tab = o.setdefault(name, {})
        key = dev.index if dev.index is not None else torch.cuda.current_device()
        t = tab.get(key)
        if t is None:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError(f"{name} scratch must be allocated before hipGraph capture")
            t = tab[key] = make(torch.device("cuda", key))
        return t


WS = _Workspace()


def _launch(x, w, b, out, epi, act, ksplit, sk):
    M, K = x.shape
    N = w.shape[0]
    fl = _ws_floats(M, N, ksplit, sk)
    ws = WS.get(x.device, fl) if fl else None
    cnt = WS.counters(x.device) if sk else None
    call("grag_gemm_tile", ptr(x), ptr(w), ptr(b), ptr(out), x.stride(0), w.stride(0), out.stride(0),
         M, N, K, epi, act, ksplit, sk, ptr(ws), ptr(cnt))
    return out


def gemm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None, act: int = ACT_NONE,
         ksplit: int | None = None, out: torch.Tensor | None = None, sk: int | None = None) -> torch.Tensor:
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
    ksplit, sk = schedule(M, N, K) if ksplit is None else (ksplit, sk or 0)
    if out is None:
        out = torch.empty(M, N, dtype=x.dtype, device=x.device)
    return _launch(x, w, b, out, EPI_STORE, act, ksplit, sk)


def gemm_silu(x: torch.Tensor, w_gu: torch.Tensor, b_gu: torch.Tensor | None = None,
              ksplit: int | None = None, out: torch.Tensor | None = None, sk: int | None = None) -> torch.Tensor:
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
    ksplit, sk = schedule(M, N2, K, True) if ksplit is None else (ksplit, sk or 0)
    if out is None:
        out = torch.empty(M, N2 // 2, dtype=x.dtype, device=x.device)
    return _launch(x, w_gu, b_gu, out, EPI_SILU, ACT_NONE, ksplit, sk)


# ---------------------------------------------------------------- decode regime (csrc/kernels/gemm_decode.hip)
DEC_DEPTH = 4  # K-steps issued ahead by the decode kernel (ring of DEC_DEPTH + 1 LDS / register slots)
_DEC_ON = os.environ.get("GRAG_DECODE_GEMM", "1") != "0"
# (mt, nwv, ntw) compiled: mt 16-row tiles of M, nwv waves per workgroup, ntw 16-row W tiles per wave
DEC_VARIANTS = [(1, 4, 2), (1, 5, 2), (2, 4, 2), (2, 5, 2), (4, 4, 2), (4, 5, 2), (8, 4, 2), (8, 5, 2), (12, 5, 2),
                (12, 8, 2), (16, 4, 2)]
DEC_MAX_M = int(os.environ.get("GRAG_DECODE_MAX_M", "256"))
# batches from this size take the decode kernel on every projection shape (A/B knob); below it dec_small decides
DEC_MIN_M = int(os.environ.get("GRAG_DEC_MIN_M", "33"))


def dec_small(M: int, N: int, K: int, silu: bool = False, deferred: bool = False) -> bool:
    """1-32 rows (the reference's 1-4 live sequences): the 1- / 2-row-tile decode variants where the hipGraph-
    timed cold-weight sweep measured them faster (profiles/gemm_graph_sweep_r5_depths_smallM.json): gate/up
    49-52 us vs the tile kernel's 76-79 (5.2-5.5 TB/s), down_proj (K >= 4 N) 30-31 vs skinny / library
    31-38 us; qkv / o stay on skinny / library (9-12 vs 12-13 us) unless their split-K reduce is ``deferred``
    into RoPE / RMSNorm (ops/linear.linear_deferred): then qkv 9.2-9.5 vs 12 us, o 8.2-8.7 vs 8.4-9.4 us
    (profiles/gemm_graph_sweep_r5_smallM_deferred.json).  Deeper rings (8 / 12) measured slower."""
    if M >= 33 or M < 1:
        return False
    return M >= DEC_MIN_M or silu or K >= 4 * N or deferred


def dec_variants(M: int) -> list[tuple[int, int, int]]:
    """Compiled variants that take an M-row batch, smallest padded row count first."""
    need = -(-M // 16)
    vs = [v for v in DEC_VARIANTS if v[0] >= need]
    if not vs:
        return []
    mt = min(v[0] for v in vs)
    return [v for v in vs if v[0] == mt]


def dec_ksplit(K: int, ksplit: int) -> int:
    """Effective K-splits of a requested count: splits of whole 4-step rounds (the rule the decode plans
    were measured with), then the launcher's own rule (ceil(kt / ks) steps per split) on that count, so the
    fp32 plane count here always equals the kernel's."""
    kt = K // 64
    kts = -(-(kt // 4) // max(1, ksplit)) * 4 if kt >= 4 else kt
    ks = -(-kt // max(1, kts))
    return -(-kt // -(-kt // ks))


def dec_plan(M: int, N: int, K: int, silu: bool = False) -> tuple | None:
    """(mt, nwv, ntw, ksplit[, gs]) for the decode kernel, or None when another path is faster.

    Measured (scripts/bench_gemm_decode.py, cold weights, profiles/gemm_decode_ab_v4.jsonl and
    gemm_decode_ab_v6.jsonl; Qwen2-7B projections, us):
      * <= 128 rows, qkv / o / down: 4 waves, about one workgroup per CU via K-splits (1.2-1.3x the
        256x256 tile kernel); gate/up (1184 wave units): the balanced 5-wave grid, 4-5 units on every CU
        (M = 128: 72.6 vs tile 88.8, library 84.6);
      * 129-192 rows: qkv / o on balanced 5-wave grids, 4 units x 7 K-splits (M = 192: qkv 33.7 vs tile
        39.0, o 32.2 vs 36.0); gate/up balanced (81.9 vs 85.6); down_proj (K = 5.3 N) stays on the tile
        kernel's split-K (58.0 vs 63.4);
      * 193-256 rows: qkv / o on 16-row-tile 4-wave groups x 7 K-splits (M = 256: 36.5 vs 42.7, 34.7 vs
        39.0); gate/up and down_proj stay on the tile kernel (88.3 vs 110, 64.3 vs 68.1)."""
    if not _DEC_ON or M < 1 or M > DEC_MAX_M or K % 256 or N % 32 or (silu and N % 64):
        return None
    ncu = _num_cus()
    if silu and DEC_TAIL:
        return dec_tail_plan(M, N, ncu)
    units = N // 32
    deep = K >= 4 * N  # down_proj-like
    if M <= 128:
        if silu or units >= 4 * ncu:  # FFN-wide: balanced 5-wave grid over every CU, no K-split
            mt = -(-M // 16) if M <= 32 else 4 if M <= 64 else 8
            gs = dec_balanced_gs(N, 2, 5, 1, ncu)
            return None if gs is None else (mt, 5, 2, 1, gs)
        vs = [v for v in dec_variants(M) if v[1] == 4 and N % (16 * v[1] * v[2]) == 0]
        if not vs:
            return None
        mt, nwv, ntw = vs[0]
        tiles = N // (16 * nwv * ntw)
        if tiles >= ncu:
            return None
        return mt, nwv, ntw, dec_ksplit(K, max(1, ncu // tiles))
    if M <= 192:
        if deep:
            return None
        if silu:
            gs = dec_balanced_gs(N, 2, 5, 1, ncu)
            return None if gs is None else (12, 5, 2, 1, gs)
        if units >= 4 * ncu:
            return None
        ks = dec_ksplit(K, max(1, round(ncu / max(1, units / 4))))
        gs = dec_balanced_gs(N, 2, 5, ks, ncu)
        return None if gs is None else (12, 5, 2, ks, gs)
    if silu or deep or units % 4 or units // 4 >= ncu:
        return None
    return 16, 4, 2, dec_ksplit(K, max(1, ncu // (units // 4)))


DEC_TAIL = os.environ.get("GRAG_DEC_TAIL", "0") == "1"


def dec_tail_plan(M: int, N: int, ncu: int | None = None, ksplit: int = 1) -> tuple | None:
    """The 8-wave tail-split schedule (gemm_decode.hip TQ): every workgroup gets 4 or 5 wave units dealt
    evenly over about one workgroup per CU; waves 0-3 own 4 of them, waves 4-7 split the 5th by row tiles.
    (mt, 8, 2, ksplit, gs, 1) or None when the units do not fill 4-5-unit workgroups."""
    ncu = ncu or _num_cus()
    mt = next((m for m in (4, 8, 12, 16) if 16 * m >= M), None)
    if mt is None:
        return None
    units = N // 32
    gs = min(units, max(-(-units // 5), ncu // max(1, ksplit)))
    if -(-units // gs) > 5:
        return None
    return mt, 8, 2, ksplit, gs, 1


def dec_ws_floats(M: int, N: int, ksplit: int) -> int:
    return ksplit * M * N if ksplit > 1 else 0


def dec_unit_rows(N: int, silu: bool, ntw: int = 2) -> torch.Tensor:
    """Weight rows of every decode-kernel wave unit, in unit order ([N] index): 16*ntw consecutive rows, or
    for the interleaved gate/up weight (ntw 2) the 16 gate rows of a 16-column output group then its 16 up
    rows (the kernel's silu unit q: rows 64 (q >> 1) + 16 (q & 1) + [0, 16) and the same + 32)."""
    if not silu:
        return torch.arange(N)
    q = torch.arange(N // 32)
    g0 = (q >> 1) * 64 + (q & 1) * 16
    g = g0[:, None] + torch.arange(16)
    return torch.cat([g, g + 32], 1).reshape(-1)


def dec_pack(w: torch.Tensor, silu: bool = False, ntw: int = 2) -> torch.Tensor:
    """[N, K] weight -> the decode kernel's unit-packed layout [N / (16 ntw), K / 64, 16 ntw, 64]: each wave
    streams one contiguous region instead of 128 B per row per K-step."""
    N, K = w.shape
    r = 16 * ntw
    idx = dec_unit_rows(N, silu, ntw).to(w.device)
    return w[idx].view(N // r, r, K // 64, 64).permute(0, 2, 1, 3).contiguous()


class DecPacked:
    """A weight kept twice: natural [N, K] (prefill GEMMs) and unit-packed for the decode kernel."""

    def __init__(self, w: torch.Tensor, silu: bool = False):
        self.shape = w.shape
        self.silu = silu
        self.data = dec_pack(w, silu)


def gemm_decode(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None, act: int = ACT_NONE,
                epi: int = EPI_STORE, plan: tuple[int, int, int, int] | None = None,
                out: torch.Tensor | None = None, packed: "DecPacked | None" = None) -> torch.Tensor:
    """Decode-regime GEMM: y = act(x @ w.T + b) (epi EPI_STORE) or the SwiGLU product of an interleaved
    gate/up weight (epi EPI_SILU, out [M, N/2]).  ``plan`` = (mt, nwv, ntw, ksplit[, gs]) overrides dec_plan
    (gs: workgroups per K-range over the N / (16 ntw) wave units; 0 = the plain N / (16 ntw nwv) tiling)."""
    M, K = x.shape
    N = w.shape[0]
    if not x.is_cuda:
        return gemm_silu(x, w, b) if epi == EPI_SILU else gemm(x, w, b, act)
    mt, nwv, ntw, ks, *rest = plan or dec_plan(M, N, K, epi == EPI_SILU)
    gs = rest[0] if rest else 0
    tail = rest[1] if len(rest) > 1 else 0
    ks = dec_ksplit(K, ks)
    if out is None:
        out = torch.empty(M, N // 2 if epi == EPI_SILU else N, dtype=x.dtype, device=x.device)
    fl = dec_ws_floats(M, N, ks)
    ws = WS.get(x.device, fl) if fl else None
    wsrc = w if packed is None else packed.data
    call("grag_gemm_decode_t", ptr(x), ptr(wsrc), ptr(b), ptr(out), x.stride(0), w.stride(0), out.stride(0),
         M, N, K, epi, act, mt, nwv, ntw, ks, gs, 0 if packed is None else 2 if packed.silu else 1, tail, ptr(ws))
    return out


# the split-K RMSNorm folded into the gate/up projection that consumes it at 1-4 rows (grag_gemm_decode_norm).
# Off by default: measured slower (profiles/norm_fold_ab_r6.json, same box): every workgroup re-reduces the
# o_proj planes in its prologue while only D = 4 K-steps of W are in flight, so the W stream -- the kernel's
# bound -- starts ~6.4 us late, more than the 5.6 us norm launch it replaces (B = 1 TPOT 3.83 vs 3.81 ms, B = 4
# 4.10 vs 3.90).  GRAG_NORM_FUSE=1 turns it on (A/B, tests/test_norm_fuse_gpu.py)
NORM_FUSE = os.environ.get("GRAG_NORM_FUSE", "0") == "1"


def norm_fuse_plan(M: int, N: int, K: int, silu: bool) -> tuple[int, int] | None:
    """(nwv, gs) when grag_gemm_decode_norm takes the consumer projection of a deferred norm: the decode plan
    of (M, N, K) is a one-tile (mt 1), one-K-range plan on the 4- / 5-wave grid and the rows fit its LDS
    image; else None."""
    if not NORM_FUSE or M < 1 or M > 4 or M * (K * 2 + 64) > 65536:
        return None
    p = dec_plan(M, N, K, silu)
    if p is None:
        return None
    mt, nwv, ntw, ks, *rest = p
    gs = rest[0] if rest else 0
    tail = rest[1] if len(rest) > 1 else 0
    if mt != 1 or ntw != 2 or nwv not in (4, 5) or tail or dec_ksplit(K, ks) != 1:
        return None
    return nwv, gs


def gemm_decode_norm(part: "SplitKPartial", res_in: torch.Tensor, res_out: torch.Tensor, w_norm: torch.Tensor,
                     eps: float, w: torch.Tensor, epi: int, plan: tuple[int, int]) -> torch.Tensor:
    """epilogue(RMSNorm(res_in + reduce(part)) * w_norm @ w.T) in one launch (csrc/kernels/gemm_decode.hip NRM
    kernel); res_out receives the new residual stream (res_in + reduce(part), bf16).  ``plan`` from
    norm_fuse_plan.  Out [M, N/2] for EPI_SILU (interleaved gate/up weight), [M, N] for EPI_STORE."""
    M, K, N = part.M, part.N, w.shape[0]
    nwv, gs = plan
    out = torch.empty(M, N // 2 if epi == EPI_SILU else N, dtype=res_in.dtype, device=res_in.device)
    call("grag_gemm_decode_norm", ptr(part.planes), part.S, ptr(res_in), ptr(res_out), ptr(w_norm), float(eps),
         ptr(w), ptr(out), w.stride(0), out.stride(0), M, N, K, epi, 1, nwv, 2, gs, 0)
    return out


class SplitKPartial:
    """The fp32 split-K planes [S, M, N] of a projection whose reduce was deferred to its consumer
    (ops/norm.py rmsnorm: split-K reduce + residual add + RMSNorm in one kernel).  The planes live in the
    thread's split-K workspace: the consumer must be the next launch that touches it on this stream."""

    __slots__ = ("planes", "S", "M", "N", "dtype", "device")

    def __init__(self, planes: torch.Tensor, S: int, M: int, N: int, dtype):
        self.planes, self.S, self.M, self.N, self.dtype = planes, S, M, N, dtype
        self.device = planes.device

    @property
    def shape(self):
        return (self.M, self.N)

    def materialize(self) -> torch.Tensor:
        return self.planes.view(self.S, self.M, self.N).sum(0).to(self.dtype)


def deferred_plan(M: int, N: int, K: int) -> tuple[str, int, tuple] | None:
    """("decode" | "tile", effective K-splits, plan) when ops/linear.py linear() would run this bias-free
    bf16 projection as a K-split on an owned kernel (its splitk_reduce is then deferrable); else None."""
    p = dec_plan(M, N, K)
    if p is not None:
        ks = dec_ksplit(K, p[3])
        return ("decode", ks, p) if ks > 1 else None
    from .linear import use_tile  # noqa: PLC0415 (linear imports this module)

    if use_tile(M, N, K):
        ks, sk = schedule(M, N, K)
        return ("tile", ks, (ks, sk)) if ks > 1 and not sk else None
    if M >= PREFILL_MIN_M:  # 257-512-row decode batches run the measured prefill plans (K-split tile kernel)
        p = prefill_plan(M, N, K)
        if p is not None and p[0] > 1 and not p[1]:
            return "tile", p[0], p
    return None


# The decoder's split-K RMSNorm folded into its producer and consumer projections at 1-4 rows
# (csrc/kernels/gemm_decode.hip RED / NRM 2): the last split of each unit group of the producer (o_proj, down)
# adds the planes into the residual stream and leaves per-group sums of squares; the consumer (gate/up, the
# next layer's qkv) reads the residual stream as A, scales it by the norm weight on the fly and its
# accumulators by 1 / rms.  The norm launch between them goes away -- but measured slower (profiles/
# norm_fold_ab_r6.json: B = 1 TPOT 4.03 / 3.99 vs 3.82 / 3.82 ms): each producer's split tickets with their
# agent-scope release / acquire fences and the last split's reduce cost ~7 us, more than the 5.6 us launch.
# Off by default; GRAG_FOLD_NORM=1 for A/B (tests/test_norm_fuse_gpu.py keeps both halves tested).
FOLD_NORM = os.environ.get("GRAG_FOLD_NORM", "0") == "1"


def fold_plan(M: int, N: int, K: int, silu: bool) -> tuple[int, int, int] | None:
    """(nwv, effective K-splits, gs) when the 1-4-row decode plan of (M, N, K) is one the folded-norm kernels
    compile (one 16-row tile, 4- / 5-wave grid, no tail split); else None."""
    if not FOLD_NORM or M < 1 or M > 4:
        return None
    p = dec_plan(M, N, K, silu)
    if p is None:
        return None
    mt, nwv, ntw, ks, *rest = p
    gs = rest[0] if rest else 0
    tail = rest[1] if len(rest) > 1 else 0
    if mt != 1 or ntw != 2 or nwv not in (4, 5) or tail:
        return None
    return nwv, dec_ksplit(K, ks), gs


class FoldedNorm:
    """The residual stream [M, H] after a producer projection's folded reduce (updated in place), with the
    per-group sums of squares [groups, 4] its consumer takes 1 / rms from."""

    __slots__ = ("residual", "ss", "groups")

    def __init__(self, residual: torch.Tensor, ss: torch.Tensor, groups: int):
        self.residual, self.ss, self.groups = residual, ss, groups


def fold_ws(dev: torch.device) -> tuple[torch.Tensor, torch.Tensor]:
    """(tickets [2 x 1024] int32, zeroed; sums of squares [2 x 1024 x 4] fp32): two slots (post-attention,
    input norm), owned by the caller's workspace owner (WS.scratch); allocate before any capture."""
    return WS.scratch("fold_norm", torch.device(dev),
                      lambda d: (torch.zeros(2 * 1024, dtype=torch.int32, device=d),
                                 torch.zeros(2 * 1024 * 4, dtype=torch.float32, device=d)))


def gemm_decode_red(x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor, slot: int) -> FoldedNorm | None:
    """The producer half: residual += x @ w.T (bf16, in place) through the split-K decode kernel whose last
    split per unit group does the add; None when the plan does not take it (the caller falls back)."""
    M, K = x.shape
    N = w.shape[0]
    plan = fold_plan(M, N, K, False)
    if plan is None or plan[1] < 2 or residual.shape != (M, N) or not residual.is_contiguous():
        return None
    nwv, ks, gs = plan
    fl = dec_ws_floats(M, N, ks)
    if torch.cuda.is_current_stream_capturing() and not WS.ready(x.device, fl):
        return None
    ws = WS.get(x.device, fl)
    cnt, ss = fold_ws(x.device)
    groups = gs if gs > 0 else (N // 32) // nwv
    ssb = ss[slot * 4096:(slot + 1) * 4096]
    call("grag_gemm_decode_red", ptr(x), ptr(w), ptr(residual), ptr(ssb), ptr(cnt[slot * 1024:(slot + 1) * 1024]),
         x.stride(0), w.stride(0), M, N, K, 1, nwv, 2, ks, gs, ptr(ws), None)
    return FoldedNorm(residual, ssb, groups)


def gemm_decode_scaled(fold: FoldedNorm, w_norm: torch.Tensor, eps: float, w: torch.Tensor, epi: int):
    """The consumer half: epilogue(RMSNorm(residual) * w_norm @ w.T) with the norm folded in -- [M, N/2] for
    EPI_SILU (interleaved gate/up), SplitKPartial planes for EPI_PARTIAL (the RoPE pass reduces them); None
    when the plan does not take it."""
    x = fold.residual
    M, K = x.shape
    N = w.shape[0]
    plan = fold_plan(M, N, K, epi == EPI_SILU)
    if plan is None:
        return None
    nwv, ks, gs = plan
    if (epi == EPI_SILU) != (ks == 1):
        return None
    if epi == EPI_SILU:
        out = torch.empty(M, N // 2, dtype=x.dtype, device=x.device)
        call("grag_gemm_decode_scaled", ptr(x), ptr(w_norm), ptr(fold.ss), fold.groups, float(eps), ptr(w), ptr(out),
             x.stride(0), w.stride(0), out.stride(0), M, N, K, EPI_SILU, 1, nwv, 2, ks, gs, None)
        return out
    fl = dec_ws_floats(M, N, ks)
    if torch.cuda.is_current_stream_capturing() and not WS.ready(x.device, fl):
        return None
    ws = WS.get(x.device, fl)
    call("grag_gemm_decode_scaled", ptr(x), ptr(w_norm), ptr(fold.ss), fold.groups, float(eps), ptr(w), None,
         x.stride(0), w.stride(0), N, M, N, K, EPI_PARTIAL, 1, nwv, 2, ks, gs, ptr(ws))
    return SplitKPartial(ws[:fl], ks, M, N, x.dtype)


def gemm_deferred(x: torch.Tensor, w: torch.Tensor, how: tuple[str, int, tuple]) -> SplitKPartial:
    """Run a K-split projection (deferred_plan) and leave its fp32 planes in the workspace (epi
    EPI_PARTIAL: no splitk_reduce launch)."""
    M, K = x.shape
    N = w.shape[0]
    kind, ks, p = how
    fl = ks * M * N
    ws = WS.get(x.device, fl)
    if kind == "decode":
        mt, nwv, ntw, ksp, *rest = p
        # the launcher gets the EFFECTIVE split count the planes were sized for (dec_ksplit of the plan's
        # request): a raw request the 4-step rounding lowers (K = 3584, 28 -> 14) would write past the slab
        ks = dec_ksplit(K, ksp)
        fl = ks * M * N
        ws = WS.get(x.device, fl)
        call("grag_gemm_decode_t", ptr(x), ptr(w), ptr(None), ptr(None), x.stride(0), w.stride(0), N,
             M, N, K, EPI_PARTIAL, ACT_NONE, mt, nwv, ntw, ks, rest[0] if rest else 0, 0,
             rest[1] if len(rest) > 1 else 0, ptr(ws))
    else:
        call("grag_gemm_tile", ptr(x), ptr(w), ptr(None), ptr(None), x.stride(0), w.stride(0), N,
             M, N, K, EPI_PARTIAL, ACT_NONE, ks, 0, ptr(ws), ptr(None))
    return SplitKPartial(ws[:fl], ks, M, N, x.dtype)


def dec_balanced_gs(N: int, ntw: int, nwv: int, ksplit: int, ncu: int | None = None) -> int | None:
    """Workgroups per K-range that put about one workgroup on every CU with at most ``nwv`` wave units each
    (None when the units do not fill ``nwv``-wave groups even at one workgroup per CU)."""
    units = N // (16 * ntw)
    ncu = ncu or _num_cus()
    gs = max(-(-units // nwv), ncu // max(1, ksplit))
    return min(gs, units) if -(-units // min(gs, units)) <= nwv else None


def dec_capture_ok(dev: torch.device, M: int, N: int, K: int, silu: bool = False) -> bool:
    p = dec_plan(M, N, K, silu)
    if p is None:
        return False
    fl = dec_ws_floats(M, N, dec_ksplit(K, p[3]))
    return fl == 0 or not torch.cuda.is_current_stream_capturing() or WS.ready(dev, fl)


def capture_ok(dev: torch.device, M: int, N: int, K: int, silu: bool = False) -> bool:
    """False only inside a hipGraph capture whose split-K slab was not sized by an eager step."""
    ks, sk = schedule(M, N, K, silu)
    fl = _ws_floats(M, N, ks, sk)
    return fl == 0 or not torch.cuda.is_current_stream_capturing() or (WS.ready(dev, fl) and (
        not sk or WS.has_counters(dev)))


def mlp_gate_up(x: torch.Tensor, w_gu: torch.Tensor, b_gu: torch.Tensor | None = None) -> torch.Tensor:
    """SwiGLU input half for an interleaved gate/up weight: the fused tile
    kernel when it takes the shape, else library GEMM + reshape (same math)."""
    M, K = x.shape
    if x.is_cuda and (M >= 33 or dec_small(M, w_gu.shape[0], K, True)) and supported(x, w_gu) and dec_plan(M, w_gu.shape[0], K, True) is not None \
            and dec_capture_ok(x.device, M, w_gu.shape[0], K, True):
        return gemm_decode(x, w_gu, b_gu, epi=EPI_SILU)
    if not x.is_cuda or (supported(x, w_gu) and capture_ok(x.device, M, w_gu.shape[0], K, True)):
        return gemm_silu(x, w_gu, b_gu)
    y = torch.nn.functional.linear(x, w_gu, b_gu).view(M, -1, 2, 32)
    return (torch.nn.functional.silu(y[:, :, 0].float()) * y[:, :, 1].float()).to(x.dtype).reshape(M, -1)
