"""Linear layers.

Decode-sized inputs (the weight-streaming regime: every weight byte read once
per step) go to hand-written MFMA kernels, chosen per shape from the cold-cache
A/B in scripts/bench_gemm.py:
* ``grag_gemm_skinny`` (M <= 16, and square projections up to M = 64):
  register-streamed W, nontemporal loads, intra-workgroup split-K;
* ``grag_gemm_stream`` (deep-K projections such as down_proj, and the LM head
  at M <= 32): stream-K over (tile, 64-k) iterations, full-line LDS-DMA ring,
  in-launch split-tile combine;
* ``grag_gemm_decode`` (ops/gemm.py, W streamed HBM -> registers 3 K-steps
  deep, A through an LDS-DMA ring) for 32 < M <= 128 on projections narrower
  than one 128-column tile per CU (qkv, o, down): 1.05-1.3x the tile kernel
  (profiles/gemm_decode_ab_v4.jsonl);
* ``grag_gemm_tile`` (ops/gemm.py, 256x256 MFMA tiles + split-K slabs) for the
  other decode batches 32 < M <= 256: 1.1-1.5x the library on every Qwen2-7B
  projection (profiles/gemm_tile_ab_v1.jsonl);
* larger M (prefill, encoder batches): the owned tile kernel wherever the
  dense M sweep of scripts/sweep_prefill_gemm.py measured it faster
  (``gemm.prefill_plan``; e.g. Qwen2-7B down_proj at the bench's ~7.1K-row
  prefill steps: 771 vs 1131 us), else hipBLASLt through
  ``torch.nn.functional.linear`` — the library is used only for plain
  (epilogue-free / bias-only) GEMMs; everything fused around them
  (bias+RoPE+KV store, SiLU*mul, bias+GELU, bias+residual+LayerNorm,
  residual+RMSNorm, pooling) is a hand-written HIP kernel in ops/*.
"""
from __future__ import annotations

import bisect
import json
import os
from pathlib import Path

import torch

from . import gemm as _tile
from ._lib import call, lib, ptr

TUNING_DIR = Path(__file__).resolve().parents[1] / "tuning"
_TUNED = {"done": False, "table": None}


def enable_tuned_gemms() -> bool:
    """Load the measured library-GEMM solutions (PyTorch TunableOp results,
    A/B-filtered by scripts/ab_tuned_gemms.py: only solutions that beat
    hipBLASLt's default heuristic by >= 3 % on cold weights) READ-ONLY —
    tuning never runs inside a timed or graph-captured region — and the
    measured decode dispatch table (scripts/gemm_dispatch_table.py).
    GRAG_TUNED_GEMMS=0 disables both."""
    if _TUNED["done"]:
        return _TUNED["table"] is not None
    _TUNED["done"] = True
    if os.environ.get("GRAG_TUNED_GEMMS", "1") == "0":
        return False
    js = TUNING_DIR / "gemm_dispatch_gfx950.json"  # plain data: loaded on the host too (dispatch tests)
    if js.exists():
        raw = json.loads(js.read_text())["table"]
        _TUNED["table"] = {tuple(map(int, k.split(","))): ([m for m, _ in v], [b for _, b in v])
                           for k, v in raw.items()}
    if not torch.cuda.is_available():
        return _TUNED["table"] is not None
    csv = TUNING_DIR / "tunableop_gfx950.csv"
    try:
        if csv.exists():
            torch.cuda.tunable.enable(True)
            torch.cuda.tunable.tuning_enable(False)
            torch.cuda.tunable.record_untuned_enable(False)
            torch.cuda.tunable.read_file(str(csv))
    except Exception:  # validator mismatch (other ROCm/hipBLASLt build): library defaults
        torch.cuda.tunable.enable(False)
    return _TUNED["table"] is not None


def measured_choice(M: int, N: int, K: int) -> str | None:
    """Fastest measured kernel for this decode shape ('library', 'skinny',
    'stream'), looked up at the smallest measured bucket >= M."""
    t = _TUNED["table"]
    if not t:
        return None
    row = t.get((N, K))
    if row is None:
        return None
    ms, best = row
    i = bisect.bisect_left(ms, M)
    return best[i] if i < len(ms) else None

SKINNY_MAX_M = int(os.environ.get("GRAG_SKINNY_MAX_M", "64"))
_SKINNY_ON = os.environ.get("GRAG_SKINNY", "1") != "0"


def gemm_skinny(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None, nt: int = 0) -> torch.Tensor:
    M, K = x.shape
    N = w.shape[0]
    out = torch.empty(M, N, dtype=x.dtype, device=x.device)
    call("grag_gemm_skinny", ptr(x), ptr(w), ptr(b), ptr(out), x.stride(0), w.stride(0), out.stride(0), M, N, K, nt)
    return out


class _StreamWorkspace:
    """Per-device split-K scratch for ``grag_gemm_stream``: an fp32 slab and a
    zero-initialised ticket-counter array (the kernel's last arriver resets
    its word, so replays inside a hipGraph need no memset).  Grown only
    outside graph capture; GEMMs on one stream reuse it in stream order."""

    def __init__(self):
        self._retired = []  # outgrown slabs stay alive: captured hipGraphs may still point at them

    # the workspace owner's (ops/gemm.py WS.owned_by: an engine's, an embedder's) or this thread's own: a
    # decode graph's LM head or an encoder graph's FFN must never share a slab or a ticket word with another
    # owner's launches on another stream (a process-wide fallback did, for every ownerless thread)
    @staticmethod
    def _home() -> dict:
        t = _tile.WS._tls
        o = getattr(t, "owner", None)
        if o is None:
            o = getattr(t, "misc", None)
            if o is None:
                o = t.misc = {}
        return o

    @property
    def slab(self) -> dict:
        return self._home().setdefault("stream_slab", {})

    @property
    def counters(self) -> dict:
        return self._home().setdefault("stream_cnt", {})

    def ready(self, dev: torch.device, M: int, N: int, K: int) -> bool:
        """True when a graph capture can use the stream kernel for this shape
        (workspace already large enough: capture cannot allocate)."""
        mt, bn, G, pmax = stream_plan(M, N, K)
        need = -(-N // bn) * -(-M // (16 * mt)) * pmax * 16 * mt * bn
        s = self.slab.get(dev.index)
        return s is not None and s.numel() >= need and dev.index in self.counters

    def get(self, dev: torch.device, slab_floats: int):
        key = dev.index
        s = self.slab.get(key)
        if s is None or s.numel() < slab_floats:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("gemm_stream workspace must be sized before hipGraph capture")
            if s is not None:
                self._retired.append(s)
            s = torch.empty(max(slab_floats, 1 << 20), dtype=torch.float32, device=dev)
            self.slab[key] = s
        c = self.counters.get(key)
        if c is None:
            c = torch.zeros(1 << 16, dtype=torch.int32, device=dev)
            self.counters[key] = c
        return s, c


_WS = _StreamWorkspace()
_PLAN_CACHE: dict = {}
_NCU: list = []
STREAM_MAX_M = int(os.environ.get("GRAG_STREAM_MAX_M", "64"))


def num_cus() -> int:
    if not _NCU:
        _NCU.append(torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
                    if torch.cuda.is_available() else 256)
    return _NCU[0]


def stream_plan(M: int, N: int, K: int, mt: int | None = None, bn: int | None = None,
                grid: int | None = None) -> tuple[int, int, int, int]:
    """(mt, bn, grid, pmax) of the stream-K split (same rule as the library's
    ``grag_gemm_stream_plan``): one 4-wave workgroup per CU by default, every
    workgroup a contiguous range of (tile, 64-k step) iterations; pmax = max
    workgroups sharing one output tile (slab slots per tile)."""
    key = (M, N, K, mt, bn, grid)
    p = _PLAN_CACHE.get(key)
    if p is None:
        mt = mt or (2 if M <= 32 else (4 if M <= 64 else 8))
        bn = bn or 128
        ntm = -(-M // (16 * mt))
        ks = -(-K // 64)
        total = -(-N // bn) * ntm * ks
        G = grid or num_cus()
        if total < G * 4:
            G = max(1, -(-total // 4))
        per = total // G
        pmax = -(-ks // per) + 1
        p = _PLAN_CACHE[key] = (mt, bn, G, pmax)
    return p


def gemm_stream(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None,
                plan: tuple | None = None) -> torch.Tensor:
    """Stream-K weight-streaming MFMA GEMM (csrc/kernels/gemm_stream.hip) for
    decode-batch M: y = x @ w.T (+ b).  ``plan`` = (mt, bn, grid) overrides."""
    M, K = x.shape
    N = w.shape[0]
    mt, bn, G, pmax = stream_plan(M, N, K, *(plan or ()))
    ntiles = -(-N // bn) * -(-M // (16 * mt))
    slab, cnt = _WS.get(x.device, ntiles * pmax * 16 * mt * bn)
    if ntiles > cnt.numel():
        raise ValueError(f"gemm_stream: {ntiles} tiles exceed the counter array")
    out = torch.empty(M, N, dtype=x.dtype, device=x.device)
    call("grag_gemm_stream", ptr(x), ptr(w), ptr(b), ptr(out), x.stride(0), w.stride(0), out.stride(0), M, N, K,
         mt, bn, G, pmax, ptr(slab), ptr(cnt))
    return out


def use_skinny(M: int, N: int, K: int) -> bool:
    """Dispatch rule from the cold-cache A/B of scripts/bench_gemm.py
    (profiles/bench_gemm_decode.json): the register-streaming kernel wins at
    M <= 16 except for very wide outputs (gate_up: N >= 8K, N >= 8K), and at
    M <= 64 for square projections (o_proj)."""
    if M <= 16:
        return not (N >= 8192 and K <= 4096 and N >= 8 * K)
    if M <= SKINNY_MAX_M:
        return N <= 4096 and K <= 4096 and N < 4096 + 512
    return False


def use_stream(M: int, N: int, K: int) -> bool:
    """Stream-K LDS-DMA kernel: deep-K projections (down_proj K = 18944: 52 us
    vs hipBLASLt 90 us at M = 64) and, at M <= 32, the vocab-wide LM head."""
    if M > 128:
        return False
    if K >= 2 * N and K >= 4096:
        return True
    return M <= 32 and N >= 65536


_SPLITK_ON = os.environ.get("GRAG_SPLITK", "1") != "0"
SPLITK_S = 8


def splitk_parts(M: int, N: int, K: int) -> int:
    """K-slices for the split-K library path (0 = not taken).  Deep-K
    projections (down_proj: K = 18944 = 5.3 N) at decode batches: hipBLASLt
    has only N/tile x M/tile output tiles (~56 workgroups for 256 CUs) and no
    split-K solution in the tuned table.  Cold-weight hipGraph timings
    (round-1 microbench, profiles/splitk_decode_gemm.jsonl), down_proj
    N=3584: 8 slices at M=160 105.7 -> 62.7 us, 192 75.9 -> 66.3, 224 117.4 ->
    70.0, 256 77.0 -> 56.7; 2 slices at M=96 63.5 -> 52.4, M=64 46.5 -> 43.0.
    At M=128 and for o/qkv/gate_up the library wins.  Decode batch range only,
    and only the measured shape family (Qwen down_proj, K >= 8192): encoder
    FFN2 / GPT-2 MLPs / prefill stay on the library."""
    if not _SPLITK_ON or K < 8192 or K < 4 * N:
        return 0
    if 128 < M <= 256 and K % (8 * 64) == 0:
        return 8
    if 32 < M <= 96 and (N, K) == (3584, 18944):  # measured only on Qwen2-7B down_proj
        return 2
    return 0


TILE_MIN_M = int(os.environ.get("GRAG_TILE_MIN_M", "33"))
TILE_MAX_M = int(os.environ.get("GRAG_TILE_MAX_M", "256"))


def use_tile(M: int, N: int, K: int) -> bool:
    """Owned tile GEMM at decode batches (measured range 64..256: every
    Qwen2-7B projection 1.1-1.5x the library); the vocab-wide LM head and
    prefill-sized M stay on the measured paths below."""
    return TILE_MIN_M <= M <= TILE_MAX_M and N <= 65536 and K >= 512


def use_splitk(M: int, N: int, K: int) -> bool:
    return splitk_parts(M, N, K) > 0


def gemm_splitk(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None, parts: int = SPLITK_S) -> torch.Tensor:
    """Split-K over the library: S strided-batched GEMMs of K/S slices (one
    hipBLASLt launch, S x more workgroups) with fp32 output, reduced in fp32
    — no weight copy (the slices are strided views of ``w``)."""
    M, K = x.shape
    N = w.shape[0]
    S = parts
    xs = x.view(M, S, K // S).transpose(0, 1)
    ws = w.view(N, S, K // S).transpose(0, 1).transpose(1, 2)
    y = torch.bmm(xs, ws, out_dtype=torch.float32).sum(0)
    if b is not None:
        y += b.float()
    return y.to(x.dtype)


def kernel_for(M: int, N: int, K: int, tile_ok: bool = True, dev: torch.device | None = None) -> str:
    """The kernel linear() runs a bf16 [M, K] x [N, K]^T projection on: "decode" / "tile" / "tile_prefill"
    (owned MFMA kernels of ops/gemm.py), "skinny" / "stream" (owned weight-streaming kernels here),
    "splitk" (K-sliced library bmm) or "library" (hipBLASLt).  ``tile_ok``: the operands meet
    ops/gemm.supported (alignment, K % 64).  ``dev``: check that a hipGraph capture in progress can use
    the split-K / stream-K workspaces (None: plan as in steady state, workspaces ready)."""
    capturing = dev is not None and torch.cuda.is_current_stream_capturing()
    if tile_ok:
        if (TILE_MIN_M <= M or _tile.dec_small(M, N, K)) and _tile.dec_plan(M, N, K) is not None and (
                dev is None or _tile.dec_capture_ok(dev, M, N, K)):
            return "decode"
        if use_tile(M, N, K) and (dev is None or _tile.capture_ok(dev, M, N, K)):
            return "tile"
        if M >= _tile.PREFILL_MIN_M and _tile.prefill_plan(M, N, K) is not None and (
                dev is None or _tile.capture_ok(dev, M, N, K)):
            return "tile_prefill"
    if splitk_parts(M, N, K):
        return "splitk"
    stream_ready = not capturing or _WS.ready(dev, M, N, K)
    choice = measured_choice(M, N, K)
    if choice == "library":
        return "library"
    if choice == "skinny" and K % 64 == 0:
        return "skinny"
    if choice == "stream" and K % 16 == 0 and N % 4 == 0 and stream_ready:
        return "stream"
    if K % 64 == 0 and use_skinny(M, N, K):
        return "skinny"
    if K % 16 == 0 and N % 4 == 0 and use_stream(M, N, K) and stream_ready:
        return "stream"
    return "library"


OWNED_KINDS = ("decode", "tile", "tile_prefill", "skinny", "stream")


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None) -> torch.Tensor:
    """y = x @ w.T (+ b); w is [out, in] (K-contiguous, TN GEMM)."""
    if not x.is_cuda:
        if x.dtype == torch.bfloat16:
            y = torch.nn.functional.linear(x.float(), w.float(), None if b is None else b.float())
            return y.to(x.dtype)
        return torch.nn.functional.linear(x, w, b)
    if not _TUNED["done"]:
        enable_tuned_gemms()
    if (_SKINNY_ON and x.dim() == 2 and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and x.stride(1) == 1 and w.stride(1) == 1):
        M, K = x.shape
        N = w.shape[0]
        kind = kernel_for(M, N, K, _tile.supported(x, w), x.device)
        if kind == "decode":
            return _tile.gemm_decode(x, w, b)
        if kind == "tile":
            return _tile.gemm(x, w, b)
        if kind == "tile_prefill":
            p = _tile.prefill_plan(M, N, K)
            return _tile.gemm(x, w, b, ksplit=p[0], sk=p[1])
        if kind == "splitk":
            return gemm_splitk(x, w, b, splitk_parts(M, N, K))
        if kind == "skinny":
            return gemm_skinny(x, w, b)
        if kind == "stream":
            return gemm_stream(x, w, b)
    return torch.nn.functional.linear(x, w, b)


def linear_deferred(x: torch.Tensor, w: torch.Tensor):
    """linear(x, w) for a bias-free projection whose output only feeds the decoder's residual add +
    RMSNorm: when linear() would run it as a K-split on an owned kernel, the fp32 planes are returned
    unreduced (ops/gemm.py SplitKPartial) and rmsnorm() folds the reduce into its pass; otherwise the
    plain bf16 result.  Same dispatch predicates as linear()."""
    if (x.is_cuda and _SKINNY_ON and _DEFER_ON and x.dim() == 2 and x.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16 and x.stride(1) == 1 and w.stride(1) == 1 and _tile.supported(x, w)):
        M, K = x.shape
        N = w.shape[0]
        if M >= TILE_MIN_M or _tile.dec_small(M, N, K, deferred=True):
            how = _tile.deferred_plan(M, N, K)
            if how is not None and (not torch.cuda.is_current_stream_capturing()
                                    or _tile.WS.ready(x.device, how[1] * M * N)):
                return _tile.gemm_deferred(x, w, how)
    return linear(x, w)


_DEFER_ON = os.environ.get("GRAG_DEFER_SPLITK", "1") != "0"
