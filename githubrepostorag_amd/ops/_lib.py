"""ctypes binding of ``libgrag_kernels.so`` (the gfx950 HIP kernel library).

The library is loaded lazily, always *after* ``import torch`` so it shares
PyTorch-ROCm's HIP runtime (same ``libamdhip64.so.7`` SONAME).  On a GPU box a
missing or unloadable library is a hard error — ops never fall back silently
to PyTorch on device tensors.  CPU tensors use the fp32 reference
implementations in the individual op modules (that is what the CPU test tier
exercises).
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path

import torch

_LIB_PATH = Path(__file__).resolve().parents[1] / "_lib" / "libgrag_kernels.so"
_lock = threading.RLock()
_lib = None

P = ctypes.c_void_p
I = ctypes.c_int
I64 = ctypes.c_int64
U64 = ctypes.c_uint64
F = ctypes.c_float

_SIGS = {
    "grag_rmsnorm": [P, P, P, P, I, I, F, P],
    "grag_splitk_add_rmsnorm": [P, I, P, P, P, I, I, F, P],
    "grag_layernorm": [P, P, P, P, P, P, I, I, F, P],
    "grag_add_layernorm": [P, P, P, P, P, P, I, I, F, P],
    "grag_bert_embed_ln": [P, P, P, P, P, P, P, P, P, I, I, I, I, F, P],
    "grag_embed_gather": [P, P, P, I, I, I, P],
    "grag_qkv_rope_kvstore": [P, I, P, P, P, P, P, P, P, I, I, I, I, I, I, I, P],
    "grag_qkv_rope_kvstore_planes": [P, I, I, P, P, P, P, P, P, P, I, I, I, I, I, I, I, P],
    "grag_silu_mul": [P, P, I, I, P],
    "grag_bias_act": [P, P, P, I, I, I, P],
    "grag_pool_l2norm": [P, P, P, P, P, I, I, I, I, I, P],
    "grag_paged_attention": [P, I, P, P, P, I, P, I, P, P, I, I, I, I, I, I, I, F, I, I, I, P, P, I, I, P],
    "grag_splitk_add_rmsnorm_small": [P, I, P, P, P, I, I, F, P, P, P],
    "grag_paged_decode_mw": [P, I, P, P, P, I, P, I, P, P, I, I, I, I, I, I, F, I, I, P, P, P, I, I, P],
    "grag_paged_decode_mw_rope": [P, I, P, P, P, P, P, P, P, I, P, I, P, P, I, I, I, I, I, I, F, I, I, P, P, P, I, I, I,
                                  I, P],
    "grag_gemm_decode_red": [P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, P, P, P],
    "grag_gemm_decode_scaled": [P, P, P, I, F, P, P, I, I, I, I, I, I, I, I, I, I, I, I, P, P],
    "grag_gemm_decode_norm": [P, I, P, P, P, F, P, P, I, I, I, I, I, I, I, I, I, I, I, P],
    "grag_paged_decode_cascade": [P, I, P, P, P, I, P, I, P, P, I, I, I, I, I, I, F, I, I, P, P, I, I, P, P, P, I, I,
                                  P, P, I, P],
    "grag_varlen_attention": [P, P, P, I, P, I, P, P, I, I, I, I, I, F, I, P],
    "grag_score_topk_flat": [P, I64, I64, I64, I, P, I, I, I, I, P, P, P, I, P, P, P, I, P, P, P, P, P],
    "grag_score_topk_work": [P, I, P, I, I, I, I, P, P, I, P, P, P, I, P, P, P, I, P, P, P, P, P],
    "grag_topk_num_waves": [],
    "grag_sample": [P, I, I, I, I, P, P, P, P, P, I, P, U64, P, P, P, I, P],
    "grag_sample_tp": [I, P, I, I, I, I, I, I, P, P, P, P, P, I, P, U64, P, P, P, I, I, I, P, P, P, P, P, I, P],
    "grag_sample_segments": [I],
    "grag_sample_ws_floats": [I, I],
    "grag_mark_seen": [P, P, I, P, I, I, P],
    "grag_gemm_skinny": [P, P, P, P, I, I, I, I, I, I, I, P],
    "grag_gemm_stream": [P, P, P, P, I, I, I, I, I, I, I, I, I, I, P, P, P],
    "grag_gemm_stream_plan": [I, I, I, I, P],
    "grag_awq_dequant": [P, P, P, P, I, I, I, P],
    "grag_ivf_plan": [P, I, I, P, I, P, P, P, P],
    "grag_ivf_plan_max_pairs": [],
    "grag_topk_merge": [P, P, I, P, I, I, I, I, P, P, I, I, I, P, P, P],
    "grag_topk_merge_cap": [],
    "grag_bitmap_update": [P, P, I, I, P],
    "grag_gemm_tile": [P, P, P, P, I, I, I, I, I, I, I, I, I, I, P, P, P],
    "grag_splitk_reduce": [P, P, P, I, I, I, I, I, I, P],
    "grag_gemm_tile_mfma": [I],
    "grag_gemm_tile_sched": [I],
    "grag_gemm_decode": [P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, I, I, P, P],
    "grag_gemm_decode_has": [I, I, I],
    "grag_gemm_decode_t": [P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, I, I, I, P, P],
    "grag_gemm_decode_has_t": [I, I, I, I],
    "grag_gemm_decode_stamps": [P],
    "grag_gemm_decode_depth": [I],
    "grag_gemm_w4": [P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, P, P],
    "grag_gemm_w4_has": [I, I],
    "grag_err_alloc": [P],
    "grag_attn_decode_xcd": [I],
}


def lib_path() -> Path:
    return _LIB_PATH


def available() -> bool:
    return _LIB_PATH.exists()


def lib():
    """Return the loaded kernel library (building it if hipcc is present)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not _LIB_PATH.exists() or os.environ.get("GRAG_REBUILD") == "1":
            from ..utils.native_build import build_kernels

            build_kernels()
        handle = ctypes.CDLL(str(_LIB_PATH), mode=ctypes.RTLD_GLOBAL)
        for name, args in _SIGS.items():
            fn = getattr(handle, name, None)
            if fn is None:
                continue
            fn.argtypes = args
            fn.restype = (ctypes.c_long if name.endswith("_ws_floats") else
                          ctypes.c_void_p if name == "grag_err_alloc" else ctypes.c_int)
        mf = os.environ.get("GRAG_GEMM_MFMA")
        if mf and getattr(handle, "grag_gemm_tile_mfma", None) is not None:
            handle.grag_gemm_tile_mfma(int(mf))  # tile GEMM MFMA shape (16 default, 32)
        xc = os.environ.get("GRAG_DECODE_XCD")
        if xc and getattr(handle, "grag_attn_decode_xcd", None) is not None:
            handle.grag_attn_decode_xcd(int(xc))  # decode workgroups of adjacent rows on one XCD (1) or not (0)
        sc = os.environ.get("GRAG_GEMM_SCHED")
        if sc and getattr(handle, "grag_gemm_tile_sched", None) is not None:
            handle.grag_gemm_tile_sched(int(sc))  # tile GEMM phase schedule (0, 1 balanced reads)
        _lib = handle
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            bind_error_guard(torch.cuda.current_device())
        return _lib


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t):
    return None if t is None else t.data_ptr()


def check(err: int, name: str) -> None:
    if err != 0:
        raise RuntimeError(f"{name}: HIP kernel launch failed with hipError_t={err}")


def call(name: str, *args) -> None:
    """Call a kernel entry point; the trailing hipStream_t is appended here."""
    fn = getattr(lib(), name)
    check(fn(*args, stream_ptr()), name)


# ---------------------------------------------------------------- device index guard (csrc/kernels/common.h)
ERR_UNITS = ("norm", "elementwise", "attention", "gemm_tile", "gemm_stream")
ERR_CODES = {1 << 0: "embed_gather: token id >= vocab", 1 << 1: "qkv_rope_kvstore: KV slot id >= cache slots",
             1 << 2: "qkv_rope_kvstore: position >= RoPE table rows",
             1 << 3: "prefill attention: block-table entry >= KV blocks",
             1 << 4: "decode attention: block-table entry >= KV blocks",
             1 << 5: "split-merge / stream-K ticket past its part count (a stale or shared ticket word)",
             1 << 6: "sampler: slot row out of range", 1 << 7: "top-k / IVF: candidate row out of range",
             1 << 8: "encoder embedding: token / position id out of range",
             1 << 9: "shared-prefix decode: group row range or prefix length out of range"}
_ERR: dict = {"host": 0, "dev": None, "bound": set()}


class DeviceIndexError(RuntimeError):
    """A kernel found an index input out of range (and skipped the access instead of faulting)."""


def bind_error_guard(device: int) -> bool:
    """Point every kernel unit's error-block pointer (on ``device``) at the process's host-mapped block.
    Idempotent per device; False when the library or the device has none (CPU hosts)."""
    if device in _ERR["bound"] or _lib is None:
        return device in _ERR["bound"]
    alloc = getattr(_lib, "grag_err_alloc", None)
    if alloc is None:
        return False
    with _lock:
        if device in _ERR["bound"]:
            return True
        with torch.cuda.device(device):
            if _ERR["dev"] is None:
                alloc.restype = ctypes.c_void_p
                alloc.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
                d = ctypes.c_void_p()
                h = alloc(ctypes.byref(d))
                if not h:
                    return False
                _ERR["host"], _ERR["dev"] = h, d
            for unit in ERR_UNITS:
                fn = getattr(_lib, f"grag_err_bind_{unit}", None)
                if fn is not None:
                    fn.argtypes = [ctypes.c_void_p]
                    if fn(_ERR["dev"]) != 0:
                        return False
        _ERR["bound"].add(device)
    return True


def device_errors() -> tuple[int, int, int, int]:
    """(codes OR-ed, last bad value, report count, code of that value) recorded by the kernels so far."""
    if not _ERR["host"]:
        return 0, 0, 0, 0
    v = (ctypes.c_uint32 * 4).from_address(_ERR["host"])
    return int(v[0]), int(v[1]), int(v[2]), int(v[3])


def check_device_errors(where: str = "") -> None:
    """Raise DeviceIndexError (and clear the block) when a kernel reported an out-of-range index.  Cheap (a
    host memory read, no device sync): the engine calls it after every step's host read."""
    if not _ERR["host"]:
        return
    v = (ctypes.c_uint32 * 4).from_address(_ERR["host"])
    if v[0] == 0:
        return
    codes, value, count, last = int(v[0]), int(v[1]), int(v[2]), int(v[3])
    v[0] = v[1] = v[2] = v[3] = 0
    names = [n for c, n in ERR_CODES.items() if codes & c] or [f"code {codes:#x}"]
    raise DeviceIndexError(f"device index guard{' (' + where + ')' if where else ''}: {'; '.join(names)}; "
                           f"{count} report(s), last value {value} ({ERR_CODES.get(last, hex(last))})")


def loaded_path() -> str | None:
    return str(_LIB_PATH) if _lib is not None else None
