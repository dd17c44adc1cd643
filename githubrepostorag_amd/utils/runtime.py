"""ctypes binding of the host C++ runtime (``libgrag_runtime.so``)."""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path

_PATH = Path(__file__).resolve().parents[1] / "_lib" / "libgrag_runtime.so"
_lock = threading.Lock()
_rt = None

P = ctypes.c_void_p
I = ctypes.c_int
I64 = ctypes.c_int64
U64 = ctypes.c_uint64
CP = ctypes.c_char_p

_SIGS = {
    "grag_alloc_create": ([I, I], P),
    "grag_alloc_destroy": ([P], None),
    "grag_alloc_num_free": ([P], I),
    "grag_alloc_allocate": ([P, I, P], I),
    "grag_alloc_free": ([P, I, P], None),
    "grag_hash_block": ([U64, P, I], U64),
    "grag_hash_blocks": ([U64, P, I, I, P], None),
    "grag_alloc_register_many": ([P, P, P, I], None),
    "grag_alloc_unregister": ([P, I, P], None),
    "grag_alloc_match_prefix": ([P, P, I, P, P], I),
    "grag_alloc_register": ([P, I, U64], None),
    "grag_alloc_stats": ([P, P], None),
    "grag_alloc_refcount": ([P, I], I),
    "grag_bpe_create": ([], P),
    "grag_bpe_destroy": ([P], None),
    "grag_bpe_train": ([P, CP, I64, I], I),
    "grag_bpe_set_merges": ([P, P, I], None),
    "grag_bpe_get_merges": ([P, P, I], I),
    "grag_bpe_add_special": ([P, CP, I], None),
    "grag_bpe_vocab_size": ([P], I),
    "grag_bpe_encode": ([P, CP, I64, P, I64], I64),
    "grag_bpe_decode": ([P, P, I64, P, I64], I64),
    "grag_wp_create": ([I, I, I], P),
    "grag_wp_destroy": ([P], None),
    "grag_wp_load_vocab": ([P, CP, I64], None),
    "grag_wp_encode": ([P, CP, I64, P, I64], I64),
}


def rt():
    global _rt
    if _rt is not None:
        return _rt
    with _lock:
        if _rt is None:
            path = _PATH
            if os.environ.get("GRAG_RUNTIME_ASAN") == "1":
                path = _PATH.with_name("libgrag_runtime_asan.so")
            if not path.exists():
                from .native_build import build_runtime

                build_runtime(sanitize=path != _PATH)
            h = ctypes.CDLL(str(path))
            for name, (args, res) in _SIGS.items():
                fn = getattr(h, name)
                fn.argtypes = args
                fn.restype = res
            _rt = h
    return _rt


def runtime_path() -> Path:
    return _PATH
