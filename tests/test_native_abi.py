"""The ctypes signatures must match the C ABI of the kernel library (parsed
from the sources) — a mismatch would pass garbage pointers to a kernel."""
import ctypes
import re
from pathlib import Path

from githubrepostorag_amd.ops._lib import _SIGS as KSIGS
from githubrepostorag_amd.parallel.custom_ar import _SIGS as _AR_SIGS
from githubrepostorag_amd.utils.runtime import _SIGS as RSIGS

# the one-shot all-reduce binds its entry points itself (argtypes, restype)
KSIGS = {**KSIGS, **{k: v[0] for k, v in _AR_SIGS.items()}}

ROOT = Path(__file__).resolve().parents[1]


def _c_decls(pattern_files, prefix):
    decls = {}
    for f in pattern_files:
        src = f.read_text()
        for m in re.finditer(prefix + r"\s+\w+\s*\*?\s*(grag_\w+)\s*\(([^)]*)\)\s*\{", src):
            params = [p.strip() for p in m.group(2).replace("\n", " ").split(",") if p.strip()]
            decls[m.group(1)] = params
    return decls


def _ctype_of(param: str):
    """ctypes type a C parameter declaration must be bound with."""
    t = param.rsplit(" ", 1)[0] if " " in param else param
    if "*" in param or "hipStream_t" in t:
        return ctypes.c_void_p
    if "uint64_t" in t:
        return ctypes.c_uint64
    if "int64_t" in t or re.search(r"\blong\b", t):
        return ctypes.c_int64
    if "float" in t:
        return ctypes.c_float
    return ctypes.c_int


def test_kernel_abi_counts_and_types():
    """Width/kind of every argument, not just the count: a 64-bit handle bound
    as c_int is silently truncated (a hipStream_t that only breaks inside a
    hipGraph capture, where the handle is a real pointer)."""
    decls = _c_decls(sorted((ROOT / "csrc" / "kernels").glob("*.hip")), r"GRAG_API")
    assert decls, "no exported kernels found"
    for name, params in decls.items():
        assert name in KSIGS, f"{name} missing from ops/_lib.py _SIGS"
        assert len(KSIGS[name]) == len(params), f"{name}: ctypes {len(KSIGS[name])} vs C {len(params)}"
        for i, (ct, cp) in enumerate(zip(KSIGS[name], params)):
            want = _ctype_of(cp)
            same = ct is want or (want is ctypes.c_int64 and ct is ctypes.c_long) or (
                want is ctypes.c_uint64 and ct is ctypes.c_ulong)
            assert same, f"{name} arg {i} ({cp!r}): ctypes {ct} vs C {want}"


def test_runtime_abi_counts():
    srcs = sorted((ROOT / "csrc" / "runtime").glob("*.cpp"))
    decls = {}
    for f in srcs:
        src = f.read_text()
        for m in re.finditer(r"\n(?:void\*|void|int|int64_t|uint64_t)\s+(grag_\w+)\s*\(([^)]*)\)\s*\{", src):
            params = [p for p in m.group(2).replace("\n", " ").split(",") if p.strip()]
            decls[m.group(1)] = len(params)
    assert decls
    for name, nargs in decls.items():
        assert name in RSIGS, name
        assert len(RSIGS[name][0]) == nargs, f"{name}: ctypes {len(RSIGS[name][0])} vs C {nargs}"
