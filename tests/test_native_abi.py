"""The ctypes signatures must match the C ABI of the kernel library (parsed
from the sources) — a mismatch would pass garbage pointers to a kernel."""
import re
from pathlib import Path

from githubrepostorag_amd.ops._lib import _SIGS as KSIGS
from githubrepostorag_amd.utils.runtime import _SIGS as RSIGS

ROOT = Path(__file__).resolve().parents[1]


def _c_decls(pattern_files, prefix):
    decls = {}
    for f in pattern_files:
        src = f.read_text()
        for m in re.finditer(prefix + r"\s+\w+\s*\*?\s*(grag_\w+)\s*\(([^)]*)\)\s*\{", src):
            params = [p for p in m.group(2).replace("\n", " ").split(",") if p.strip()]
            decls[m.group(1)] = len(params)
    return decls


def test_kernel_abi_counts():
    decls = _c_decls(sorted((ROOT / "csrc" / "kernels").glob("*.hip")), r"GRAG_API")
    assert decls, "no exported kernels found"
    for name, nargs in decls.items():
        assert name in KSIGS, f"{name} missing from ops/_lib.py _SIGS"
        assert len(KSIGS[name]) == nargs, f"{name}: ctypes {len(KSIGS[name])} vs C {nargs}"


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
