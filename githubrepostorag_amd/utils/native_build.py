"""Build the native libraries in-tree.

* ``libgrag_kernels.so`` — every HIP kernel under ``csrc/kernels`` compiled by
  ``hipcc --offload-arch=gfx950`` (CDNA4 only, no hipify, no CUDA shims).  The
  library exposes a plain C ABI (raw device pointers + hipStream_t) and is
  loaded with ctypes *after* ``import torch`` so it binds to the same
  ``libamdhip64.so.7`` (same SONAME) that PyTorch-ROCm already loaded — one HIP
  runtime per process, PyTorch's streams are valid handles for our launches and
  our launches are captured by ``torch.cuda.CUDAGraph`` (hipGraph).
* ``libgrag_runtime.so`` — host C++ runtime (paged-KV block allocator with
  prefix-hash cache, byte-level BPE + WordPiece tokenizers, top-k merge, code
  splitter scan) compiled with g++.

Both land in ``githubrepostorag_amd/_lib`` so they travel with the repo
snapshot to the GPU box.
"""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
CSRC = ROOT / "csrc"
LIBDIR = ROOT / "githubrepostorag_amd" / "_lib"
OBJDIR = ROOT / "build" / "obj"
ARCH = os.environ.get("GRAG_OFFLOAD_ARCH", "gfx950")
KERNEL_LIB = LIBDIR / "libgrag_kernels.so"
RUNTIME_LIB = LIBDIR / "libgrag_runtime.so"

HIPCC_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-ffp-contract=fast",
    "-munsafe-fp-atomics",
    "-Wno-unused-result",
]
CXX_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function"]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found; the gfx950 kernel library cannot be built")


def _digest(paths) -> str:
    h = hashlib.sha1()
    for p in sorted(paths):
        h.update(p.name.encode())
        h.update(p.read_bytes())
    return h.hexdigest()


def _run(cmd):
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"command failed: {' '.join(map(str, cmd))}\n{res.stdout}\n{res.stderr}")
    return res


def build_kernels(force: bool = False, jobs: int = 8, verbose: bool = False) -> Path:
    srcs = sorted((CSRC / "kernels").glob("*.hip"))
    hdrs = sorted((CSRC / "kernels").glob("*.h"))
    stamp = LIBDIR / "libgrag_kernels.sha1"
    digest = _digest(srcs + hdrs) + ARCH
    if not force and KERNEL_LIB.exists() and stamp.exists() and stamp.read_text() == digest:
        return KERNEL_LIB
    LIBDIR.mkdir(parents=True, exist_ok=True)
    OBJDIR.mkdir(parents=True, exist_ok=True)
    hipcc = _hipcc()
    hdr_digest = _digest(hdrs) if hdrs else ""

    def compile_one(src: Path) -> Path:
        obj = OBJDIR / (src.stem + ".o")
        osig = OBJDIR / (src.stem + ".sig")
        sig = _digest([src]) + hdr_digest + ARCH
        if not force and obj.exists() and osig.exists() and osig.read_text() == sig:
            return obj
        cmd = [hipcc, *HIPCC_FLAGS, "-I", str(CSRC / "kernels"), "-c", str(src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        _run(cmd)
        osig.write_text(sig)
        return obj

    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(compile_one, srcs))
    tmp = KERNEL_LIB.with_suffix(".so.tmp")
    _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs)])
    os.replace(tmp, KERNEL_LIB)
    stamp.write_text(digest)
    return KERNEL_LIB


def build_runtime(force: bool = False, sanitize: bool = False) -> Path:
    srcs = sorted((CSRC / "runtime").glob("*.cpp"))
    hdrs = sorted((CSRC / "runtime").glob("*.h"))
    out = RUNTIME_LIB if not sanitize else LIBDIR / "libgrag_runtime_asan.so"
    stamp = out.with_suffix(".sha1")
    digest = _digest(srcs + hdrs) + ("asan" if sanitize else "")
    if not force and out.exists() and stamp.exists() and stamp.read_text() == digest:
        return out
    LIBDIR.mkdir(parents=True, exist_ok=True)
    cxx = os.environ.get("CXX", "g++")
    flags = list(CXX_FLAGS)
    if sanitize:
        flags = ["-O1", "-g", "-std=c++17", "-fPIC", "-fsanitize=address,undefined", "-fno-omit-frame-pointer"]
    tmp = out.with_suffix(".so.tmp")
    _run([cxx, *flags, "-shared", "-I", str(CSRC / "runtime"), "-o", str(tmp), *map(str, srcs), "-lpthread"])
    os.replace(tmp, out)
    stamp.write_text(digest)
    return out


def build_all(force: bool = False, verbose: bool = False) -> None:
    build_runtime(force=force)
    build_kernels(force=force, verbose=verbose)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv, verbose="-v" in sys.argv)
    print(KERNEL_LIB, RUNTIME_LIB)
