"""Sanitizer builds of the C++ host runtime (SURVEY §5.2 race detection /
sanitizers): the tokenizers and the paged-KV block allocator, driven by
csrc/runtime/tests/runtime_selftest.cpp, compiled and run under
AddressSanitizer + UndefinedBehaviorSanitizer and under ThreadSanitizer
(8 threads sharing one allocator and one BPE).  Host code only — GPU
sanitizers are not available on the MI355X pool."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
SRC = sorted((ROOT / "csrc" / "runtime").glob("*.cpp")) + [ROOT / "csrc" / "runtime" / "tests" / "runtime_selftest.cpp"]


def _build_and_run(tmp_path, flags, name):
    cxx = shutil.which(os.environ.get("CXX", "g++"))
    if cxx is None:
        pytest.skip("no C++ compiler")
    exe = tmp_path / name
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *flags, "-I", str(ROOT / "csrc" / "runtime"),
           *map(str, SRC), "-o", str(exe), "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
    env.pop("LD_PRELOAD", None)
    run = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=env)
    out = run.stdout + run.stderr
    return run.returncode, out


def test_runtime_asan_ubsan(tmp_path):
    rc, out = _build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
                             "selftest_asan")
    assert rc == 0 and "runtime selftest ok" in out, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out


def test_runtime_tsan(tmp_path):
    rc, out = _build_and_run(tmp_path, ["-fsanitize=thread"], "selftest_tsan")
    if rc != 0 and "unexpected memory mapping" in out:  # TSan vs. high-entropy ASLR on some kernels
        pytest.skip("ThreadSanitizer cannot map its shadow on this kernel")
    assert rc == 0 and "runtime selftest ok" in out, out[-4000:]
    assert "WARNING: ThreadSanitizer" not in out
