"""The per-device enqueue thread pool (EnqueuePool, crossbow_amd/csrc/
context_internal.h) on the CPU under ThreadSanitizer: every device's job runs
exactly once per run and before run() returns, the device count changes
between runs, the first failure in device order is reported with its message,
and the pool survives a failure and its own destruction
(tests/native/enqueue_pool_test.cpp).  No GPU: the pool runs host functions
only; the library's multi-device GPU tests run it with real HIP calls."""
from __future__ import annotations

import os
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/llvm/bin/clang++"


@pytest.mark.skipif(not os.path.exists(CLANG) or shutil.which("ld") is None, reason="ROCm clang++ needed")
def test_enqueue_pool_under_thread_sanitizer():
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "enqueue_pool_test")
        subprocess.run([CLANG, "-std=c++17", "-O1", "-g", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                        "-fsanitize=thread", "-o", exe, os.path.join(ROOT, "tests", "native", "enqueue_pool_test.cpp"),
                        "-lpthread"], check=True, capture_output=True, timeout=240)
        env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:exitcode=66")
        p = subprocess.run([exe], capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0, (p.stdout + p.stderr)[-3000:]
    assert p.stdout.startswith("ok "), p.stdout
