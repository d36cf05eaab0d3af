"""The C-ABI's host code under AddressSanitizer + UndefinedBehaviorSanitizer,
on the GPU (the reference runs no sanitizers).

tests/native/abi_driver.c drives every host-side path of libcrossbow_sma from
plain C; scripts/build_sanitized.sh links it with the library sources built
with -Xarch_host -fsanitize=address,undefined (device code uninstrumented).
The binary is built on the CPU side beforehand and travels with the tree;
without it the test is skipped.  Leak checking is off: the HIP runtime keeps
process-lifetime allocations."""
from __future__ import annotations

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "native", "abi_driver_asan")

pytestmark = pytest.mark.gpu


@pytest.mark.skipif(not os.path.exists(EXE), reason="run scripts/build_sanitized.sh first")
def test_abi_host_code_under_asan_ubsan():
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([EXE], capture_output=True, text=True, env=env, timeout=110)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "runtime error" not in out and "ERROR: AddressSanitizer" not in out, out[-4000:]
    assert "abi_driver: ok" in r.stdout
