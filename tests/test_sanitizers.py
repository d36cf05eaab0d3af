"""Host-code sanitizers (the reference has none).

The CPU oracle is built into a standalone driver with AddressSanitizer and
UndefinedBehaviorSanitizer (no LD_PRELOAD: the sanitizer runtimes are linked
into the executable) and run over every entry point: ragged sizes, G x R
mixes, partial locks, `first`, copy flags, optimiser / DEFAULT / S-SGD task
steps, BN averaging, and the OpenBLAS replays, which must still agree bit for
bit with the fmaf restatement.  GPU code is not sanitized (no GPU ASan on
this pool)."""
from __future__ import annotations

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_oracle_under_asan_ubsan(tmp_path):
    exe = tmp_path / "sanitize_oracle"
    cmd = ["gcc", "-O1", "-g", "-std=c11", "-Wall", "-ffp-contract=off", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-o", str(exe), os.path.join(ROOT, "tests", "sanitize_oracle.c"),
           os.path.join(ROOT, "oracle", "sma_oracle.c"), "-lm", "-ldl"]
    subprocess.run(cmd, check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    from oracle import oracle as O
    blas = O.openblas_path()
    r = subprocess.run([str(exe)] + ([blas] if blas else []), capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr
    assert "sanitize_oracle: ok" in r.stdout
    if blas:
        assert "no BLAS" not in r.stdout, "the OpenBLAS replays must run under the sanitizers too"
