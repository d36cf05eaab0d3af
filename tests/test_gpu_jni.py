"""The JNI drop-in, end to end on the GPU.

tests/native/jni_driver.c calls the shim's TheGPU natives
(crossbow_amd/csrc/jni/TheGPU_jni.c) the way Crossbow's Java side does, with a
hand-made JNIEnv in place of a JVM (there is no JDK in this image), and checks
one SMA step, as written by checkpointModel in the reference's file format,
bit for bit against the oracle; then overrideModelData, acquireAccess /
upgradeAccess (boxed Integers), addModel / delModel and free.
scripts/build_jni_harness.sh builds the shim against tests/jni_stub/jni.h and
the driver (both on the CPU side, beforehand; __graft_entry__.build() does it).
"""
from __future__ import annotations

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "native", "jni_driver")

pytestmark = pytest.mark.gpu


def test_jni_natives_end_to_end():
    assert os.path.exists(EXE), "run scripts/build_jni_harness.sh (or __graft_entry__.build()) first"
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "jni_driver: ok" in r.stdout
