"""The C++ host side above the C-ABI, on the GPU (run with -m gpu).

crossbow_amd/host/ModelManager.hpp restates the GPU body of Crossbow's Java
ModelManager (trySynchronise, autotune, checkpoint; ModelManager.java:73-353)
for hosts without a JVM.  tests/native/modelmanager_driver.cpp drives the
library with it: registration, eight barriers with autotuning on a scripted
throughput monitor (+1, +1, -1 replica per GPU), checkpoints every two clocks,
the first step bit for bit against the oracle, and a library error surfacing
as CbxError.  Built by scripts/build_host_harness.sh (via
__graft_entry__.build()) on the CPU side beforehand.
"""
from __future__ import annotations

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "native", "modelmanager_driver")

pytestmark = pytest.mark.gpu


def test_cpp_model_manager_drives_the_library():
    assert os.path.exists(EXE), "run scripts/build_host_harness.sh (or __graft_entry__.build()) first"
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "modelmanager_driver: ok" in r.stdout
