"""The JNI drop-in, end to end on the GPU.

tests/native/jni_driver.c calls the shim's TheGPU natives
(crossbow_amd/csrc/jni/TheGPU_jni.c) the way Crossbow's Java side does, with a
hand-made JNIEnv in place of a JVM (there is no JDK in this image), and checks
one SMA step, as written by checkpointModel in the reference's file format,
bit for bit against the oracle; then overrideModelData, acquireAccess /
upgradeAccess (boxed Integers), addModel / delModel and free.
scripts/build_jni_harness.sh builds the shim against tests/jni_stub/jni.h and
the driver (both on the CPU side, beforehand; __graft_entry__.build() does it).

With G > 1 the same natives drive G devices from one process, the reference's
own multi-GPU form (init with G devices -> ncclCommInitAll, grouped
all-reduces; executioncontext.c:185-201).  The box has one GPU, so init gets
G copies of device 0 and the shim is linked against the library build over
the loopback collective (tests/native/fake_rccl.cpp, scripts/build_fake_rccl.sh);
the checkpoint then holds every device's files, each bit for bit equal to the
oracle run with the same G.
"""
from __future__ import annotations

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "native", "jni_driver")
# the same driver over the library build linked against the loopback collective
EXE_LOOPBACK = os.path.join(ROOT, "tests", "native", "jni_driver_fakerccl")

pytestmark = pytest.mark.gpu


def test_jni_natives_end_to_end():
    assert os.path.exists(EXE), "run scripts/build_jni_harness.sh (or __graft_entry__.build()) first"
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "jni_driver: ok" in r.stdout


@pytest.mark.parametrize("G,env", [(2, {}), (4, {}), (8, {}),
                                   # the pipeline settings a deployment picks through the environment
                                   (4, {"CBX_ALLREDUCE": "rsag", "CBX_BUCKET_ELEMENTS": "4096",
                                        "CBX_PIPELINE_MODE": "1", "CBX_CROSS_WAIT_STRIDE": "2"}),
                                   (4, {"CBX_ALLREDUCE": "peer"}),
                                   (2, {"CBX_BUCKET_ELEMENTS": "8192", "CBX_ALLREDUCE_GROUP": "2",
                                        "CBX_STAGING": "dma"})])
def test_jni_natives_single_process_multi_device(G, env):
    assert os.path.exists(EXE_LOOPBACK), "run scripts/build_fake_rccl.sh (or __graft_entry__.build()) first"
    r = subprocess.run([EXE_LOOPBACK, str(G)], capture_output=True, text=True, timeout=110,
                       env=dict(os.environ, **env))
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert f"jni_driver: ok (G={G})" in r.stdout


def test_jni_environment_settings_are_checked():
    # a refused setting is fatal at init, as every error of the shim is
    assert os.path.exists(EXE_LOOPBACK)
    for env in ({"CBX_ALLREDUCE": "ring"}, {"CBX_PIPELINE_MODE": "7"}, {"CBX_BUCKET_ELEMENTS": "12x"},
                {"CBX_PIPELINE_MODE": "4294967297"}, {"CBX_ALLREDUCE_GROUP": "0"}):
        r = subprocess.run([EXE_LOOPBACK, "2"], capture_output=True, text=True, timeout=110,
                           env=dict(os.environ, **env))
        assert r.returncode != 0 and "error:" in r.stderr, (env, r.stderr[-2000:])
