"""C-ABI boundary checks that need no GPU.

* every function ``include/crossbow_sma.h`` declares is exported by
  ``libcrossbow_sma.so`` and bound by ``crossbow_amd._lib`` (and vice versa);
* the JNI shim defines every Java native of the model path that
  ``TheGPU.java:268-354`` declares (names as javah mangles them);
* on a host without an MI355X the product path fails loudly
  (``CBX_ERR_NO_DEVICE``) instead of falling back to the CPU.
"""
from __future__ import annotations

import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "crossbow_sma.h")
JNI_SRC = os.path.join(ROOT, "crossbow_amd", "csrc", "jni", "TheGPU_jni.c")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(cbx_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_barrier_path():
    names = declared_functions()
    for must in ("cbx_init", "cbx_init_rank", "cbx_set_model", "cbx_set_model_variable",
                 "cbx_set_model_manager", "cbx_lock_any", "cbx_merge", "cbx_synchronise",
                 "cbx_unlock_any", "cbx_checkpoint_model", "cbx_override_model_data", "cbx_free"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from crossbow_amd import _lib
    lib = _lib.load()
    raw = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(raw, n)]
    assert not missing, f"declared in crossbow_sma.h but not exported: {missing}"
    unbound = [n for n in declared_functions() if n not in _lib.SIGNATURES]
    assert not unbound, f"declared but not bound in _lib.SIGNATURES: {unbound}"
    extra = [n for n in _lib.SIGNATURES if n not in declared_functions()]
    assert not extra, f"bound in _lib but not declared in the header: {extra}"
    assert lib.cbx_abi_version() == 1


def test_no_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible; this checks the no-device behaviour")
    from crossbow_amd import CbxError, TheGPU, _lib
    assert TheGPU.device_count() == 0
    g = TheGPU()
    with pytest.raises(CbxError) as e:
        g.init([0])
    assert e.value.code == _lib.CBX_ERR_NO_DEVICE


def test_null_context_is_an_error_not_a_crash():
    from crossbow_amd import _lib
    lib = _lib.load()
    assert lib.cbx_set_model(None, 1, 16) == _lib.CBX_ERR_INVALID
    assert lib.cbx_lock_any(None) == _lib.CBX_ERR_INVALID
    assert lib.cbx_synchronise(None, 0, 1, 0, 0) == _lib.CBX_ERR_INVALID
    assert "null context" in _lib.last_error()
    assert lib.cbx_free(None) == _lib.CBX_OK


def test_model_sizes_must_fit_a_java_int():
    # TheGPU.setModel(II) / setModelVariable take Java ints (model.h:35 `int bytes`);
    # the wrapper refuses a size ctypes would silently wrap, before any library call.
    from crossbow_amd import CbxError, TheGPU
    g = TheGPU()
    with pytest.raises(CbxError, match="Java int"):
        g.setModel(1, 2**31)
    with pytest.raises(CbxError, match="Java int"):
        g.setModelVariable(0, 1, [2**29], 2**31)


# The model-path natives of TheGPU.java (:268-354) the shim must export.
JNI_NATIVES = [
    "init", "free", "setModel", "setModelVariable", "setModelVariableBuffer",
    "setModelVariableLearningRateMultiplier", "setModelWorkPerClock", "setLearningRateDecayPolicyCircular",
    "setUpdateModelType", "setLearningRateDecayPolicyFixed", "setLearningRateDecayPolicyInv",
    "setLearningRateDecayPolicyStep", "setLearningRateDecayPolicyMultiStep", "setLearningRateDecayPolicyExp",
    "setBaseModelMomentum", "setMomentum", "setWeightDecay", "setEamsgdAlpha", "setEamsgdTau",
    "setModelManager", "lockAny", "merge", "synchronise", "unlockAny", "checkpointModel",
    "overrideModelData", "addModel", "delModel", "acquireAccess", "upgradeAccess", "release",
]


def test_jni_shim_defines_model_path_natives():
    src = open(JNI_SRC).read()
    defined = set(re.findall(r"NATIVE\(\s*\w+\s*,\s*(\w+)\s*\)", src))
    missing = [n for n in JNI_NATIVES if n not in defined]
    assert not missing, f"JNI shim lacks {missing}"
    # Every native forwards to a declared C-ABI function.
    used = set(re.findall(r"\b(cbx_[a-z0-9_]+)\s*\(", src))
    assert used <= set(declared_functions()), used - set(declared_functions())


def test_jni_shim_compiles_against_the_c_abi():
    # No JDK in this image: compile-check the shim against a minimal jni.h
    # stand-in (tests/jni_stub/jni.h, JNI-spec signatures of the few JNIEnv
    # functions it calls) so a type mismatch with crossbow_sma.h is caught.
    import shutil
    import subprocess
    gcc = shutil.which("gcc")
    if gcc is None:
        pytest.skip("no gcc")
    r = subprocess.run([gcc, "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-std=c11",
                        "-I", os.path.join(ROOT, "tests", "jni_stub"), "-I", os.path.join(ROOT, "include"),
                        JNI_SRC], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


CPP_POLICY = r"""
#include <cstdio>
#include <stdexcept>
#include "ModelManager.hpp"
#define EXPECT(c) do { if (!(c)) { std::printf("failed: %s\n", #c); return 1; } } while (0)
int main() {
  crossbow::SystemConf c;
  c.wpc = 3; c.checkpointInterval = 7;             // ModelManager.java:73-80: 7 tasks -> 9 -> 3 clocks
  EXPECT(crossbow::ModelManager(nullptr, c).checkpointStep() == 3);
  c.autotuneModels = true; c.autotuneInterval = 2; c.autotuneThreshold = 0.1;
  crossbow::ModelManager m(nullptr, c);
  bool threw = false;                              // :243-244: no monitor
  try { m.autotune(); m.autotune(); } catch (const std::logic_error &) { threw = true; }
  EXPECT(threw);
  crossbow::ModelManager a(nullptr, c);
  const double tp[] = {10.0, 12.0, 12.5};
  int k = 0;
  a.setPerformanceMonitor([&] { return tp[k++]; });
  int got[8];
  for (int i = 0; i < 8; ++i) got[i] = a.autotune();  // :257-274
  const int want[8] = {0, 1, 0, 1, 0, -1, 0, 0};   // first reading, +20 %, +4.2 % (< 10 %)
  for (int i = 0; i < 8; ++i) EXPECT(got[i] == want[i]);
  EXPECT(k == 3 && !a.autotuning());
  crossbow::SystemConf off;                        // SystemConf.java:228: autotuning off
  EXPECT(crossbow::ModelManager(nullptr, off).autotune() == 0);
  std::printf("ok\n");
  return 0;
}
"""


def test_cpp_model_manager_policy(tmp_path):
    # crossbow_amd/host/ModelManager.hpp (the Java ModelManager restated in C++):
    # compiled against crossbow_sma.h and run here for its host-side policy
    # (checkpoint step, autotune decisions, null monitor); the GPU test
    # (tests/test_gpu_host.py) runs its barrier and checkpoint calls.
    import shutil
    import subprocess
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    src = tmp_path / "policy.cpp"
    src.write_text(CPP_POLICY)
    exe = tmp_path / "policy"
    lib_dir = os.path.join(ROOT, "crossbow_amd")
    r = subprocess.run([gxx, "-std=c++17", "-Wall", "-Wextra", "-Werror",
                        "-I", os.path.join(ROOT, "crossbow_amd", "host"), "-I", os.path.join(ROOT, "include"),
                        "-o", str(exe), str(src), "-L", lib_dir, "-lcrossbow_sma", f"-Wl,-rpath,{lib_dir}"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


def test_code_object_digest_ties_traffic_to_the_build():
    # bench.py reports profiles/traffic.json's PMC bytes only for the code
    # object they were measured on: the digest is the library's .hip_fatbin.
    import json

    from crossbow_amd import _lib
    from crossbow_amd.build import code_object_digest
    d = code_object_digest(_lib.LIB_PATH)
    assert re.fullmatch(r"[0-9a-f]{64}", d)
    assert code_object_digest(_lib.LIB_PATH) == d
    with open(os.path.join(ROOT, "profiles", "traffic.json")) as f:
        tj = json.load(f)
    for key, entry in tj.items():
        if key.startswith("sma_") and "code_object_sha256" in entry:
            assert re.fullmatch(r"[0-9a-f]{64}", entry["code_object_sha256"]), key


def test_seam_fails_loudly_without_device():
    # the sma.c seam (cbx_sma_plan_*) has no CPU fallback either
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible; this checks the no-device behaviour")
    from crossbow_amd import CbxError, _lib
    from crossbow_amd.seam import SmaPlan
    with pytest.raises(CbxError) as e:
        SmaPlan([0], 1024)
    assert e.value.code == _lib.CBX_ERR_NO_DEVICE
    lib = _lib.load()
    assert lib.cbx_sma_plan_step(None, None, None, None, 0, None, None, None, None, None, 0.1, 0.0, 0) \
        == _lib.CBX_ERR_INVALID
    assert lib.cbx_sma_plan_free(None) == _lib.CBX_OK
